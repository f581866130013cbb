# upper bound of removing the split-K reduce launches (timing only, wrong results):
# nored1 = no weight-gradient reduces, nored2 = no reduce launches at all
set -e
O=$1; mkdir -p $O
for r in 1 2; do
  for v in base nored1 nored2; do
    L=""; [ $v != base ] && L=build_variants/$v/libtlod.so
    TLOD_LIB=$L timeout -k 10 300 python3 bench.py --cpu-baseline-steps 0 > $O/vgg.$v.$r.json 2>/dev/null
    TLOD_LIB=$L timeout -k 10 300 python3 bench.py --method daf --net res101 --cpu-baseline-steps 0 > $O/r101.$v.$r.json 2>/dev/null
    echo "$v r$r vgg $(python3 -c "import json;print(json.load(open('$O/vgg.$v.$r.json'))['value'])") r101 $(python3 -c "import json;print(json.load(open('$O/r101.$v.$r.json'))['value'])")"
  done
done
