set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 tools/torch_prof.py daf res101 3 > $O/daf_r101.txt 2>&1
timeout -k 10 300 python3 tools/torch_prof.py atf res101 2 > $O/atf_r101.txt 2>&1
timeout -k 10 300 python3 tools/torch_prof.py daf vgg16 3 > $O/daf_vgg.txt 2>&1
