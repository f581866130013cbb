set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 tools/host_prof.py 10 res101 daf 45 > $O/daf_r101.txt 2>&1
timeout -k 10 300 python3 tools/host_prof.py 4 res101 atf 45 > $O/atf_r101.txt 2>&1
timeout -k 10 300 python3 tools/host_prof.py 10 vgg16 daf 45 > $O/daf_vgg.txt 2>&1
