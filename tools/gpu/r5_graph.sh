set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 tools/graph_probe.py res101 daf 10 > $O/daf_r101.txt 2>&1; tail -1 $O/daf_r101.txt
timeout -k 10 300 python3 tools/graph_probe.py vgg16 daf 10 > $O/daf_vgg.txt 2>&1; tail -1 $O/daf_vgg.txt
timeout -k 10 300 python3 tools/graph_probe.py res101 atf 5 > $O/atf_r101.txt 2>&1; tail -1 $O/atf_r101.txt
