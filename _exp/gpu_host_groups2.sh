set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05hg2}
mkdir -p $O
timeout -k 10 400 python3 -u _exp/host_groups_ab.py C4 3 4,6,8 > $O/c4.txt 2>&1 || { echo "c4 failed"; tail $O/c4.txt; exit 1; }
cat $O/c4.txt
