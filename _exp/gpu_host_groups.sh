set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05hg}
mkdir -p $O
timeout -k 10 400 python3 -u _exp/host_groups_ab.py C4 3 0,2,3,4 > $O/c4.txt 2>&1 || { echo "c4 failed"; tail $O/c4.txt; exit 1; }
cat $O/c4.txt
timeout -k 10 300 python3 -u _exp/host_groups_ab.py C3 5 0,1,2,4,8 > $O/c3.txt 2>&1 || { echo "c3 failed"; tail $O/c3.txt; exit 1; }
cat $O/c3.txt
timeout -k 10 300 python3 -u _exp/host_groups_ab.py C2 5 0,2 > $O/c2.txt 2>&1 || { echo "c2 failed"; tail $O/c2.txt; exit 1; }
cat $O/c2.txt
