set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05sp}
mkdir -p $O
timeout -k 10 300 python -u _exp/c2_ab.py 20 3 SPIN_US=200,1000000 > $O/c2.txt 2>&1 || { echo "c2 failed"; tail $O/c2.txt; exit 1; }
grep -v "^{" $O/c2.txt
timeout -k 10 300 python -u _exp/c2_ab.py --config C4 5 2 SPIN_US=200,1000000 > $O/c4.txt 2>&1 || { echo "c4 failed"; tail $O/c4.txt; exit 1; }
grep -v "^{" $O/c4.txt
timeout -k 10 600 python -u _exp/c2_ab.py --config C5 2 1 SPIN_US=200,1000000 > $O/c5.txt 2>&1 || { echo "c5 failed"; tail $O/c5.txt; exit 1; }
grep -v "^{" $O/c5.txt
