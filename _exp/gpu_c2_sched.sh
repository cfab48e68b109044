set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05sch}
mkdir -p $O
timeout -k 10 300 python -u _exp/c2_ab.py 20 3 DENSE_SPEC=2,3 > $O/spec.txt 2>&1 || { echo "spec failed"; tail -20 $O/spec.txt; exit 1; }
grep -v "^{" $O/spec.txt
timeout -k 10 300 python -u _exp/c2_ab.py 20 3 SWEEP_PARTS=2,3 > $O/parts.txt 2>&1 || { echo "parts failed"; tail -20 $O/parts.txt; exit 1; }
grep -v "^{" $O/parts.txt
