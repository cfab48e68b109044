# incremental lean rounds on C5: A/B over the in-degree threshold
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05x3}
mkdir -p $O
timeout -k 10 900 python -u _exp/c2_ab.py --config C5 2 1 CSR_INCREMENTAL=${2:-0,8,32} > $O/c5_ab.txt 2>&1 || { echo "c5 ab failed"; tail -20 $O/c5_ab.txt; exit 1; }
grep -v "^{" $O/c5_ab.txt
