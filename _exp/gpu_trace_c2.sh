# per-round change counts of the C2 step (SHADOWTOPO_TRACE_ROUNDS=1), chained and host-driven
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05tc}
mkdir -p $O
SHADOWTOPO_TRACE_ROUNDS=1 timeout -k 10 300 python -u _exp/c2_ab.py 2 1 CHAIN_PARTS=1,0 DENSE_SPEC=2,0 > $O/c2.txt 2> $O/c2.err || { echo "c2 failed"; tail -20 $O/c2.err; exit 1; }
grep -v "^{" $O/c2.txt; grep round $O/c2.err | tail -24
