# per-round item counts and times of the sparse rounds (SHADOWTOPO_TRACE_ROUNDS=1)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05z}
mkdir -p $O
SHADOWTOPO_TRACE_ROUNDS=1 timeout -k 10 300 python -u _exp/c2_ab.py --config C4 1 1 CSR_INCREMENTAL=0,32 > $O/c4.txt 2> $O/c4.err || { echo "c4 failed"; tail -20 $O/c4.err; exit 1; }
SHADOWTOPO_TRACE_ROUNDS=1 timeout -k 10 600 python -u _exp/c2_ab.py --config C5 1 1 CSR_INCREMENTAL=0,32 > $O/c5.txt 2> $O/c5.err || { echo "c5 failed"; tail -20 $O/c5.err; exit 1; }
grep -v "^{" $O/c4.txt $O/c5.txt
