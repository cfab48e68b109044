# generic A/B on the GPU box: _exp/gpu_ab.sh TAG CONFIG STEPS REPS OPT=a,b ...
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}
shift
mkdir -p $O
CFG=$1; shift
timeout -k 10 900 python -u _exp/c2_ab.py --config $CFG "$@" > $O/ab.txt 2> $O/ab.err || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
grep -v "^{" $O/ab.txt
