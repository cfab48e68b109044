#!/bin/bash
# Round check on one GPU box: the GPU suite, smoke, the default bench line (C2 + the C4
# north-star record), then optional extra bench configs.  Logs under gpurun_out/$TAG.
#   scripts/gpu_check.sh TAG [C3 C4 C5 ...]
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:?tag}
shift
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && { echo "gpu tests failed rc=$rc"; grep -E "FAILED|Error" $O/gpu_tests.log | head; exit 1; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || { echo "default bench failed"; tail -20 $O/bench_default.err; exit 1; }
python3 scripts/bench_summary.py $O/bench_default.json
for cfg in "$@"; do
  timeout -k 10 400 python -u bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$cfg.json 2> $O/bench_$cfg.err || { echo "bench $cfg failed"; tail -20 $O/bench_$cfg.err; exit 1; }
  python3 scripts/bench_summary.py $O/bench_$cfg.json
done
