#!/bin/bash
# tests -> smoke -> bench (cpu baseline) -> rocprof kernel-trace; extra bench configs after
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
shift
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/gputests_$TAG.log 2>&1
rc=$?; tail -5 gpurun_out/gputests_$TAG.log
[ $rc -ne 0 ] && { echo "gpu tests failed rc=$rc"; grep -E "FAILED|Error|assert" gpurun_out/gputests_$TAG.log | head -20; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/bench_prof_$TAG.err || { echo "rocprof failed"; tail -20 gpurun_out/bench_prof_$TAG.err; exit 1; }
head -4 gpurun_out/prof_$TAG/run_kernel_stats.csv | cut -c1-220
for cfg in "$@"; do
  timeout -k 10 400 python -u bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${TAG}_$cfg.json 2> gpurun_out/bench_${TAG}_$cfg.err || { echo "bench $cfg failed"; tail -20 gpurun_out/bench_${TAG}_$cfg.err; exit 1; }
  cat gpurun_out/bench_${TAG}_$cfg.json
done
