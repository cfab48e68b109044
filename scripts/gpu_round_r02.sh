#!/bin/bash
# Round measurement session: GPU suite, smoke, default bench (C2, CPU baseline, host rate),
# rocprof kernel-trace stats of it, then per-config counter passes + bench lines
# (scripts/gpu_roofline.sh) for C2, C4 and C5, and the C3 bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r02f}
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/gputests_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/gputests_$TAG.log
[ $rc -ne 0 ] && { echo "gpu tests failed rc=$rc"; grep -E "FAILED|Error|assert" gpurun_out/gputests_$TAG.log | head -20; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/bench_prof_$TAG.err || { echo "rocprof failed"; tail -20 gpurun_out/bench_prof_$TAG.err; exit 1; }
bash scripts/gpu_roofline.sh ${TAG}_C2 C2 1.0 "k_relax_dense_f<8, 2, 1, true>" || exit 1
bash scripts/gpu_roofline.sh ${TAG}_C4 C4 1.0 "k_relax\(|k_relax_wl\(" || exit 1
bash scripts/gpu_roofline.sh ${TAG}_C5 C5 1.0 "k_relax\(|k_relax_wl\(" || exit 1
for c in C3; do
  timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err || { echo "bench $c failed"; tail -5 gpurun_out/bench_${TAG}_$c.err; exit 1; }
  cat gpurun_out/bench_${TAG}_$c.json
done
