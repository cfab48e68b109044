#!/bin/bash
# End-of-round check on the current tree: GPU suite, smoke, default bench (-> gpurun_out/*_r02k*)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/gputests_r02k.log 2>&1
rc=$?; tail -2 gpurun_out/gputests_r02k.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/gputests_r02k.log | head -20; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r02k.log 2>&1 || { tail -20 gpurun_out/smoke_r02k.log; exit 1; }
tail -1 gpurun_out/smoke_r02k.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r02k.json 2> gpurun_out/bench_r02k.err || { tail -20 gpurun_out/bench_r02k.err; exit 1; }
cut -c1-300 gpurun_out/bench_r02k.json
