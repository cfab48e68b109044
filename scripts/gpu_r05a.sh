#!/bin/bash
# r05: the new walk / self-rule / pool tests first, then the whole GPU suite, smoke and the
# default bench line.  Every GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05a}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -m gpu \
  -k "scrambled or unconverged or long_paths or pool_enomem or alternating or vertex_loss or multigraph or self" > $O/new_tests.log 2>&1
rc=$?; tail -3 $O/new_tests.log; [ $rc -ne 0 ] && { echo "new tests failed rc=$rc"; grep -E "FAILED|Error" $O/new_tests.log | head -20; exit 1; }
timeout -k 10 1000 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && { echo "gpu tests failed rc=$rc"; grep -E "FAILED|Error" $O/gpu_tests.log | head -20; exit 1; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python -u bench.py --steps 10 --warmup 2 > $O/bench_default.json 2> $O/bench_default.err || { echo "default bench failed"; tail -20 $O/bench_default.err; exit 1; }
python3 scripts/bench_summary.py $O/bench_default.json
