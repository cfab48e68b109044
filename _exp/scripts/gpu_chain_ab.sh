#!/bin/bash
# Read-back-free delta rounds on each sweep part's stream (OPT_CHAIN_PARTS 0 / 1): the dense,
# C2 and random parity tests, then C2 interleaved on one box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_fullsize_gpu.py tests/test_fuzz_gpu.py -q -m gpu -k "dense or c2 or random or chained" --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/tests.log | head; exit 1; }
for rep in 1 2 3; do
  for c in 0 1; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-north-star --no-shim --no-host-rate --chain-parts $c > $O/c2_c${c}_$rep.json 2> $O/c2_c${c}_$rep.err || { tail $O/c2_c${c}_$rep.err; exit 1; }
    echo -n "chain $c rep $rep: "; python3 -c "import json; d=json.load(open('$O/c2_c${c}_$rep.json')); r=d['roofline']; print(round(d['ms_per_step'],4), 'sweep', round(r['avg_launch_ms'],4), 'delta', r.get('delta_kernel'))"
  done
done
