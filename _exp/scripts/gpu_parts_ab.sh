#!/bin/bash
# Pruned dense sweep in parts on their own streams (OPT_SWEEP_PARTS 1 / 2 / 4): dense and C2
# parity tests, then C2 interleaved on one box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py tests/test_fullsize_gpu.py tests/test_fuzz_gpu.py -q -m gpu -k "dense or c2 or random" --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/tests.log | head; exit 1; }
for rep in 1 2; do
  for p in 1 2 4; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-north-star --no-shim --no-host-rate --sweep-parts $p > $O/c2_p${p}_$rep.json 2> $O/c2_p${p}_$rep.err || { tail $O/c2_p${p}_$rep.err; exit 1; }
    echo -n "parts $p rep $rep: "; python3 -c "import json; d=json.load(open('$O/c2_p${p}_$rep.json')); print(round(d['ms_per_step'],4), 'sweep', round(d['roofline']['avg_launch_ms'],4))"
  done
done
