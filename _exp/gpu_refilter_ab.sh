#!/bin/bash
# refilter with per-lane f64 fetches: dense parity tests, then the C2 step A/B (refilter 0 / 1)
set -o pipefail
O=gpurun_out/${1:?tag}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py -k "refilter or dense or heavy_first" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u _exp/c2_ab.py 20 4 SWEEP_REFILTER=0,1 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v '^{' $O/ab.txt
