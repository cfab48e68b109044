#!/bin/bash
# pruned delta rounds with fp16 slabs: dense parity (incl. the whole C2
# matrix), then the C2 step A/B (DELTA_W16 0 / 1)
set -o pipefail
O=gpurun_out/${1:?tag}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_engine_gpu.py tests/test_fullsize_gpu.py -k "dense or heavy_first or refilter or C2 or c2" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u _exp/c2_ab.py 20 4 DELTA_W16=0,1 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v '^{' $O/ab.txt
