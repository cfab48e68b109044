#!/bin/bash
# Uneven two-part split of the sweep (experiments build, SHADOWTOPO_PART0_PERMILLE): parity
# of the dense and chained tests with 9/7 batches, then C2 interleaved over part-0 shares.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}
mkdir -p $O
L=$PWD/_exp/ab/libshadowtopo_p0.so
SHADOWTOPO_EXP_LIB=$L SHADOWTOPO_PART0_PERMILLE=600 timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_fullsize_gpu.py -q -m gpu -k "dense or c2 or chained" --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/tests.log | head; exit 1; }
for rep in 1 2; do
  for pm in 500 438 562 625; do
    SHADOWTOPO_EXP_LIB=$L SHADOWTOPO_PART0_PERMILLE=$pm timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-north-star --no-shim --no-host-rate > $O/c2_${pm}_$rep.json 2> $O/c2_${pm}_$rep.err || { tail $O/c2_${pm}_$rep.err; exit 1; }
    echo -n "part0 $pm rep $rep: "; python3 -c "import json; d=json.load(open('$O/c2_${pm}_$rep.json')); print(round(d['ms_per_step'],4), 'sweep', round(d['roofline']['avg_launch_ms'],4))"
  done
done
