#!/bin/bash
# The split sweep per half of the batches on two streams (experiments build, SHADOWTOPO_SWEEP_HALVES=1):
# the larger random parity cases, the dense parity tests with the variant, then C2 interleaved.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fuzz_gpu.py -q -m gpu -k larger --timeout 200 --timeout-method thread > $O/fuzz.log 2>&1
rc=$?; tail -1 $O/fuzz.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/fuzz.log | head; exit 1; }
SHADOWTOPO_EXP_LIB=$PWD/_exp/ab/libshadowtopo_halves.so SHADOWTOPO_SWEEP_HALVES=1 timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_fullsize_gpu.py -q -m gpu -k "dense or c2" --timeout 200 --timeout-method thread > $O/halves_tests.log 2>&1
rc=$?; tail -1 $O/halves_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/halves_tests.log | head; exit 1; }
for rep in 1 2; do
  for v in cur halves; do
    if [ $v = cur ]; then unset SHADOWTOPO_EXP_LIB SHADOWTOPO_SWEEP_HALVES; else export SHADOWTOPO_EXP_LIB=$PWD/_exp/ab/libshadowtopo_halves.so SHADOWTOPO_SWEEP_HALVES=1; fi
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-north-star --no-shim --no-host-rate > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || { tail $O/c2_${v}_$rep.err; exit 1; }
    echo -n "$v $rep: "; python3 -c "import json; d=json.load(open('$O/c2_${v}_$rep.json')); print(round(d['ms_per_step'],4), 'sweep', round(d['roofline']['avg_launch_ms'],4))"
  done
done
