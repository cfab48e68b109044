#!/bin/bash
# Round 1's chunk bounds from the sweep epilogues (OPT fuse_mindc; experiments knob
# SHADOWTOPO_FUSE_MINDC 0/1): the dense, C2, chained and random parity tests with the product
# build (fused, the default), then C2 interleaved with the experiments build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_engine_gpu.py tests/test_fullsize_gpu.py tests/test_fuzz_gpu.py -q -m gpu -k "dense or c2 or random or chained" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/tests.log | head; exit 1; }
L=$PWD/_exp/ab/libshadowtopo_fuse.so
for rep in 1 2 3; do
  for f in 0 1; do
    SHADOWTOPO_EXP_LIB=$L SHADOWTOPO_FUSE_MINDC=$f timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-north-star --no-shim --no-host-rate > $O/c2_f${f}_$rep.json 2> $O/c2_f${f}_$rep.err || { tail $O/c2_f${f}_$rep.err; exit 1; }
    echo -n "fuse $f rep $rep: "; python3 -c "import json; d=json.load(open('$O/c2_f${f}_$rep.json')); r=d['roofline']; print(round(d['ms_per_step'],4), 'sweep', round(r['avg_launch_ms'],4), 'delta', round(r['delta_kernel']['avg_launch_ms'],4))"
  done
done
