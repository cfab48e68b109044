#!/bin/bash
# The exact pass with 4 logged rows in flight per wave instead of 2 (experiments builds of the
# same tree: _exp/ab/libshadowtopo_base.so vs libshadowtopo_xr4.so): the dense and chained
# parity tests with xr4, then C2 interleaved.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}
mkdir -p $O
SHADOWTOPO_EXP_LIB=$PWD/_exp/ab/libshadowtopo_xr4.so timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -q -m gpu -k "dense or chained" --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/tests.log | head; exit 1; }
for rep in 1 2 3; do
  for v in base xr4; do
    SHADOWTOPO_EXP_LIB=$PWD/_exp/ab/libshadowtopo_$v.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-north-star --no-shim --no-host-rate > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || { tail $O/c2_${v}_$rep.err; exit 1; }
    echo -n "$v rep $rep: "; python3 -c "import json; d=json.load(open('$O/c2_${v}_$rep.json')); r=d['roofline']; print(round(d['ms_per_step'],4), 'sweep', round(r['avg_launch_ms'],4))"
  done
done
