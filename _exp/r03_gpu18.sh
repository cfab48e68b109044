#!/bin/bash
# r03 session 18: the pruned sweep split in two kernels (chunk loop at 62-73 VGPRs with LDS
# reads a row ahead; exact pass + epilogue) -- parity, then A/B: fused (default) vs split vs
# split without the row-ahead reads
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03r
mkdir -p $O
for v in sp spnr; do
  SHADOWTOPO_SWEEP_SPLIT=1 SHADOWTOPO_EXP_LIB=_exp/lib/libshadowtopo_$v.so timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k "dense or c2" > $O/tests_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 $O/tests_$v.log)"; [ $rc -ne 0 ] && { echo "tests $v failed"; exit 1; }
done
B="--steps 10 --warmup 2 --no-cpu-baseline --no-host-rate --no-north-star"
for run in "sp 0" "sp 1" "spnr 1" "sp 0" "sp 1" "spnr 1"; do
  set -- $run
  export SHADOWTOPO_EXP_LIB=_exp/lib/libshadowtopo_$1.so SHADOWTOPO_SWEEP_SPLIT=$2
  timeout -k 10 200 python -u bench.py $B > $O/c2_$1_$2.json 2> $O/c2_$1_$2.err || { echo "c2 $1 failed"; tail $O/c2_$1_$2.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c2_$1_$2.json')); r=d['roofline']; print('$1 split=$2 C2', round(d['ms_per_step'],3), 'sweep_ms', round(r['avg_launch_ms'],3), 'delta', round(r['delta_kernel']['avg_launch_ms'],3))"
done
