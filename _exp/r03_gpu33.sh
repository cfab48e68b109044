#!/bin/bash
# r03 session 33b: delta walk stages only the slab rows holding a listed pair (masks two chunks ahead); PH2 epilogue loads hoisted
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03zd
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu -k "dense or c2" > $O/tests.log 2>&1
rc=$?; echo "tests: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
SHADOWTOPO_DELTA_COLBOUND=1 timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu -k "dense" > $O/tests4.log 2>&1
rc=$?; echo "tests xr4: $(tail -1 $O/tests4.log)"; [ $rc -ne 0 ] && { echo "tests failed"; tail -30 $O/tests4.log; exit 1; }
for run in "C2 2" "C2 1" "C2 2" "C2 1"; do
  set -- $run
  SHADOWTOPO_DELTA_COLBOUND=$2 timeout -k 10 300 python -u bench.py --config $1 --steps 10 --warmup 2 --no-cpu-baseline --no-host-rate --no-north-star --no-shim > $O/$1_$2.json 2> $O/$1_$2.err || { echo "$run failed"; tail $O/$1_$2.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$1_$2.json')); r=d['roofline']; print('$1 colbound=$2', round(d['ms_per_step'],3), 'sweep', round(r['avg_launch_ms'],3), 'delta', round(r['delta_kernel']['avg_launch_ms'],3))"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config C2 --steps 4 --warmup 1 --no-cpu-baseline --no-host-rate --no-north-star --no-shim > $GRAFT_REPO_ROOT/$O/kt.json 2> $GRAFT_REPO_ROOT/$O/kt.err || { echo "trace failed"; exit 1; }
grep -E "k_relax_dense_f<8, 2, 1, true, [12]" $GRAFT_REPO_ROOT/$O/kt/run_kernel_stats.csv | cut -d, -f1-4
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config C2 --steps 4 --warmup 1 --no-cpu-baseline --no-host-rate --no-north-star --no-shim > $GRAFT_REPO_ROOT/$O/kt.json 2> $GRAFT_REPO_ROOT/$O/kt.err || { echo "trace failed"; exit 1; }
echo traced
