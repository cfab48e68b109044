#!/bin/bash
# Quiet-predecessor gather skip (pull rounds' change masks): CSR parity tests, then C3 / C4 / C5
# with the current build against the previous engine (_exp/ab/libshadowtopo_base.so), interleaved.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_csr_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
for cfg in ${CFGS:-C3 C4 C5}; do
  for rep in 1 2; do
    for v in ${VARIANTS:-cur base}; do
      if [ $v = cur ]; then unset SHADOWTOPO_EXP_LIB; else export SHADOWTOPO_EXP_LIB=$PWD/_exp/ab/libshadowtopo_$v.so; fi
      timeout -k 10 400 python -u bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate > $O/bench_${cfg}_${v}_$rep.json 2> $O/bench_${cfg}_${v}_$rep.err || { echo "bench $cfg $v failed"; tail -20 $O/bench_${cfg}_${v}_$rep.err; exit 1; }
      echo -n "$cfg $v $rep: "; python3 -c "import json; d=json.load(open('$O/bench_${cfg}_${v}_$rep.json')); print(d['ms_per_step'], d['engine'].get('host_syncs_per_step'))"
    done
  done
done
