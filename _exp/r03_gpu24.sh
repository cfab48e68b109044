#!/bin/bash
# r03 session 24: batched delta-stepping rounds on the GPU (OPT_DELTA_STEP: propagation gated
# by a per-batch threshold, pending vertices released as it rises) -- parity, then C4 / C5
# against the ungated rounds
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03x
mkdir -p $O
export SHADOWTOPO_EXP_LIB=_exp/lib/libshadowtopo_ds.so
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k "delta_stepping or random_sparse or directed" > $O/tests.log 2>&1
rc=$?; echo "tests: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && { echo "tests failed"; exit 1; }
for run in "C4 0" "C4 10000" "C4 20000" "C4 40000" "C4 0" "C4 20000" "C4 0 p" "C4 20000 p" "C5 0" "C5 20000"; do
  set -- $run
  P=""; [ "$3" = p ] && P="--profile-counts"
  timeout -k 10 300 python -u bench.py --config $1 --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate --no-north-star --delta-step $2 $P > $O/$1_$2$3.json 2> $O/$1_$2$3.err || { echo "$1 $2 failed"; tail $O/$1_$2$3.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$1_$2$3.json')); e=d['engine']; print('$1 delta=$2 $3', round(d['ms_per_step'],2), 'relax', round(e['relax_ms_per_step'],2), 'rounds', e['rounds_per_step'], 'visits', e['visits_per_step'])"
done
