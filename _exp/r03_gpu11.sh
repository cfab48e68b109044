#!/bin/bash
# r03 session 11: grid rounds with K batches interleaved vertex-major per XCD (a smaller
# Gauss-Seidel window per batch) -- CSR parity on il16, A/B against head on C4 and C5
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03k
mkdir -p $O
SHADOWTOPO_EXP_LIB=_exp/lib/libshadowtopo_il16.so timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu -k "not dense and not c2 and not c_harness" > $O/tests_il16.log 2>&1
rc=$?; tail -1 $O/tests_il16.log; [ $rc -ne 0 ] && { echo "tests failed"; exit 1; }
for run in "C4 head" "C4 il4" "C4 il16" "C4 head" "C4 il4" "C4 il16" "C4 il4 p" "C4 il16 p" "C5 head" "C5 il16"; do
  set -- $run
  export SHADOWTOPO_EXP_LIB=_exp/lib/libshadowtopo_$2.so
  P=""; [ "$3" = p ] && P="--profile-counts"
  timeout -k 10 300 python -u bench.py --config $1 --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate $P > $O/$1_$2$3.json 2> $O/$1_$2$3.err || { echo "$1 $2 failed"; tail $O/$1_$2$3.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$1_$2$3.json')); e=d['engine']; r=d['roofline']; print('$1 $2 $3', round(d['ms_per_step'],2), 'relax', round(e['relax_ms_per_step'],2), 'rounds', e['rounds_per_step'], 'visits', e['visits_per_step'], 'changes', e['changes_per_step'])"
done
