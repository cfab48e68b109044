#!/bin/bash
# r03 session 10: sparse-state loads past the CU's L1 (sc1) so a round sees the values written
# earlier in the same round -- CSR parity on the variant, then A/B against head on C4, C3, C5
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03j
mkdir -p $O
SHADOWTOPO_EXP_LIB=_exp/lib/libshadowtopo_l2.so timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu -k "not dense and not c2 and not c_harness" > $O/tests_l2.log 2>&1
rc=$?; tail -2 $O/tests_l2.log; [ $rc -ne 0 ] && { echo "tests failed"; exit 1; }
for run in "C4 head" "C4 l2" "C4 head" "C4 l2" "C4 head p" "C4 l2 p" "C3 head" "C3 l2" "C5 head" "C5 l2"; do
  set -- $run
  export SHADOWTOPO_EXP_LIB=_exp/lib/libshadowtopo_$2.so
  P=""; [ "$3" = p ] && P="--profile-counts"
  timeout -k 10 300 python -u bench.py --config $1 --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate $P > $O/$1_$2$3.json 2> $O/$1_$2$3.err || { echo "$1 $2 failed"; tail $O/$1_$2$3.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$1_$2$3.json')); e=d['engine']; r=d['roofline']; print('$1 $2 $3', round(d['ms_per_step'],2), 'relax', round(e['relax_ms_per_step'],2), 'rounds', e['rounds_per_step'], 'visits', e['visits_per_step'], 'changes', e['changes_per_step'])"
done
