#!/bin/bash
# PMC A/B of bench variants: FETCH, WRITE and an SQ pass per variant, summed per kernel
# usage: scripts/gpu_pmc_ab.sh TAG CFG "args A" "args B" ...
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; CFG=$2; shift 2
i=0
for a in "$@"; do
  O=gpurun_out/pmc_${TAG}_$i
  mkdir -p $O
  B="bench.py --config $CFG --steps 1 --warmup 1 --no-cpu-baseline --no-host-rate $a"
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/f -o pmc --output-format csv -- python3 $B > $O/f.json 2> $O/f.err || { echo "fetch failed"; tail -5 $O/f.err; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/w -o pmc --output-format csv -- python3 $B > $O/w.json 2> $O/w.err || { echo "write failed"; tail -5 $O/w.err; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $O/s -o pmc --output-format csv -- python3 $B > $O/s.json 2> $O/s.err || { echo "sq failed"; tail -5 $O/s.err; exit 1; }
  echo "### variant $i: $a"
  python3 scripts/pmc_summary.py $O/f $O/w $O/s | grep -A12 -E "== k_relax" | head -40
  i=$((i+1))
done
