#!/bin/bash
# Stall counters of the dense sweep's chunk loop (two --pmc passes over the same C2 bench command)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}
mkdir -p $O
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate --no-north-star --no-fresh"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM -d $O/p1 -o pmc --output-format csv -- python3 $B > $O/p1.json 2> $O/p1.err || { echo "pass 1 failed"; tail -5 $O/p1.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MISC -d $O/p2 -o pmc --output-format csv -- python3 $B > $O/p2.json 2> $O/p2.err || { echo "pass 2 failed"; tail -5 $O/p2.err; exit 1; }
for k in "k_relax_dense_f<8, 2, 1, true, 1," "k_relax_dense_f<8, 2, 1, true, 2," "k_relax_dense_delta_s<true>"; do  # (the stall pass of r06k ran the LDS-DMA form)
  echo "== $k"
  python3 scripts/sq_stall_counters.py "$k" 8 $O/p1 $O/p2
done
