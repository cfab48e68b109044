#!/bin/bash
# LDS-array utilisation of the dense sweep's chunk loop (one --pmc pass over the C2 bench command)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}
mkdir -p $O
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate --no-north-star --no-fresh"
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE -d $O/p -o pmc --output-format csv -- python3 $B > $O/p.json 2> $O/p.err || { echo "pass failed"; tail -5 $O/p.err; exit 1; }
for k in "k_relax_dense_f<8, 2, 1, true, 1," "k_relax_dense_f<8, 2, 1, true, 2," "k_relax_dense_delta_s<true>"; do
  echo "== $k"
  python3 scripts/sq_stall_counters.py "$k" 8 $O/p
done
