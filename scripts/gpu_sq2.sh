#!/bin/bash
# LDS / VALU occupancy counters for one bench invocation: gpu_sq2.sh TAG "<bench args>"
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-sq2}
ARGS=${2:-"--steps 1 --warmup 1 --no-cpu-baseline --no-host-rate"}
P1="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_WAVES SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P -d gpurun_out/sq2_${TAG}_$i -o pmc --output-format csv -- python3 bench.py $ARGS > /dev/null 2> gpurun_out/sq2_${TAG}_$i.err || { echo "pmc pass $i failed"; tail -20 gpurun_out/sq2_${TAG}_$i.err; exit 1; }
done
python3 scripts/pmc_summary.py gpurun_out/sq2_${TAG}_1 gpurun_out/sq2_${TAG}_2 | head -48
