#!/bin/bash
# pmc.sh LIB TAG "counters1" "counters2" ... : one rocprofv3 pass per counter group over a short bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
LIB=$1; TAG=$2; shift 2
i=0; dirs=""
for P in "$@"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P -d gpurun_out/xp_${TAG}_$i -o pmc --output-format csv -- python3 _exp/run.py $PWD/_exp/lib_$LIB.so --steps 1 --warmup 1 --no-cpu-baseline --no-host-rate > /dev/null 2> gpurun_out/xp_${TAG}_$i.err || { echo "pmc pass $i failed"; tail -5 gpurun_out/xp_${TAG}_$i.err; exit 1; }
  dirs="$dirs gpurun_out/xp_${TAG}_$i"
done
python3 scripts/pmc_summary.py $dirs | grep -A30 "delta_p" | head -30
