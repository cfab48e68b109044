#!/bin/bash
# kernel-trace stats + two separate PMC passes (FETCH_SIZE, WRITE_SIZE) over a short
# bench run -> profiles/relax_traffic.json key CFG@SCALE@1
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pmc}
CFG=${2:-C2}
SCALE=${3:-1.0}
B="bench.py --config $CFG --scale $SCALE --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 $B > gpurun_out/kt_$TAG.json 2> gpurun_out/kt_$TAG.err || { echo "kernel-trace failed"; tail -20 gpurun_out/kt_$TAG.err; exit 1; }
cat gpurun_out/kt_$TAG.json
head -6 gpurun_out/prof_$TAG/run_kernel_stats.csv | cut -c1-200
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf_$TAG -o pmc --output-format csv -- python3 $B > /dev/null 2> gpurun_out/pmcf_$TAG.err || { echo "pmc fetch failed"; tail -20 gpurun_out/pmcf_$TAG.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_$TAG -o pmc --output-format csv -- python3 $B > /dev/null 2> gpurun_out/pmcw_$TAG.err || { echo "pmc write failed"; tail -20 gpurun_out/pmcw_$TAG.err; exit 1; }
python3 scripts/pmc_traffic.py "$CFG@$SCALE@1" gpurun_out/pmcf_$TAG gpurun_out/pmcw_$TAG --kernel "${KERNEL:-k_relax_dense(}"
cp profiles/relax_traffic.json gpurun_out/relax_traffic_$TAG.json
