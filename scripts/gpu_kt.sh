#!/bin/bash
# rocprofv3 kernel-trace stats of one bench invocation: gpu_kt.sh TAG "<bench args>"
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-kt}
ARGS=${2:-"--steps 3 --warmup 1 --no-cpu-baseline"}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/kt_$TAG.json 2> gpurun_out/kt_$TAG.err || { echo "kernel-trace failed"; tail -20 gpurun_out/kt_$TAG.err; exit 1; }
cat gpurun_out/kt_$TAG.json
cut -d, -f1-4 gpurun_out/prof_$TAG/run_kernel_stats.csv | sed 's/(anonymous namespace):://g' | cut -c1-160 | head -12
