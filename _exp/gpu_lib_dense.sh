#!/bin/bash
# dense build variant: dense parity subset, then the library A/B on C2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py -k "heavy_first" > gpurun_out/wg_tests.log 2>&1 || { tail -20 gpurun_out/wg_tests.log; exit 1; }
tail -2 gpurun_out/wg_tests.log
bash _exp/gpu_lib_ab.sh wg2 C2
