#!/bin/bash
# readlane-weights chunk loop: parity, then a C2 A/B
set -o pipefail
mkdir -p gpu_out_tmp gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py -k "readlane" > gpurun_out/wl_tests.log 2>&1 &&
timeout -k 10 400 python -u _exp/c2_ab.py 20 4 SWEEP_WL=0,1 > gpurun_out/wl_ab.log 2>&1
rc=$?
tail -3 gpurun_out/wl_tests.log; cat gpurun_out/wl_ab.log | tail -12
exit $rc
