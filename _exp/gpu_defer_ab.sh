#!/bin/bash
# deferred-tightening chunk loop: dense parity with the variant library, then the library A/B on C2
set -o pipefail
O=gpurun_out/${1:?tag}
mkdir -p $O
SHADOWTOPO_EXP_LIB=$PWD/_exp/ablib/defer.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py -k "dense or heavy_first or glds or refilter or eight_wave" > $O/defer_tests.log 2>&1 || { tail -20 $O/defer_tests.log; exit 1; }
tail -2 $O/defer_tests.log
bash _exp/gpu_lib_ab.sh $1 C2
