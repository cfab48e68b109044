#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "dense or geometric or prune" > gpurun_out/win_tests.log 2>&1
rc=$?; tail -2 gpurun_out/win_tests.log
[ $rc -ne 0 ] && { echo "tests failed rc=$rc"; grep -E "FAILED|Error|assert" gpurun_out/win_tests.log | head -20; exit 1; }
bash _exp/ab2.sh "base:" "win:" "base:" "win:"
