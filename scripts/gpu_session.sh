#!/bin/bash
# GPU session: tests, then per-config roofline measurement (scripts/gpu_roofline.sh)
# usage: scripts/gpu_session.sh TAG [tests|notests] CFG:KERNEL ...
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
MODE=$1; shift
if [ "$MODE" = tests ]; then
  timeout -k 10 600 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/gputests_$TAG.log 2>&1
  rc=$?
  tail -5 gpurun_out/gputests_$TAG.log
  [ $rc -ne 0 ] && { echo "gpu tests failed rc=$rc"; tail -60 gpurun_out/gputests_$TAG.log; exit 1; }
fi
for spec in "$@"; do
  cfg=${spec%%:*}; k=${spec#*:}
  bash scripts/gpu_roofline.sh ${TAG}_$cfg $cfg 1.0 "$k" || exit 1
done
