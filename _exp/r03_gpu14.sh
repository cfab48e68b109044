#!/bin/bash
# r03 session 14: upload strategies for the edge list (tools/upload), and the drop-in's GPU
# tests after the directed-graph cache change
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03n
mkdir -p $O
timeout -k 10 120 tools/upload/upload_bench > $O/upload.jsonl 2> $O/upload.err || { echo "upload bench failed"; tail $O/upload.err; exit 1; }
cat $O/upload.jsonl
timeout -k 10 400 python -u -m pytest tests/test_topology_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && { echo "tests failed"; exit 1; }
