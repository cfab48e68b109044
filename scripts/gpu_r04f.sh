#!/bin/bash
# r04 session: full GPU suite on the renumbered-view tree, then the push A/B (C4, C5), the
# lookup A/B against the r02k build, and the C5 / C4 bench lines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && { echo "gpu tests failed rc=$rc"; grep -E "FAILED|Error|assert" $O/gpu_tests.log | head -20; exit 1; }
bash scripts/gpu_push_ab.sh r04f || exit 1
timeout -k 10 600 python -u scripts/shim_ab.py 2 > $O/shim_ab.jsonl 2> $O/shim_ab.err || { tail $O/shim_ab.err; exit 1; }
python3 -c "
import json
for l in open('$O/shim_ab.jsonl'):
    d=json.loads(l); print(d['build'], d['rep'], 'warm' if d['warm'] else 'cold', d['threads'], round(d['ns_per_call_per_thread'],1))"
