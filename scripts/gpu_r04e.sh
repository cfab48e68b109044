set -o pipefail
bash scripts/gpu_push_ab.sh r04e || exit 1
timeout -k 10 400 python -u -m pytest tests/test_topology_gpu.py tests/test_oracle.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04e/topo_tests.log 2>&1; rc=$?; tail -4 gpurun_out/r04e/topo_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/r04e/topo_tests.log | head; exit 1; }
timeout -k 10 600 python -u scripts/shim_ab.py 2 > gpurun_out/r04e/shim_ab.jsonl 2> gpurun_out/r04e/shim_ab.err || { tail gpurun_out/r04e/shim_ab.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r04e/shim_ab.jsonl'):
    d=json.loads(l); print(d['build'], d['rep'], 'warm' if d['warm'] else 'cold', d['threads'], round(d['ns_per_call_per_thread'],1))"
