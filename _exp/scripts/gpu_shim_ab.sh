#!/bin/bash
# Lookup A/B (verdict r03 item 6): current vs r02k, one harness, warm pass finished before timing
# (the r02k build, tools/abshim/r02k, is listed in .gpurunignore since the A/B is recorded:
# drop that line to run this again)
set -o pipefail
O=gpurun_out/${1:?tag}
mkdir -p $O
timeout -k 10 900 python -u _exp/scripts/shim_ab.py ${2:-4} > $O/shim_ab.jsonl 2> $O/shim_ab.err || { tail $O/shim_ab.err; exit 1; }
python3 - $O <<'PY'
import json, statistics as S, collections, sys
r = collections.defaultdict(list); x = {}; pr = collections.defaultdict(list)
for l in open(sys.argv[1] + '/shim_ab.jsonl'):
    d = json.loads(l); k = (d['build'], 'warm' if d['warm'] else 'cold', d['threads'])
    r[k].append(d['ns_per_call_per_thread']); pr[k].append(d['prepare_s'])
    x[k] = (d.get('dijkstra_runs_after_warm'), d.get('dijkstra_runs'), d.get('cached_paths'))
for k in sorted(r): print(k, 'median', round(S.median(r[k]), 1), 'all', [round(v) for v in r[k]], 'runs warm/total, paths', x[k], 'prepare_s', round(S.median(pr[k]), 3))
PY
