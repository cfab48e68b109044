#!/bin/bash
# C2 headline step with the sweep's chunk loop staged by LDS-DMA (1) or registers (0), interleaved
set -o pipefail
O=gpurun_out/${1:?tag}
mkdir -p $O
for rep in 1 2 3; do
  for g in 0 1; do
    timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-rate --no-north-star --no-fresh --no-shim --sweep-glds $g > $O/c2_g${g}_r$rep.json 2> $O/c2_g${g}_r$rep.err || { echo "glds $g failed"; tail -5 $O/c2_g${g}_r$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c2_g${g}_r$rep.json')); r=d['roofline']; print('rep $rep glds $g step', round(d['ms_per_step'],3), 'sweep', round(r['avg_launch_ms'],3))"
  done
done
