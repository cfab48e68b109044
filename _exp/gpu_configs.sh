#!/bin/bash
# the other configurations' bench lines (C3, C4, C5; C4 with vertex loss), one after another
set -o pipefail
O=gpurun_out/${1:?tag}
mkdir -p $O
for cfg in C3 C4 C5; do
  timeout -k 10 400 python -u bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$cfg.json 2> $O/bench_$cfg.err || { echo "bench $cfg failed"; tail -20 $O/bench_$cfg.err; exit 1; }
  python3 scripts/bench_summary.py $O/bench_$cfg.json
done
