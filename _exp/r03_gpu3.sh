#!/bin/bash
# r03 session 3: dense-sweep phase stamps, drop-in lookup rates (lock-free cache), C3/C5
# benches, kernel-trace stats of the default bench line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03c
mkdir -p $O
SHADOWTOPO_EXP_LIB=_exp/lib/libshadowtopo_phase.so timeout -k 10 120 python -u _exp/r03_phase.py > $O/phase.json 2> $O/phase.err || { echo phase failed; tail $O/phase.err; exit 1; }
cat $O/phase.json
timeout -k 10 300 python -u scripts/shim_rates.py --queries > $O/shim_lookups_c4.jsonl 2> $O/shim_lookups.err || { echo shim rates failed; tail $O/shim_lookups.err; exit 1; }
cat $O/shim_lookups_c4.jsonl
for cfg in C3 C5; do
  timeout -k 10 400 python -u bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$cfg.json 2> $O/bench_$cfg.err || { echo "bench $cfg failed"; tail -20 $O/bench_$cfg.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$cfg.json')); print('$cfg', d['ms_per_step'], d['value'], d['roofline']['frac'], d['engine'].get('host_buffers_ms'))"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/kt_bench.json 2> $O/kt_bench.err || { echo "kernel trace failed"; tail -20 $O/kt_bench.err; exit 1; }
find $O/kt -name "*kernel_stats.csv" -exec cp {} $O/default_kernel_stats.csv \;
head -12 $O/default_kernel_stats.csv
