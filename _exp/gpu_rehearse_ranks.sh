#!/bin/bash
# bench.py's N-rank path rehearsed on a one-GPU box: N ranks on device 0, gloo for the
# exchange (SHADOWTOPO_BENCH_ONE_GPU=1).  Checks the launcher, sharding, codecs, barriers and
# the report; the timings are not measurements.
O=gpurun_out/${1:-rehearse}; mkdir -p $O
shift
for n in "${@:-2}"; do
  SHADOWTOPO_BENCH_ONE_GPU=1 timeout -k 10 500 python -u bench.py --gpus $n --steps 3 --warmup 1 --no-shim \
    > $O/n$n.json 2> $O/n$n.err || { echo "N=$n failed rc=$?"; tail -30 $O/n$n.err; exit 1; }
  python3 scripts/bench_summary.py $O/n$n.json || true
done
