set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench1.json 2> gpurun_out/bench1.err
echo "bench exit $?"
tail -5 gpurun_out/bench1.err
cat gpurun_out/bench1.json
