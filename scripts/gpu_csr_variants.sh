set -o pipefail
mkdir -p gpurun_out
for v in 1 2 0; do
  timeout -k 10 300 python -u bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --no-host-rate --csr-variant $v > gpurun_out/csr_v$v.json 2> gpurun_out/csr_v$v.err || { echo "variant $v failed"; tail -5 gpurun_out/csr_v$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/csr_v$v.json')); print('v$v', round(d['ms_per_step'],2), d['engine']['rounds_per_step'], round(d['roofline']['avg_launch_ms'],2), d['roofline'].get('worklist_kernel'))"
done
timeout -k 10 300 python -u bench.py --config C4 --steps 1 --warmup 1 --no-cpu-baseline --no-host-rate --profile-counts > gpurun_out/csr_prof.json 2> gpurun_out/csr_prof.err && python3 -c "
import json; d=json.load(open('gpurun_out/csr_prof.json')); print('prof', d['ms_per_step'], d['engine'])"
