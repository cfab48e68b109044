#!/bin/bash
# Dense rounds without host read-backs (OPT_DENSE_SPEC): dense parity tests, then C2 with
# spec 0 / 2 interleaved on one box, and a kernel timeline of the default.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "dense or pinned or interleaved" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
for rep in 1 2; do
  for sp in 0 2; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-north-star --no-shim --dense-spec $sp > $O/c2_s${sp}_$rep.json 2> $O/c2_s${sp}_$rep.err || { tail $O/c2_s${sp}_$rep.err; exit 1; }
    echo -n "spec $sp rep $rep: "; python3 -c "import json; d=json.load(open('$O/c2_s${sp}_$rep.json')); e=d['engine']; print(round(d['ms_per_step'],4), 'host', round(d['config']['matrix_build_host_ms'],4), 'syncs', e['host_syncs_per_step'], 'rounds', e['rounds_per_step'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/kt -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-host-rate --no-north-star --no-shim > $O/kt.json 2> $O/kt.err && python3 scripts/timeline.py $O/kt --steps 3 > $O/timeline.txt && head -24 $O/timeline.txt
