#!/bin/bash
# r03 session 27: dense tables by transposed scatter + in-place tile transpose (parity); staged upload with 1/2/4 filler threads inside the bench process (C2 create)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03z2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu -k "dense or c2 or directed" > $O/tests.log 2>&1
rc=$?; echo "tests: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
export SHADOWTOPO_TRACE_BUILD=1
for w in 2 4 1 4 2 3; do
  SHADOWTOPO_UPLOAD_FILLERS=$w timeout -k 10 300 python -u bench.py --config C2 --steps 2 --warmup 1 --no-cpu-baseline --no-host-rate --no-north-star > $O/w$w.json 2> $O/w$w.err || { echo "$w failed"; tail $O/w$w.err; exit 1; }
  echo "== fillers=$w"; grep -E "^\[(upload|create)\]" $O/w$w.err | tr '\n' ';'; echo
  python3 -c "import json; d=json.load(open('$O/w$w.json')); print(d['engine']['cold_start_parts_ms'], d['engine']['cold_start_ms'])"
done
