#!/bin/bash
# r03 first GPU session: counter calibration of the sparse relax access shapes, C4 batch-group
# exploration, default bench.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03a
mkdir -p $O
timeout -k 10 120 tools/calib/calib_fetch 2 > $O/calib_plain.json 2> $O/calib_plain.err || { echo calib failed; cat $O/calib_plain.err; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/cf -o pmc --output-format csv -- tools/calib/calib_fetch 1 > $O/calib_f.json 2> $O/calib_f.err || { echo pmc f failed; tail $O/calib_f.err; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/cw -o pmc --output-format csv -- tools/calib/calib_fetch 1 > $O/calib_w.json 2> $O/calib_w.err || { echo pmc w failed; tail $O/calib_w.err; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d $O/cr -o pmc --output-format csv -- tools/calib/calib_fetch 1 > $O/calib_r.json 2> $O/calib_r.err || { echo pmc r failed; tail $O/calib_r.err; }
timeout -k 10 400 python3 -u _exp/r03_c4_groups.py C4 > $O/c4_groups.jsonl 2> $O/c4_groups.err || { echo c4 groups failed; tail -20 $O/c4_groups.err; exit 1; }
cat $O/c4_groups.jsonl
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
