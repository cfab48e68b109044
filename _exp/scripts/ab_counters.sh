#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per step of the relax-family kernels for one bench command, two
# separate --pmc passes (_exp/scripts/ab_counters.py).
#   _exp/scripts/ab_counters.sh OUTDIR CFG "EXTRA BENCH ARGS" KERNEL_RE
set -o pipefail
export TMPDIR=/tmp
O=${1:?outdir}; CFG=$2; EXTRA=$3; KRE=$4
mkdir -p $O
B="bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate --no-north-star $EXTRA"
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d $O/pf -o pmc --output-format csv -- python3 $B > $O/pf.json 2> $O/pf.err || { echo "pmc fetch failed"; tail -20 $O/pf.err; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -d $O/pw -o pmc --output-format csv -- python3 $B > $O/pw.json 2> $O/pw.err || { echo "pmc write failed"; tail -20 $O/pw.err; exit 1; }
python3 _exp/scripts/ab_counters.py $O/pf $O/pw 4 "$KRE" $O/traffic.json
rm -rf $O/pf $O/pw
