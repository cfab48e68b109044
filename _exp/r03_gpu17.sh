#!/bin/bash
# r03 session 17: the first transfer of a process, per upload strategy (tools/upload)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03q
mkdir -p $O
: > $O/upload_first.jsonl
for rep in 1 2; do for m in pageable ring1 ring2 register; do
  timeout -k 10 60 tools/upload/upload_first $m >> $O/upload_first.jsonl 2>> $O/upload_first.err || { echo "$m failed"; tail $O/upload_first.err; exit 1; }
done; done
cat $O/upload_first.jsonl
