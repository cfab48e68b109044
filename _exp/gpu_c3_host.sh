set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05c3h}
mkdir -p $O
timeout -k 10 300 python3 -u _exp/c3_host.py > $O/plain.txt 2>&1 || { echo "plain failed"; tail $O/plain.txt; exit 1; }
cat $O/plain.txt
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/kt -o run --output-format csv -- python3 _exp/c3_host.py > $O/prof.txt 2>&1 || { echo "prof failed"; tail $O/prof.txt; exit 1; }
