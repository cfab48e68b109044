set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05c3s}
mkdir -p $O
for sp in 200 5000 50000; do
timeout -k 10 300 python3 -u _exp/c3_host.py $sp > $O/spin$sp.txt 2>&1 || { echo "spin $sp failed"; tail $O/spin$sp.txt; exit 1; }
echo spin $sp; cat $O/spin$sp.txt
done
timeout -k 10 300 python -u _exp/c2_ab.py --config C3 5 2 SPIN_US=200,50000 > $O/c3_ab.txt 2>&1 || { echo "ab failed"; tail $O/c3_ab.txt; exit 1; }
grep -v "^{" $O/c3_ab.txt
