# incremental lean rounds: CSR + fuzz suites, then C4 (and optionally C5) A/B over the threshold
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05x}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_csr_gpu.py tests/test_fuzz_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 600 python -u _exp/c2_ab.py --config C4 5 2 CSR_INCREMENTAL=0,2,8,32 > $O/c4_ab.txt 2>&1 || { echo "ab failed"; tail -20 $O/c4_ab.txt; exit 1; }
grep -v "^{" $O/c4_ab.txt
if [ -n "$2" ]; then
  timeout -k 10 600 python -u _exp/c2_ab.py --config C5 2 1 CSR_INCREMENTAL=$2 > $O/c5_ab.txt 2>&1 || { echo "c5 ab failed"; tail -20 $O/c5_ab.txt; exit 1; }
  grep -v "^{" $O/c5_ab.txt
fi
