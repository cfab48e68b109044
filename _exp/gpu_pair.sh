set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05dp}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu -k "delta_pair" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u _exp/c2_ab.py 20 3 DELTA_PAIR=0,1 > $O/c2_ab.txt 2>&1 || { echo "ab failed"; tail -20 $O/c2_ab.txt; exit 1; }
grep -v "^{" $O/c2_ab.txt
