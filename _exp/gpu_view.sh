set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05vw}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_csr_gpu.py tests/test_fuzz_gpu.py tests/test_engine_gpu.py tests/test_topology_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
SHADOWTOPO_TRACE_PREP=1 timeout -k 10 400 python3 -u _exp/fresh_prep.py C5 > $O/c5.txt 2>&1 || { echo "c5 failed"; tail $O/c5.txt; exit 1; }
grep -v amdgpu.ids $O/c5.txt | tail -12
