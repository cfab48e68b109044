set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05fr}
mkdir -p $O
SHADOWTOPO_TRACE_PREP=1 timeout -k 10 400 python3 -u _exp/fresh_prep.py C5 > $O/c5.txt 2>&1 || { echo "c5 failed"; tail $O/c5.txt; exit 1; }
grep -v amdgpu.ids $O/c5.txt
