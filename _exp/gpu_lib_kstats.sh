#!/bin/bash
# per-kernel times of every _exp/ablib/*.so on one config (rocprofv3 --kernel-trace --stats over
# _exp/c2_ab.py): which kernel a variant moves
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}
CFG=${2:-C2}
mkdir -p $O
for v in $(cd _exp/ablib && ls *.so | sed 's/\.so$//'); do
  export SHADOWTOPO_EXP_LIB=$PWD/_exp/ablib/$v.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o k -- python3 _exp/c2_ab.py --config $CFG 10 1 TIMING=1 > $O/$v.txt 2>&1 || { echo "$v failed"; tail -20 $O/$v.txt; exit 1; }
  echo "$v: $(grep TIMING $O/$v.txt | head -1)"
done
