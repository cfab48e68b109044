# A/B of builds of the engine (every _exp/ablib/*.so, e.g. old.so vs new.so) on one config, interleaved
# (the libraries travel with the tree: delete _exp/ablib after the A/B)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}
CFG=${2:-C2}
mkdir -p $O
for rep in 1 2 3; do
  for v in $(cd _exp/ablib && ls *.so | sed 's/\.so$//'); do
    SHADOWTOPO_EXP_LIB=$PWD/_exp/ablib/$v.so timeout -k 10 300 python -u _exp/c2_ab.py --config $CFG 20 1 TIMING=1 > $O/$v$rep.txt 2>&1 || { echo "$v failed"; tail -20 $O/$v$rep.txt; exit 1; }
    echo "$v: $(grep -v '^{' $O/$v$rep.txt | grep TIMING)"
  done
done
