#!/bin/bash
# Fused layer backward per-launch times (tools/bwd_bench.py) for the in-tree
# library and each A/B library given.  usage (GPU box, repo root):
#   bash tools/ab_bwd.sh <layers> [ab/libpaig_x.so ...]
O=$GRAFT_REPO_ROOT/gpurun_out/abb
mkdir -p $O
LAY=$1; shift
echo "== default"; timeout -k 10 180 python3 -u tools/bwd_bench.py $LAY > $O/default.txt 2>&1 || { tail -5 $O/default.txt; exit 1; }
grep -v amdgpu.ids $O/default.txt
for lib in "$@"; do
  n=$(basename $lib .so)
  echo "== $n"; PAIG_AB_LIB=$lib timeout -k 10 180 python3 -u tools/bwd_bench.py $LAY > $O/$n.txt 2>&1 || { tail -5 $O/$n.txt; exit 1; }
  grep -v amdgpu.ids $O/$n.txt
done
