#!/bin/bash
# Graph-mode kernel stats of the secondary configurations (mnist B=256,
# 3bp B=512), run on the GPU box from the repo root.  Output: gpurun_out/pc_<tag>/
set -e
TAG=${1:-cur}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pc_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --cpu_baseline 0 --legs 0 --probe_steps 0 --steps 10 --warmup 3"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o mnist -- python3 $B --task mnist_spring_color --batch 256 --seq_len 12 > $O/mnist.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o 3bp -- python3 $B --task 3bp_color --batch 512 --seq_len 20 > $O/3bp.log 2>&1
echo done
