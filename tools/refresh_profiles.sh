#!/bin/bash
# Round profiles of the bench workload (run on the GPU box from the repo root):
#   graph-mode and eager-mode rocprofv3 kernel stats, FETCH_SIZE / WRITE_SIZE
#   PMC passes (one counter per run).  Output: gpurun_out/prof_<tag>/
set -e
TAG=${1:-r03}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --cpu_baseline 0 --legs 0"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o graph -- python3 $B --steps 20 --warmup 3 --probe_steps 0 > $O/graph.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o eager -- python3 $B --graph 0 --steps 20 --warmup 3 --probe_steps 5 > $O/eager.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O -o f -- python3 $B --graph 0 --steps 3 --warmup 1 --probe_steps 1 > $O/f.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O -o w -- python3 $B --graph 0 --steps 3 --warmup 1 --probe_steps 1 > $O/w.log 2>&1
echo profiles done
