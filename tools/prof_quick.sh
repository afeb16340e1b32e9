#!/bin/bash
# Quick graph-mode kernel stats of the bench workload (extra bench args in $2..).
# Output: gpurun_out/pq_<tag>/
TAG=${1:-cur}; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pq_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o graph -- python3 $R/bench.py --cpu_baseline 0 --legs 0 --steps 20 --warmup 3 --probe_steps 0 "$@" > $O/graph.log 2>&1
cd $R && python tools/prof_summary.py $O/graph_kernel_stats.csv 24 40
