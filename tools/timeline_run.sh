#!/bin/bash
# Graph-mode kernel trace of a few bench steps (GPU box, repo root) for tools/timeline.py
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/tl_${1:-x}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O -o tl -- python3 $R/bench.py --cpu_baseline 0 --legs 0 --steps 10 --warmup 3 --probe_steps 0 > $O/log.txt 2>&1
echo rc=$?
