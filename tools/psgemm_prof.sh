#!/bin/bash
# Kernel-trace durations of tools/psgemm_bench.py per wave tile (GPU box, repo root):
# gpurun_out/psprof_<tile>/ps_kernel_stats.csv and a one-line-per-kernel summary
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for t in ${TILES:-0 1 2 3}; do
  O=$R/gpurun_out/psprof_$t
  mkdir -p $O
  PAIG_PS_TILE=$t timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o ps -- python3 $R/tools/psgemm_bench.py 20 > $O/log.txt 2>&1 || exit 1
  echo "== tile $t"
  python3 $R/tools/prof_summary.py $(find $O -name 'ps_kernel_stats.csv' | head -1) 1 20
done
