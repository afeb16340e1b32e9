#!/bin/bash
# mnist kernel stats under two environment settings (A/B of a U-Net option).
# usage (GPU box): bash tools/prof_mnist_ab.sh <tag> "<env A>" "<env B>"   ("-" = defaults)
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pm_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --cpu_baseline 0 --legs 0 --probe_steps 0 --steps 10 --warmup 3 --task mnist_spring_color --batch 256 --seq_len 12"
n=0
for cfg in "$@"; do
  n=$((n+1)); e=""; [ "$cfg" != "-" ] && e="$cfg"
  for kv in $e; do export "$kv"; done
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o m$n -- python3 $B > $O/m$n.log 2>&1 || exit 1
  for kv in $e; do unset "${kv%%=*}"; done
  echo "[$cfg]"; cd $R && python tools/prof_summary.py $O/m${n}_kernel_stats.csv 14 30; cd /tmp
done
