#!/bin/bash
# Whole-step A/B of environment knobs: one bench line per setting.
# usage (GPU box, repo root): bash tools/ab_bench.sh "ENV=.. ENV2=.." "ENV=.." ...
O=$GRAFT_REPO_ROOT/gpurun_out/ab
mkdir -p $O
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 150 python3 $GRAFT_REPO_ROOT/bench.py --cpu_baseline 0 --legs 0 --probe_steps 0 --steps 100 --warmup 10 > $O/b$i.log 2>&1 || { echo "bench failed: $cfg"; exit 1; }
  echo "$cfg :: $(python3 -c "import json,sys; d=json.loads(open('$O/b$i.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
