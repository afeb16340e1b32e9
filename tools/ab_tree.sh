#!/bin/bash
# Whole-step A/B of two source trees (this one vs another checkout with its
# own built library, e.g. ab/tree_prev): bench lines alternating, R rounds.
# usage (GPU box, repo root): bash tools/ab_tree.sh <other tree> <task> <rounds>
O=$GRAFT_REPO_ROOT/gpurun_out/abt
mkdir -p $O
OT=$1; T=$2; R=$3
case $T in
  spring) A="--steps 100 --warmup 10";;
  mnist) A="--task mnist_spring_color --batch 256 --seq_len 12 --steps 10 --warmup 3";;
  3bp) A="--task 3bp_color --batch 512 --seq_len 20 --steps 20 --warmup 3";;
  bouncing) A="--task bouncing_balls --batch 1024 --seq_len 100 --steps 20 --warmup 3";;
  bf16) A="--batch 512 --conv_math bf16 --steps 50 --warmup 5";;
esac
for r in $(seq $R); do
  for tree in . $OT; do
    (cd $tree && timeout -k 10 200 python3 bench.py --cpu_baseline 0 --legs 0 --probe_steps 0 $A > $O/b.json 2> $O/b.err) || { echo "bench failed: $tree"; tail -5 $O/b.err; exit 1; }
    echo "$T [$tree] :: $(python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
  done
done
