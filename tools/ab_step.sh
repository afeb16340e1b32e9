#!/bin/bash
# Whole-step A/B of libraries: spring (headline) and mnist (config #4) bench
# lines for the in-tree library and each PAIG_AB_LIB given, alternating.
# usage (GPU box, repo root): bash tools/ab_step.sh <rounds> [ab/libpaig_x.so ...]
O=$GRAFT_REPO_ROOT/gpurun_out/abs
mkdir -p $O
R=$1; shift
one() {  # lib task args...
  local lib=$1 task=$2; shift 2
  local env=""; [ "$lib" != default ] && env="PAIG_AB_LIB=$lib"
  env $env timeout -k 10 200 python3 bench.py --cpu_baseline 0 --legs 0 --probe_steps 0 "$@" > $O/b.json 2> $O/b.err || { echo "bench failed: $lib $task"; tail -5 $O/b.err; exit 1; }
  echo "$task $lib :: $(python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
}
for r in $(seq $R); do
  for lib in default "$@"; do one $lib spring --steps 100 --warmup 10 || exit 1; done
done
for r in $(seq $R); do
  for lib in default "$@"; do one $lib mnist --task mnist_spring_color --batch 256 --seq_len 12 --steps 10 --warmup 3 || exit 1; done
done
