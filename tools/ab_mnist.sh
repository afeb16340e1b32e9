#!/bin/bash
# mnist (config #4) step time per library: default, then each PAIG_AB_LIB given.
# usage (GPU box, repo root): bash tools/ab_mnist.sh [ab/libpaig_x.so ...]
O=$GRAFT_REPO_ROOT/gpurun_out/abm
mkdir -p $O
run() {
  timeout -k 10 200 python3 $GRAFT_REPO_ROOT/bench.py --task mnist_spring_color --batch 256 --seq_len 12 --legs 0 \
    --cpu_baseline 0 --probe_steps 0 --steps 10 --warmup 3 > $O/b.json 2> $O/b.err || { echo "bench failed: $1"; tail -5 $O/b.err; exit 1; }
  echo "$1 :: $(python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
}
run default
for lib in "$@"; do PAIG_AB_LIB=$lib run $lib; done
