#!/bin/bash
# One bench line per BASELINE.json configuration besides the headline
# (GPU box, repo root): config #2 (spring bf16 B=512), spring split B=512,
# bouncing B=1024 R=96, plus the spring fp32-MFMA arithmetic.  Output:
# gpurun_out/cfg/<name>.log (last line = the JSON line)
O=$GRAFT_REPO_ROOT/gpurun_out/cfg
mkdir -p $O
B="python3 $GRAFT_REPO_ROOT/bench.py --cpu_baseline 0 --probe_steps 0 --steps 30 --warmup 5"
run() { n=$1; shift; timeout -k 10 200 $B "$@" > $O/$n.log 2>&1 || { echo "$n failed"; exit 1; }; echo "$n :: $(tail -1 $O/$n.log | cut -c1-200)"; }
run bf16_b512 --conv_math bf16 --batch 512
run split_b512 --batch 512
run fp32_b100 --conv_math fp32
run bouncing_b1024 --task bouncing_balls --batch 1024 --seq_len 100
