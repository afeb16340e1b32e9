# merged rollout launch at the legs' batch sizes: bf16 B=512 and bouncing B=1024, alternating 3x
mkdir -p gpurun_out/r6z
for r in 1 2 3; do
  for m in 1 0; do
    PAIG_MERGE_ROLL=$m timeout -k 10 200 python -u bench.py --legs 0 --cpu_baseline 0 --probe_steps 0 --batch 512 --conv_math bf16 --steps 60 --warmup 5 >> gpurun_out/r6z/bf16_m$m.txt 2>&1 || exit 1
    PAIG_MERGE_ROLL=$m timeout -k 10 200 python -u bench.py --legs 0 --cpu_baseline 0 --probe_steps 0 --task bouncing_balls --batch 1024 --seq_len 100 --steps 30 --warmup 3 >> gpurun_out/r6z/bounce_m$m.txt 2>&1 || exit 1
  done
done
for r in 1 2 3; do
  for m in 1 0; do
    PAIG_MERGE_ROLL=$m timeout -k 10 300 python -u bench.py --legs 0 --cpu_baseline 0 --probe_steps 0 --steps 200 --warmup 20 >> gpurun_out/r6z/spring_m$m.txt 2>&1 || exit 1
  done
done
