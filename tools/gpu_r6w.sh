# rollout + reconstruction decode in one launch: bit-identity vs two launches, parity, then A/B bench
mkdir -p gpurun_out/r6w
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_byte_targets.py \
  tests/test_gpu_parity.py tests/test_gpu_training.py tests/test_gpu_decoder.py -m gpu > gpurun_out/r6w/tests.log 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --legs 0 --cpu_baseline 0 --steps 200 --warmup 20 >> gpurun_out/r6w/bench_merge.txt 2>&1 || exit 1
  PAIG_MERGE_ROLL=0 timeout -k 10 300 python -u bench.py --legs 0 --cpu_baseline 0 --steps 200 --warmup 20 >> gpurun_out/r6w/bench_sep.txt 2>&1 || exit 1
done
timeout -k 10 400 python -u bench.py --cpu_baseline 0 --steps 100 --warmup 10 > gpurun_out/r6w/legs_merge.txt 2>&1 || exit 1
PAIG_MERGE_ROLL=0 timeout -k 10 400 python -u bench.py --cpu_baseline 0 --steps 100 --warmup 10 > gpurun_out/r6w/legs_sep.txt 2>&1 || exit 1
