# xmax slots zeroed by the first split forward (no memset): U-Net / parity / training tests, then A/B vs the memset
mkdir -p gpurun_out/r6t
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_unet_abi.py \
  tests/test_gpu_composite.py tests/test_gpu_parity.py tests/test_gpu_training.py tests/test_gpu_modules.py -m gpu > gpurun_out/r6t/tests.log 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --legs 0 --cpu_baseline 0 --steps 200 --warmup 20 >> gpurun_out/r6t/bench_new.txt 2>&1 || exit 1
  PAIG_XMAX_MEMSET=1 timeout -k 10 300 python -u bench.py --legs 0 --cpu_baseline 0 --steps 200 --warmup 20 >> gpurun_out/r6t/bench_memset.txt 2>&1 || exit 1
done
