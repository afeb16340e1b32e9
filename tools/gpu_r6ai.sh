# the batched slab reduction carried by the first layer's weight gradient: tests, then A/B bench
mkdir -p gpurun_out/r6ai
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_byte_targets.py \
  tests/test_gpu_parity.py tests/test_gpu_training.py tests/test_gpu_modules.py tests/test_gpu_decoder.py \
  tests/test_gpu_fullsize.py tests/test_gpu_dp.py tests/test_gpu_composite.py tests/test_gpu_unet_abi.py tests/test_gpu_kernels.py -m gpu > gpurun_out/r6ai/tests.log 2>&1 || exit 1
for r in 1 2 3; do
  for m in 1 0; do
    PAIG_SLAB_MERGE=$m timeout -k 10 300 python -u bench.py --legs 0 --cpu_baseline 0 --probe_steps 0 --steps 200 --warmup 20 >> gpurun_out/r6ai/spring_m$m.txt 2>&1 || exit 1
  done
done
