# float4 block epilogue of the 64 x 64 split GEMM (PAIG_GEMM_VST): bit-identity tests, GEMM A/B, step A/B
mkdir -p gpurun_out/r6an
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py \
  tests/test_gpu_byte_targets.py tests/test_gpu_parity.py -m gpu > gpurun_out/r6an/tests.log 2>&1 || exit 1
for r in 1 2; do
  for v in 1 0; do
    PAIG_GEMM_VST=$v timeout -k 10 120 python -u tools/gemm_bench.py 6 200 2000 l1_dgrad,l1_wgrad,l2_wgrad,l2_dgrad >> gpurun_out/r6an/gemm_v$v.txt 2>&1 || exit 1
  done
done
for r in 1 2 3; do
  for v in 1 0; do
    PAIG_GEMM_VST=$v timeout -k 10 300 python -u bench.py --legs 0 --cpu_baseline 0 --probe_steps 0 --steps 200 --warmup 20 >> gpurun_out/r6an/spring_v$v.txt 2>&1 || exit 1
  done
done
