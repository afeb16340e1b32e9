# merged rollout launch (final form): bit-identity + parity subset, then the default bench twice
mkdir -p gpurun_out/r6aa
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_byte_targets.py \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu > gpurun_out/r6aa/tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 600 python -u bench.py --cpu_baseline 0 > gpurun_out/r6aa/bench_$r.txt 2>&1 || exit 1
done
