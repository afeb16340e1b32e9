# byte targets: parity (bit-identical steps, all task shapes) + decoder/data tests, then A/B bench
mkdir -p gpurun_out/r6n
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_byte_targets.py \
  tests/test_device_data.py tests/test_gpu_decoder.py -m gpu > gpurun_out/r6n/tests.log 2>&1 || exit 1
for bt in 1 0 1 0; do
  timeout -k 10 300 python -u bench.py --legs 0 --cpu_baseline 0 --steps 200 --warmup 20 --byte_targets $bt \
    >> gpurun_out/r6n/bench_bt$bt.txt 2>&1 || exit 1
done
for bt in 1 0; do
  timeout -k 10 400 python -u bench.py --cpu_baseline 0 --steps 100 --warmup 10 --byte_targets $bt \
    >> gpurun_out/r6n/legs_bt$bt.txt 2>&1 || exit 1
done
