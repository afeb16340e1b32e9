# full GPU suite, part 2: the full-size files
mkdir -p gpurun_out/r6r
timeout -k 10 1100 python -u -m pytest -x -v --timeout 650 --timeout-method thread tests/test_gpu_fullsize.py \
  tests/test_gpu_fullsize_oracle.py -m gpu > gpurun_out/r6r/tests2.log 2>&1 || exit 1
