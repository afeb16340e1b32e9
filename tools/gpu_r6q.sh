# full GPU suite, part 1 (all but the full-size files) + smoke
mkdir -p gpurun_out/r6q
timeout -k 10 1100 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu \
  --ignore=tests/test_gpu_fullsize_oracle.py --ignore=tests/test_gpu_fullsize.py > gpurun_out/r6q/tests1.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6q/smoke.log 2>&1 || exit 1
