# final tree re-check after the weight-prep block size change: whole GPU suite incl. full-size oracle tests, smoke, a default bench line
mkdir -p gpurun_out/r6as
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
  --ignore=tests/test_gpu_fullsize_oracle.py > gpurun_out/r6as/tests1.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize_oracle.py \
  -m gpu > gpurun_out/r6as/tests2.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6as/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r6as/bench.json 2> gpurun_out/r6as/bench.err || exit 1
