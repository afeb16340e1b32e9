# final tree: the full-size oracle tests, then the default bench (legs + cpu baseline)
mkdir -p gpurun_out/r6al
timeout -k 10 800 python -u -m pytest -x -q --timeout 650 --timeout-method thread tests/test_gpu_fullsize_oracle.py -m gpu > gpurun_out/r6al/tests2.log 2>&1 || exit 1
timeout -k 10 350 python -u bench.py > gpurun_out/r6al/bench.txt 2> gpurun_out/r6al/bench.err || exit 1
