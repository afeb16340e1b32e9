# final-tree checks: GPU suite (all but full size) + smoke, then profiles (graph/eager stats, FETCH/WRITE passes)
mkdir -p gpurun_out/r6ad
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
  --ignore=tests/test_gpu_fullsize_oracle.py --ignore=tests/test_gpu_fullsize.py > gpurun_out/r6ad/tests1.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6ad/smoke.log 2>&1 || exit 1
bash tools/refresh_profiles.sh r06b || exit 1
