# final tree: whole GPU suite (two parts), smoke, profiles r06c
mkdir -p gpurun_out/r6ak
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
  --ignore=tests/test_gpu_fullsize_oracle.py > gpurun_out/r6ak/tests1.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6ak/smoke.log 2>&1 || exit 1
bash tools/refresh_profiles.sh r06c || exit 1
