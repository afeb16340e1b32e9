set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv_bwd.py > gpurun_out/ab1_tests.log 2>&1 && \
for cfg in "base" "PAIG_AB_LIB=ab/libpaig_s1.so" "PAIG_BWD_MIN_TPB=2" "PAIG_BWD_MIN_TPB=3" "PAIG_GEMM_SMALLK=1" "base"; do
  if [ "$cfg" = base ]; then e=""; else e="$cfg"; fi
  env $e timeout -k 10 200 python bench.py --steps 200 --warmup 30 > gpurun_out/ab1_$(echo $cfg|tr '=/' '__').json 2>gpurun_out/ab1_err.log || exit 1
  echo "$cfg $(python -c "import json,sys;d=json.loads(open('gpurun_out/ab1_$(echo $cfg|tr '=/' '__').json').read().strip().splitlines()[-1]);print(d['value'],d.get('value_median'),d['ms_per_step'])")"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr1 -o tr -- python bench.py --steps 6 --warmup 3 > gpurun_out/tr1.log 2>&1
