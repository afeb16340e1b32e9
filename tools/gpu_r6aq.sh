# weight-prep block size (PAIG_WPREP_S build macro: 2 / 4 (default) / 8 k-steps per block), swapped-in libraries:
# the prep tests, the first conv + prep launch's duration, step A/B
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6aq
mkdir -p $O
L=$R/paig_reproduction_amd
cp $L/libpaig_hip.so $L/libpaig_hip_s4.so
for s in 2 8 4; do
  cp $L/libpaig_hip_s$s.so $L/libpaig_hip.so
  timeout -k 10 200 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_conv_bwd.py tests/test_gpu_byte_targets.py \
    -m gpu -k wprep > $O/tests_s$s.log 2>&1
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o k$s -- python3 $R/bench.py --cpu_baseline 0 --legs 0 --steps 40 --warmup 3 --probe_steps 0 > $O/k$s.log 2>&1
  cd $R
done
for r in 1 2; do
  for s in 2 8 4; do
    cp $L/libpaig_hip_s$s.so $L/libpaig_hip.so
    timeout -k 10 300 python -u bench.py --legs 0 --cpu_baseline 0 --probe_steps 0 --steps 200 --warmup 20 >> $O/spring_s$s.txt 2>&1
  done
done
