# weight-prep blocks after the first conv's blocks in their shared launch (PAIG_WPREP_LAST): tests, kernel stats, step A/B
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6ap
mkdir -p $O
PAIG_WPREP_LAST=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_byte_targets.py tests/test_gpu_unet_abi.py -m gpu > $O/tests.log 2>&1
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --cpu_baseline 0 --legs 0"
for v in 1 0; do
  PAIG_WPREP_LAST=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o k$v -- python3 $B --steps 40 --warmup 3 --probe_steps 0 > $O/k$v.log 2>&1
done
cd $R
for r in 1 2 3; do
  for v in 1 0; do
    PAIG_WPREP_LAST=$v timeout -k 10 300 python -u bench.py --legs 0 --cpu_baseline 0 --probe_steps 0 --steps 200 --warmup 20 >> $O/spring_v$v.txt 2>&1
  done
done
