# byte-target forward decoder (K=2, H=32) at 5 blocks per CU (A/B library) vs 4: decoder tests on the A/B lib, bench alternating
mkdir -p gpurun_out/r6aj
PAIG_AB_LIB=paig_reproduction_amd/csrc/diag/libpaig_decm5.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_byte_targets.py tests/test_gpu_decoder.py -m gpu > gpurun_out/r6aj/tests.log 2>&1 || exit 1
for r in 1 2 3; do
  PAIG_AB_LIB=paig_reproduction_amd/csrc/diag/libpaig_decm5.so timeout -k 10 300 python -u bench.py --legs 0 --cpu_baseline 0 --steps 200 --warmup 20 >> gpurun_out/r6aj/m5.txt 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --legs 0 --cpu_baseline 0 --steps 200 --warmup 20 >> gpurun_out/r6aj/m4.txt 2>&1 || exit 1
done
