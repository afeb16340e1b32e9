# c10 fused layer backward at 128-pixel tiles: A = 3 blocks per CU (even dY pitch), B = 2 blocks per CU; vs the in-tree 256
mkdir -p gpurun_out/r6v
for r in 1 2; do
  for lib in base A B; do
    L=""; [ $lib != base ] && L=paig_reproduction_amd/csrc/diag/libpaig_c10$lib.so
    echo "lib=$lib" >> gpurun_out/r6v/bwd.txt
    PAIG_AB_LIB=$L timeout -k 10 120 python -u tools/bwd_bench.py c10 1000 30 >> gpurun_out/r6v/bwd.txt 2>&1 || exit 1
  done
done
for lib in A B; do
  PAIG_AB_LIB=paig_reproduction_amd/csrc/diag/libpaig_c10$lib.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_persistent.py tests/test_gpu_conv_bwd.py -m gpu -k "16-16-32 or c10 or ups" > gpurun_out/r6v/tests_$lib.log 2>&1 || exit 1
done
