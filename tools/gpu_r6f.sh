# fused layer backward A/B (ReLU'-mask prefetch before / after the next tile's prefetch) + bf16 envelope tests
mkdir -p gpurun_out/r6f
timeout -k 10 600 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu -s tests/test_gpu_parity.py tests/test_gpu_fullsize_oracle.py tests/test_gpu_conv_bwd.py tests/test_gpu_persistent.py -k "bf16 or fused or bwd" > gpurun_out/r6f/t.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit $rc; fi
L=c2,c4,c7,c8,c9,c10,c11,c12
for lib in early new early new; do
  if [ $lib = early ]; then export PAIG_AB_LIB=ab/libpaig_early.so; else unset PAIG_AB_LIB; fi
  timeout -k 10 120 python -u tools/bwd_bench.py $L 1000 20 >> gpurun_out/r6f/bwd_$lib.txt 2>&1 || exit 1
done
unset PAIG_AB_LIB
PAIG_AB_LIB=ab/libpaig_stamps.so timeout -k 10 120 python -u tools/bwd_bench.py $L 1000 20 > gpurun_out/r6f/stamps.txt 2>&1 || exit 1
for lib in early new early new; do
  if [ $lib = early ]; then export PAIG_AB_LIB=ab/libpaig_early.so; else unset PAIG_AB_LIB; fi
  timeout -k 10 200 python -u bench.py --legs 0 --cpu_baseline 0 --steps 100 --warmup 20 >> gpurun_out/r6f/bench_$lib.txt 2>&1 || exit 1
done
