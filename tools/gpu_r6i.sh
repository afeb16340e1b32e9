# persistent-kernel tests (tree) + co-resident tests on the DPP variant + slab-reduction A/B
mkdir -p gpurun_out/r6i
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu -s tests/test_gpu_persistent.py > gpurun_out/r6i/tree.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit $rc; fi
PAIG_AB_LIB=ab/libpaig_dpp.so timeout -k 10 300 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu -s tests/test_gpu_persistent.py -k "coresident" > gpurun_out/r6i/dpp.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit $rc; fi
PAIG_AB_LIB=ab/libpaig_slabnew.so timeout -k 10 300 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k slab > gpurun_out/r6i/slab_test.log 2>&1 || exit 1
for lib in old new old new old new; do
  if [ $lib = new ]; then export PAIG_AB_LIB=ab/libpaig_slabnew.so; else unset PAIG_AB_LIB; fi
  timeout -k 10 200 python -u bench.py --legs 0 --cpu_baseline 0 --steps 100 --warmup 20 >> gpurun_out/r6i/bench_$lib.txt 2>&1 || exit 1
done
