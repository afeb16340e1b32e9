# persistent-kernel tests (tree library), then the co-resident tests on the round-5 DPP variant (must fail)
mkdir -p gpurun_out/r6h
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu -s tests/test_gpu_persistent.py > gpurun_out/r6h/tree.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit $rc; fi
PAIG_AB_LIB=ab/libpaig_dpp.so timeout -k 10 300 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu -s tests/test_gpu_persistent.py -k "coresident" > gpurun_out/r6h/dpp.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit $rc; fi
exit 0
