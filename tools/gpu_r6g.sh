# the round-5 DPP upsample staging defect, reproduced on an A/B library (ab/libpaig_dpp.so)
mkdir -p gpurun_out/r6g
export PAIG_AB_LIB=ab/libpaig_dpp.so
timeout -k 10 300 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu -s tests/test_gpu_persistent.py -k "wgrad_fused_upsample" > gpurun_out/r6g/t_dpp.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit $rc; fi
for s in "128 32 16" "64 32 32" "32 32 64"; do
  timeout -k 10 120 python -u tools/ups_probe.py $s 64 24 >> gpurun_out/r6g/probe_dpp.txt 2>&1 || exit 1
done
unset PAIG_AB_LIB
for s in "128 32 16" "64 32 32"; do
  timeout -k 10 120 python -u tools/ups_probe.py $s 64 24 >> gpurun_out/r6g/probe_tree.txt 2>&1 || exit 1
done
