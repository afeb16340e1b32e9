set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in m2 new; do
  if [ $v = new ]; then unset PAIG_AB_LIB; else export PAIG_AB_LIB=$R/tools/ab/libpaig_$v.so; fi
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $R/gpurun_out/pmc_$v -o p1 -- python3 $R/tools/conv_bench.py 1000 split 3 c1 wgrad > $R/gpurun_out/pmc_$v.p1.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM --kernel-trace --output-format csv -d $R/gpurun_out/pmc_$v -o p2 -- python3 $R/tools/conv_bench.py 1000 split 3 c1 wgrad > $R/gpurun_out/pmc_$v.p2.log 2>&1
done
echo done
