#!/bin/bash
# SQ counters of the split GEMMs at the step's shapes (PMC passes, one run each).
# usage (GPU box, repo root): tools/pmc_gemm.sh [math]
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_gemm
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
M=${1:-4}
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $O -o p1 -- python3 $R/tools/gemm_bench.py $M 3 2000 > $O/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM --kernel-trace --output-format csv -d $O -o p2 -- python3 $R/tools/gemm_bench.py $M 3 2000 > $O/p2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O -o p3 -- python3 $R/tools/gemm_bench.py $M 3 2000 > $O/p3.log 2>&1
echo pmc done
