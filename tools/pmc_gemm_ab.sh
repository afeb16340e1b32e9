#!/bin/bash
# SQ counters of one GEMM shape, 64x64 tiles (PAIG_GEMM_TILE=0) vs the plan's
# wide tiles.  usage (GPU box, repo root): bash tools/pmc_gemm_ab.sh l1_fwd 4
set -e
S=${1:-l1_fwd}; M=${2:-4}
O=$GRAFT_REPO_ROOT/gpurun_out/pmcg_$S
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES"
for T in 0 1; do
  PAIG_GEMM_TILE=$T timeout -s KILL 60 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O -o t$T -- python3 $GRAFT_REPO_ROOT/tools/gemm_bench.py $M 5 2000 $S > $O/t$T.log 2>&1
done
echo ok
