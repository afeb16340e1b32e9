#!/bin/bash
# PMC passes over tools/conv_bench.py for a few conv kernels (one counter set
# per rocprofv3 run, each under its own time limit).  usage:
#   tools/pmc_run.sh OUTDIR "layers" "passes"
set -e
OUT=$1; LAYERS=$2; PASSES=$3
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $R/$OUT -o p1 -- python3 $R/tools/conv_bench.py 1000 split 3 $LAYERS $PASSES > $R/$OUT/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_MISC --kernel-trace --output-format csv -d $R/$OUT -o p2 -- python3 $R/tools/conv_bench.py 1000 split 3 $LAYERS $PASSES > $R/$OUT/p2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/$OUT -o p3 -- python3 $R/tools/conv_bench.py 1000 split 3 $LAYERS $PASSES > $R/$OUT/p3.log 2>&1
echo pmc done
