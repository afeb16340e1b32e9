#!/bin/bash
# PMC passes over tools/dec_bench.py (decoder kernels at the BASELINE shapes):
# SQ issue/wait breakdown, LDS, and memory-side traffic, one counter set per
# rocprofv3 run under its own time limit.  usage (GPU box, repo root):
#   bash tools/pmc_dec.sh OUTDIR "case,case"
set -e
OUT=$GRAFT_REPO_ROOT/$1; CASES=$2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $OUT -o p1 -- python3 $R/tools/dec_bench.py 3 $CASES > $OUT/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC --kernel-trace --output-format csv -d $OUT -o p2 -- python3 $R/tools/dec_bench.py 3 $CASES > $OUT/p2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT -o p3 -- python3 $R/tools/dec_bench.py 3 $CASES > $OUT/p3.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT -o p4 -- python3 $R/tools/dec_bench.py 3 $CASES > $OUT/p4.log 2>&1
echo pmc done
