#!/bin/bash
# SQ counters (one pass, 8 SQ counters) over eager bench steps: where each
# kernel's wave cycles go (issue / VALU / LDS / waits).  GPU box, repo root.
O=$GRAFT_REPO_ROOT/gpurun_out/sq
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O -o sq -- python3 $GRAFT_REPO_ROOT/bench.py --cpu_baseline 0 --legs 0 --graph 0 --steps 2 --warmup 1 --probe_steps 0 > $O/sq.log 2>&1
echo rc=$?
