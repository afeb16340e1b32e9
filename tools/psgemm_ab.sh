#!/bin/bash
# psgemm micro-bench kernel times, default library vs PAIG_AB_LIB=$1 (GPU box, repo root)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in base ab; do
  O=$R/gpurun_out/psab_$v
  mkdir -p $O
  if [ $v = ab ]; then export PAIG_AB_LIB=$R/$1; fi
  PAIG_PS_TILE=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o ps -- python3 $R/tools/psgemm_bench.py 20 > $O/log.txt 2>&1 || exit 1
done
echo done
