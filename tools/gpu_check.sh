#!/bin/bash
# GPU-box validation at HEAD: the GPU test suite, smoke(), the bench line
# (no legs unless LEGS=1).  Output: gpurun_out/chk_<tag>/
TAG=${1:-cur}
O=gpurun_out/chk_$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py --legs ${LEGS:-0} --cpu_baseline 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json,sys; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('ms_per_step_median'))"
