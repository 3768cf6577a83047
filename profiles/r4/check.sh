#!/bin/bash
# GPU check while iterating (round 4): the GPU suite, smoke, one C2 bench line.
# usage: profiles/r4/check.sh <out-dir-name> [pytest -k expr]
O=gpurun_out/${1:-check}; mkdir -p $O
K=${2:+-k "$2"}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $K > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1; cat $O/smoke.log
timeout -k 10 300 python bench.py --no-cpu --host-steps 0 > $O/bench.json 2> $O/bench.err || exit 1
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value']/1e9, d['ms_per_step'], d['kernel_ms_per_launch'], d['latency_batch1']['ms_per_frame'])"
