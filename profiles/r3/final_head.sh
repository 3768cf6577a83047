#!/bin/bash
# End-of-session evidence at HEAD: the GPU suite, smoke, the default bench line, rocprofv3 stats of the same command
O=gpurun_out/final; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1; cat $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value']/1e9, d['ms_per_step'], d['kernel_ms_per_launch'], d['latency_batch1']['ms_per_frame'], d['roofline']['fabric_frac'])"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o trace -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --latency-steps 0 --host-steps 0 > $GRAFT_REPO_ROOT/$O/bench_traced.json 2> $GRAFT_REPO_ROOT/$O/trace.err ) || exit 1
head -5 $O/trace/trace_kernel_stats.csv
