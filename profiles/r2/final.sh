#!/bin/bash
# Round-2 final measurement set: C2 bench line + rocprof stats + PMC (HBM, SQ,
# TCC, TA/TD/TCP), a kernel trace of the single-frame configuration, then the
# C4 and C5 lines.  GPU box, repo root.
O=gpurun_out/r2final
bash profiles/round_profile.sh $O || exit 1
bash profiles/collect_pmc_ta.sh $O/pmc_ta || exit 1
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/trace_b1" -o trace \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --batch 1 --steps 50 --no-cpu --latency-steps 0 --host-steps 0 > "$GRAFT_REPO_ROOT/$O/bench_b1.json" 2> "$GRAFT_REPO_ROOT/$O/trace_b1.err" ) || exit 1
timeout -k 10 300 python3 bench.py --config C4 --no-cpu --latency-steps 0 --host-steps 0 > $O/bench_C4.json 2> $O/bench_C4.err || exit 1
timeout -k 10 300 python3 bench.py --config C5 --no-cpu --latency-steps 0 --host-steps 0 > $O/bench_C5.json 2> $O/bench_C5.err || exit 1
cat $O/bench.json
