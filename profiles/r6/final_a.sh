#!/bin/bash
# Round 6 evidence at HEAD, part A (code frozen): the GPU suite, smoke, the
# default bench line (C2 with the CPU baseline and the one-frame latency leg),
# C1 / C4 / C5 lines, rocprofv3 kernel-trace summaries of the default command
# and of one frame per step.  Part B (final_b.sh): the PMC passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=gpurun_out/r6final; mkdir -p $R/$O; cd $R
bash profiles/run.sh r6final pytest smoke || exit 1
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench.json'));print('C2', d['value']/1e9, d['ms_per_step'], d['kernel_ms_per_launch'], d['latency_batch1']['ms_per_frame'], d.get('cpu_baseline',{}).get('value'))"
bash profiles/run.sh r6final "bench bench_C4 --config C4" "bench bench_C5 --config C5" "rocprof trace" \
  "rocprof trace_b1 --batch 1 --steps 50" || exit 1
timeout -k 10 300 python3 bench.py --config C1 > $O/bench_C1.json 2> $O/bench_C1.err || exit 1
timeout -k 10 240 python3 profiles/r5/latency_legs.py > $O/legs.json 2> $O/legs.err || exit 1
echo final_a done
