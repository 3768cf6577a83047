#!/bin/bash
# Round 4, last check at HEAD: the GPU suite, smoke, the default bench line
# (C2 with the CPU baseline, the one-frame leg and the PMC roofline fields),
# C4 and C5 lines.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
bash profiles/run.sh r4final3 pytest smoke || exit 1
timeout -k 10 400 python3 bench.py > gpurun_out/r4final3/bench.json 2> gpurun_out/r4final3/bench.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/r4final3/bench.json'));r=d['roofline'];print('C2', d['value']/1e9, d['ms_per_step'], d['latency_batch1']['ms_per_frame'], {k:r.get(k) for k in ('frac','fabric_frac','td_frac','td_busy_frac','l2_hit','pmc_stale')})"
bash profiles/run.sh r4final3 "bench bench_C4 --config C4" "bench bench_C5 --config C5"
