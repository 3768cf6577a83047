#!/bin/bash
# Round 4: the colseg tests (column_pass 3, crossings inside a middle segment)
# and a C2 bench line whose roofline carries the re-stamped PMC fields.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
mkdir -p gpurun_out/r4segtest
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "segments or column_pass or extreme" > gpurun_out/r4segtest/pytest.log 2>&1 || { tail -20 gpurun_out/r4segtest/pytest.log; exit 1; }
tail -2 gpurun_out/r4segtest/pytest.log
timeout -k 10 400 python3 bench.py > gpurun_out/r4segtest/bench_c2_pmc_fresh.json 2> gpurun_out/r4segtest/bench.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/r4segtest/bench_c2_pmc_fresh.json'));r=d['roofline'];print(d['value']/1e9, d['ms_per_step'], d['latency_batch1']['ms_per_frame'], {k:r.get(k) for k in ('frac','fabric_frac','td_frac','td_busy_frac','l2_hit','traffic_ratio','pmc_stale')})"
