#!/bin/bash
# Round 4: one-frame launches deal bottom-up blocks of 8 rows (rows1), the
# bench's detector on torch's stream: GPU suite, A/B of the watchdog's host
# store (nostore = the same tree without it) at C2 and one frame, bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
bash profiles/run.sh r4stream2 "pytest" "ab c2 3 nostore cur" "ab b1 3 nostore cur -- --batch 1 --steps 50" "bench bench_c2" || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/r4stream2/bench_c2.json'));print(d['latency_batch1'])"
