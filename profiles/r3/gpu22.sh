#!/bin/bash
# Round 3, call 22: configs suite + fused parity on the final fuse rule, the
# C4 line (separate integral again by default), C5 PMC on the fused build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g22
mkdir -p $O
cd $R
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_parity.py -k "configs or fused or integral" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 400 python3 bench.py --config C4 --no-cpu > $O/bench_C4.json 2> $O/bench_C4.err || { tail -20 $O/bench_C4.err; exit 1; }
cut -c1-300 $O/bench_C4.json
bash profiles/collect_pmc_cfg.sh gpurun_out/r3g22/C5 --config C5 && echo pmc ok
