#!/bin/bash
# Round 3, call 52: colsum in table order from 2 frames (colsum4 for one):
# GPU parity of the integral paths, then a kernel trace of a short bench
# (the gaps between a step's kernels).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g52
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --latency-steps 10 --host-steps 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json | head -c 400; echo
find $O/trace -name "*.csv" | head
