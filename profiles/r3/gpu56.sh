#!/bin/bash
# Round 3, call 56: final evidence on HEAD: full GPU suite, smoke, the C2
# bench line (default command), its rocprofv3 kernel-trace summary, and the
# C5 line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g56
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
timeout -k 10 400 python3 bench.py --config C5 --no-cpu > $O/bench_C5.json 2> $O/bench_C5.err || { tail -20 $O/bench_C5.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o prof -- \
  python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --host-steps 0 > $O/prof_bench.json 2> $O/prof_bench.err || { tail -20 $O/prof_bench.err; exit 1; }
head -4 $O/prof/prof_kernel_stats.csv | cut -c1-160
