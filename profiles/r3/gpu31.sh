#!/bin/bash
# Round 3, call 31: idle waves of the 12-wave chain kernel evaluate a waiting
# task's first windows (both parities) ahead of its entry: parity, one-frame
# and C5 A/B, one-frame wave timeline.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g31
mkdir -p $O
cd $R
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
bash profiles/ab.sh gpurun_out/r3g31/b1 3 old cur -- --batch 1 --steps 50 && python3 profiles/ab_report_kernels.py gpurun_out/r3g31/b1 > $O/b1.txt && cat $O/b1.txt || exit 1
bash profiles/ab.sh gpurun_out/r3g31/c5 2 old cur -- --config C5 && python3 profiles/ab_report_kernels.py gpurun_out/r3g31/c5 > $O/c5.txt && cat $O/c5.txt || exit 1
export SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/prof/libsurfcascade.so
timeout -k 10 200 python3 bench.py --steps 3 --warmup 0 --no-cpu --latency-steps 0 --host-steps 0 --batch 1 --opt profile=1 > $O/p1.json 2> $O/p1.err || { tail -5 $O/p1.err; exit 1; }
grep SC_PROF $O/p1.err | tail -2
