#!/bin/bash
# Round 3, call 16: entry words polled one round ahead (LDS DMA) vs blocking
# polls: parity, C2 and batch-1 A/B, phase counters.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g16
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
bash profiles/ab.sh gpurun_out/r3g16/c2 2 cur pa0 && \
  python3 profiles/ab_report_kernels.py gpurun_out/r3g16/c2 > $O/c2.txt && cat $O/c2.txt && \
bash profiles/ab.sh gpurun_out/r3g16/b1 2 cur pa0 -- --batch 1 --steps 50 && \
  python3 profiles/ab_report_kernels.py gpurun_out/r3g16/b1 > $O/b1.txt && cat $O/b1.txt || exit 1
export SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/prof/libsurfcascade.so
for b in 1 32; do
  timeout -k 10 200 python3 bench.py --steps 10 --warmup 0 --no-cpu --latency-steps 0 --host-steps 0 --batch $b --opt profile=1 > $O/p$b.json 2> $O/p$b.err || { tail -5 $O/p$b.err; exit 1; }
  grep SC_PROF_CHAIN $O/p$b.err | tail -1
done
