#!/bin/bash
# Round 3, call 29: bench without a host sync per step (N = 1), and a re-sweep
# of the row block on the fused kernel.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g29
mkdir -p $O
cd $R
timeout -k 10 300 python3 bench.py --no-cpu --host-steps 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-250 $O/bench.json
bash profiles/ab_opts.sh gpurun_out/r3g29/rb 2 rb32: rb24:row_block=24 rb48:row_block=48 rb16:row_block=16 && \
  python3 profiles/ab_report_kernels.py gpurun_out/r3g29/rb > $O/rb.txt && cat $O/rb.txt
export SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/prof/libsurfcascade.so
for b in 1 32; do
  timeout -k 10 200 python3 bench.py --steps 3 --warmup 0 --no-cpu --latency-steps 0 --host-steps 0 --batch $b --opt profile=1 > $O/p$b.json 2> $O/p$b.err || { tail -5 $O/p$b.err; exit 1; }
  grep SC_PROF_WAVES $O/p$b.err | tail -1
done
unset SURFCASCADE_LIB
bash profiles/ab.sh gpurun_out/r3g29/b1slots 2 cur s3 s3b64 -- --batch 1 --steps 50 && python3 profiles/ab_report_kernels.py gpurun_out/r3g29/b1slots > $O/b1slots.txt && cat $O/b1slots.txt
