#!/bin/bash
# Round 4: rowcarry4 with its R rows staged through LDS and stored one
# phase-plane run per instruction (SC_RC_LDS): integral parity on that build,
# then one-frame and C2 A/B against the product build.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=gpurun_out/r4rclds; mkdir -p $R/$O; cd $R
SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/rclds/libsurfcascade.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "integral or segments or fused or c5_bench or batch" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash profiles/run.sh r4rclds "ab b1 4 cur rclds -- --batch 1 --steps 50" "ab c2 3 cur rclds"
