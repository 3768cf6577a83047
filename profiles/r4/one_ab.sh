#!/bin/bash
# Round 4: the one-launch one-frame integral (sc1 row loads) -- integral
# parity, one-frame A/B against the two-launch form; and the calibration
# kernels' L2 hit / miss counts (beyond-L2 ceilings from measured misses).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=gpurun_out/r4one2; mkdir -p $R/$O; cd $R
bash profiles/run.sh r4one2 "pytest tests/test_gpu_parity.py -k integral" \
    "abopt b1 3 base: two:integral_one=1 -- --batch 1 --steps 50" \
    "abopt c5 2 base: w14:chain_waves=14 -- --config C5" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv \
    -d $R/$O/calib_pmc -o pmc -- $R/profiles/calib/fetch_calib > $R/$O/calib_pmc.txt 2>&1 || exit 1
echo calib pmc done
