#!/bin/bash
# Round 6, call d: the lane-pair form with each item projected once (its
# offsets handed to the pair by DPP), chosen for frame tables > 128 MiB
# (variant pair) or for every frame (pairall).  Parity, A/B, counters.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6d; mkdir -p $O
SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/pairall/libsurfcascade.so timeout -k 10 400 \
  python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_soak.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "grid_parity or chain or spec or waves or soak or subq or shard or ped or permissive" > $O/pytest_pairall.log 2>&1 || { tail -30 $O/pytest_pairall.log; exit 1; }
tail -1 $O/pytest_pairall.log
SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/pair/libsurfcascade.so timeout -k 10 400 \
  python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "c4_bench_form or 4k or C4" > $O/pytest_pair_c4.log 2>&1 || { tail -30 $O/pytest_pair_c4.log; exit 1; }
tail -1 $O/pytest_pair_c4.log
bash profiles/ab.sh $O/c2 2 base pairall || exit 1
bash profiles/ab.sh $O/c4 3 base pair -- --config C4 || exit 1
bash profiles/pmc_variants.sh $O/pmc2 base pairall || exit 1
bash profiles/pmc_variants.sh $O/pmc4 pair -- --config C4 || exit 1
echo done
