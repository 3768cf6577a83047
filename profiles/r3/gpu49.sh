#!/bin/bash
# Round 3, call 49: the walkers' row carries with opaque lane ids in the
# walker block (the 12-wave hang of gpu46-48 gone): parity, then C2 A/B
# of carries fused (default) against walks only (integral_fuse=3).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g49
mkdir -p $O
cd $R
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for r in 1 2 3; do
  for v in rc w3; do
    X=""; [ $v == w3 ] && X="--opt integral_fuse=3"
    timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu --latency-steps 0 --host-steps 0 $X > $O/$v.$r.json 2> $O/$v.$r.err || { tail -5 $O/$v.$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/$v.$r.json')); print('$v', $r, d['ms_per_step'], d['value'])"
  done
done
