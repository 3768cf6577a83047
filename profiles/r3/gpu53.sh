#!/bin/bash
# Round 3, call 53: one-frame calls with the column pass inside the chain
# kernel (colsum walks published per 96-row band): parity, then one-frame
# A/B against the separate column pass (integral_fuse=1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g53
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "one_frame or fused or integral" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for r in 1 2 3; do
  for v in sep fused; do
    X=""; [ $v == sep ] && X="--opt integral_fuse=1"
    timeout -k 10 200 python3 bench.py --batch 1 --steps 60 --warmup 5 --no-cpu --latency-steps 60 --host-steps 0 $X > $O/$v.$r.json 2> $O/$v.$r.err || { tail -5 $O/$v.$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$v.$r.json')); k=d['kernel_ms_per_launch']; print('$v', $r, 'b1step %.4f' % d['ms_per_step'], 'lat %.4f' % d['latency_batch1']['ms_per_frame'], {a: round(b, 4) for a, b in k.items()})"
  done
done
