#!/bin/bash
# Round 3, call 51: colsum in table order (lane = cell x channel, whole
# lines per access) against colsum4: integral parity, then one-frame and
# C2 A/B (kernel times per launch from the bench line).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g51
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "integral" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for r in 1 2 3; do
  for v in cs4 pl; do
    SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/$v/libsurfcascade.so timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --latency-steps 40 --host-steps 0 > $O/$v.$r.json 2> $O/$v.$r.err || { tail -5 $O/$v.$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$v.$r.json')); k=d['kernel_ms_per_launch']; print('$v', $r, 'step %.3f' % d['ms_per_step'], 'colscan %.4f' % k['colscan'], 'b1 %.4f' % d['latency_batch1']['ms_per_frame'])"
  done
done
for v in cs4 pl; do
  SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/$v/libsurfcascade.so timeout -k 10 200 python3 bench.py --batch 1 --steps 40 --warmup 5 --no-cpu --latency-steps 0 --host-steps 0 > $O/$v.b1.json 2> $O/$v.b1.err || { tail -5 $O/$v.b1.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$v.b1.json')); print('$v batch1', d['ms_per_step'], d['kernel_ms_per_launch'])"
done
