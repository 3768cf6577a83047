#!/bin/bash
# Normalize's sqrt / reciprocal without the range-end steps (SC_SHORT_RN): full GPU suite on the product build, then A/B
O=gpurun_out/shortrn; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in base short; do
    SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/$v/libsurfcascade.so timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --latency-steps 10 --host-steps 0 > $O/$v.$r.json 2> $O/$v.$r.err || exit 1
    python -c "import json;d=json.load(open('$O/$v.$r.json'));print('$v', round(d['ms_per_step'],3), round(d['kernel_ms_per_launch']['windows'],3), round(d['latency_batch1']['ms_per_frame'],4))"
  done
done
for c in C5 C4; do for v in base short; do
  SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/$v/libsurfcascade.so timeout -k 10 200 python bench.py --config $c --steps 5 --warmup 1 --no-cpu --latency-steps 0 --host-steps 0 > $O/$v.$c.json 2> $O/$v.$c.err || exit 1
  python -c "import json;d=json.load(open('$O/$v.$c.json'));print('$v $c', round(d['ms_per_step'],3), round(d['kernel_ms_per_launch']['windows'],3))"
done; done
