#!/bin/bash
# SC_SPEC_FILL: a stage's idle item lanes evaluate the next stage's items (parity on the variant, then A/B)
O=gpurun_out/spec; mkdir -p $O
SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/spec/libsurfcascade.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in base spec; do
    SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/$v/libsurfcascade.so timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --latency-steps 10 --host-steps 0 > $O/$v.$r.json 2> $O/$v.$r.err || exit 1
    python -c "import json;d=json.load(open('$O/$v.$r.json'));print('$v', round(d['ms_per_step'],3), round(d['kernel_ms_per_launch']['windows'],3), round(d['latency_batch1']['ms_per_frame'],4))"
  done
done
for c in C5 C4; do for v in base spec; do
  SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/$v/libsurfcascade.so timeout -k 10 200 python bench.py --config $c --steps 5 --warmup 1 --no-cpu --latency-steps 0 --host-steps 0 > $O/$v.$c.json 2> $O/$v.$c.err || exit 1
  python -c "import json;d=json.load(open('$O/$v.$c.json'));print('$v $c', round(d['ms_per_step'],3), round(d['kernel_ms_per_launch']['windows'],3))"
done; done
