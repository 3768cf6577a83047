#!/bin/bash
# slot-9 skip (all-2x2 item instructions issue 18 corner loads, not 20): parity on the variant, then A/B
O=gpurun_out/skip9; mkdir -p $O
SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/skip9/libsurfcascade.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_mine.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in base skip9; do
    SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/$v/libsurfcascade.so timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --latency-steps 10 --host-steps 0 > $O/$v.$r.json 2> $O/$v.$r.err || exit 1
    python -c "import json;d=json.load(open('$O/$v.$r.json'));print('$v', round(d['ms_per_step'],3), round(d['kernel_ms_per_launch']['windows'],3), round(d['latency_batch1']['ms_per_frame'],4))"
  done
done
for v in base skip9; do
  SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/$v/libsurfcascade.so timeout -k 10 200 python bench.py --config C5 --steps 5 --warmup 1 --no-cpu --latency-steps 0 --host-steps 0 > $O/$v.C5.json 2> $O/$v.C5.err || exit 1
  python -c "import json;d=json.load(open('$O/$v.C5.json'));print('$v C5', round(d['ms_per_step'],3), round(d['kernel_ms_per_launch']['windows'],3))"
done
