#!/bin/bash
# colsum with one lane per (column, channel), 48 rows of loads in flight: integral parity, then
# colscan (rowfull + colsum) ms per launch at 1 and 2 frames, interleaved vs base
O=gpurun_out/colsum4; mkdir -p $O
SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/c4/libsurfcascade.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "integral" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for v in base c4; do
    for b in 1 2; do
      SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/$v/libsurfcascade.so timeout -k 10 200 python3 bench.py --batch $b --steps 20 --warmup 3 --no-cpu --latency-steps 0 --host-steps 0 > $O/$v.b$b.$r.json 2> $O/$v.b$b.$r.err || { tail -3 $O/$v.b$b.$r.err; exit 1; }
    done
  done
done
python3 -c "
import json,glob
for v in ('base','c4'):
    for b in (1,2):
        xs=[json.load(open(f)) for f in sorted(glob.glob('$O/%s.b%d.*.json'%(v,b)))]
        print(v, b, 'colscan', [round(x['kernel_ms_per_launch']['colscan'],4) for x in xs], 'step', [round(x['ms_per_step'],4) for x in xs])
"
