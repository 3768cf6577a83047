#!/bin/bash
# rowcarry carries collected in lanes, one coalesced store per 32 strips: integral parity, A/B rowscan ms
O=gpurun_out/rcacc; mkdir -p $O
SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/acc/libsurfcascade.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -k "integral" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for v in base acc; do
    for b in 32 1; do
      SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/$v/libsurfcascade.so timeout -k 10 200 python3 bench.py --batch $b --steps 10 --warmup 2 --no-cpu --latency-steps 0 --host-steps 0 > $O/$v.b$b.$r.json 2> $O/$v.b$b.$r.err || { tail -3 $O/$v.b$b.$r.err; exit 1; }
    done
  done
done
python3 -c "
import json,glob
for v in ('base','acc'):
    for b in (32,1):
        xs=[json.load(open(f))['kernel_ms_per_launch'] for f in sorted(glob.glob('$O/%s.b%d.*.json'%(v,b)))]
        print(v, b, 'rowscan', [round(x['rowscan'],4) for x in xs], 'colscan', [round(x['colscan'],4) for x in xs])
"
