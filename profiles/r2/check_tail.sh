#!/bin/bash
# launch drain: the last rows (SC_TAIL_Q quarter frames) as 2-segment rows from a shared queue:
# parity with t4, then windows ms per launch at 32 and 8 frames, interleaved
O=gpurun_out/tail; mkdir -p $O
SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/t4/libsurfcascade.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for v in base t2 t4 t8; do
    for b in 32 8; do
      SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/$v/libsurfcascade.so timeout -k 10 200 python3 bench.py --batch $b --steps 8 --warmup 2 --no-cpu --latency-steps 0 --host-steps 0 > $O/$v.b$b.$r.json 2> $O/$v.b$b.$r.err || { tail -3 $O/$v.b$b.$r.err; exit 1; }
    done
  done
done
python3 -c "
import json,glob
for v in ('base','t2','t4','t8'):
    for b in (32,8):
        xs=[json.load(open(f))['kernel_ms_per_launch']['windows'] for f in sorted(glob.glob('$O/%s.b%d.*.json'%(v,b)))]
        print(v, b, [round(x,4) for x in xs])
"
