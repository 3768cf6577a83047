#!/bin/bash
# the step's memsets folded into rowcarry: full gpu suite, then step / latency A/B vs HEAD's build
O=gpurun_out/zero; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for v in base new; do
    SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/$v/libsurfcascade.so timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --latency-steps 50 --host-steps 0 > $O/$v.$r.json 2> $O/$v.$r.err || { tail -3 $O/$v.$r.err; exit 1; }
  done
done
python3 -c "
import json,glob
for v in ('base','new'):
    xs=[json.load(open(f)) for f in sorted(glob.glob('$O/%s.*.json'%v))]
    print(v, 'step', [round(x['ms_per_step'],3) for x in xs], 'batch1', [round(x['latency_batch1']['ms_per_frame'],4) for x in xs])
"
