#!/bin/bash
# per-launch segment count (4 for one-frame launches): gpu suite, batch-1 and batch-32 timing
O=gpurun_out/segs; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for b in 1 2 32 1; do timeout -k 10 100 python3 bench.py --batch $b --steps 20 --warmup 3 --no-cpu --latency-steps 0 --host-steps 0 | python3 -c "import json,sys; j=json.load(sys.stdin); print($b, round(j['ms_per_step'],4), j['kernel_ms_per_launch'], round(j['value']/1e9,3))" || exit 1; done
