#!/bin/bash
# speculative first batch for slots waiting on their entry: gpu suite, A/B vs base, phase counters
O=gpurun_out/spec; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 bash profiles/ab.sh $O/ab 3 base spec && python3 profiles/ab_report.py $O/ab || exit 1
SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/specp/libsurfcascade.so timeout -k 10 120 \
  python3 bench.py --steps 1 --warmup 0 --no-cpu --latency-steps 0 --host-steps 0 --opt profile=1 > $O/prof.json 2> $O/prof.err
grep SC_PROF $O/prof.err | tail -1
