#!/bin/bash
# task records (3 or 4) separate from the 2 evaluation slots: gpu suite, A/B vs base, round counters
O=gpurun_out/tasks; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash profiles/ab.sh $O/ab 3 base t3 t4 && python3 profiles/ab_report.py $O/ab || exit 1
SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/t3p/libsurfcascade.so timeout -k 10 120 \
  python3 bench.py --steps 1 --warmup 0 --no-cpu --latency-steps 0 --host-steps 0 --opt profile=1 > $O/prof.json 2> $O/prof.err
grep SC_PROF $O/prof.err | tail -1
