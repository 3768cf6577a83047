#!/bin/bash
# item-stream check: gpu tests on the default build, interleaved A/B of the
# stage-synchronous (s0) and cross-stage stream (s1) chain kernels, then the
# item-schedule counters of both (SC_PROF_CHAIN builds)
O=gpurun_out/stream2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 bash profiles/ab.sh $O/ab 3 s0 s1 && python3 profiles/ab_report.py $O/ab || exit 1
for v in s0p s1p; do
  SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/$v/libsurfcascade.so timeout -k 10 120 \
    python3 bench.py --steps 1 --warmup 0 --no-cpu --latency-steps 0 --host-steps 0 --opt profile=1 \
    > $O/$v.json 2> $O/$v.err || exit 1
  echo $v; grep SC_PROF $O/$v.err | tail -1
done
