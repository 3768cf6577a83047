#!/bin/bash
# Round 3, call 4: parity suite on the 16-wave product build, the bench line
# with a rocprofv3 kernel trace, and the chain kernel's phase profile
# (SC_PROF_CHAIN build) at 16 and 12 waves.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g4
mkdir -p $O
cd $R
echo "pytest" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
echo "bench" && timeout -k 10 300 python3 bench.py --cpu-seconds 5 > $O/bench.json 2> $O/bench.err && cat $O/bench.json | head -c 600 && echo &&
echo "trace" && (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 10 --no-cpu --host-steps 0 --latency-steps 0 > $O/trace.log 2>&1) &&
echo "prof" && for w in 16 12; do SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/prof/libsurfcascade.so timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu --host-steps 0 --latency-steps 0 --opt profile=1 --opt chain_waves=$w > $O/prof$w.json 2> $O/prof$w.err || exit 1; grep SC_PROF $O/prof$w.err | tail -1; done
