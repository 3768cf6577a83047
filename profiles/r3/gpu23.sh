#!/bin/bash
# Round 3, call 23: item results stored in item order (inverse shape-order
# table for the k-order sum) vs the previous commit: parity, C2 / C5 A/B, and
# the LDS bank-conflict counters of both.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g23
mkdir -p $O
cd $R
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_mine.py tests/test_gpu_configs.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
bash profiles/ab.sh gpurun_out/r3g23/c2 2 old cur && python3 profiles/ab_report_kernels.py gpurun_out/r3g23/c2 > $O/c2.txt && cat $O/c2.txt || exit 1
bash profiles/ab.sh gpurun_out/r3g23/c5 2 old cur -- --config C5 && python3 profiles/ab_report_kernels.py gpurun_out/r3g23/c5 > $O/c5.txt && cat $O/c5.txt || exit 1
cd /tmp && export TMPDIR=/tmp
for v in old cur; do for c in C2 C5; do
  SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/$v/libsurfcascade.so timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS --kernel-trace --output-format csv -d $O/lds_${v}_$c -o pmc -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --host-steps 0 --latency-steps 0 --config $c > $O/lds_${v}_$c.json 2> $O/lds_${v}_$c.err || exit 1
done; done
echo lds ok
