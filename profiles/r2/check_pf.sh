#!/bin/bash
# next task prefetched during a round (SC_PREFETCH): parity with the variant, then A/B vs base
O=gpurun_out/pf; mkdir -p $O
SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/pf/libsurfcascade.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash profiles/ab.sh $O/ab 3 base pf && python3 profiles/ab_report.py $O/ab
