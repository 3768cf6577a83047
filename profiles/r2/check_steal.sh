#!/bin/bash
# waves whose own task waits help segment 0 (SC_STEAL0): parity with the variant, then A/B vs base
O=gpurun_out/steal; mkdir -p $O
SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/steal/libsurfcascade.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash profiles/ab.sh $O/ab 3 base steal && python3 profiles/ab_report.py $O/ab
