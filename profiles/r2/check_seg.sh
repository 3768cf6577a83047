#!/bin/bash
# segments per row: 8 (base) vs 4 / 2 (XCD pairs / quads, alternate rows per XCD)
O=gpurun_out/seg; mkdir -p $O
SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/seg4/libsurfcascade.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_seg4.log 2>&1; rc=$?
tail -2 $O/pytest_seg4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash profiles/ab.sh $O/ab 3 base seg4 seg2 && python3 profiles/ab_report.py $O/ab
