#!/bin/bash
# paired-half loads in the chain kernel: full gpu suite, then A/B against the round-2 base
O=gpurun_out/pair; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 bash profiles/ab.sh $O/ab 3 base pair && python3 profiles/ab_report.py $O/ab
