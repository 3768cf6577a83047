#!/bin/bash
# square-only waves skip corner slot 9: A/B against the round-2 base + VMEM counts
O=gpurun_out/sq; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 bash profiles/ab.sh $O/ab 3 base sq && python3 profiles/ab_report.py $O/ab || exit 1
timeout -k 10 300 bash profiles/pmc_variants.sh $O/pmc base sq -- --latency-steps 0 --host-steps 0 && python3 profiles/pmc_variants_report.py $O/pmc 16
