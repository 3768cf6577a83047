#!/bin/bash
# chain kernel at 16 waves per CU (128 VGPRs) vs 12
O=gpurun_out/w16; mkdir -p $O
timeout -k 10 300 bash profiles/ab.sh $O/ab 2 base w16 && python3 profiles/ab_report.py $O/ab
