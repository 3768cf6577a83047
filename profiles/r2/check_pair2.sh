#!/bin/bash
# paired-half loads: base vs pair (interleaved), pair build on the split table, pair at 8 waves/CU
O=gpurun_out/pair2; mkdir -p $O
timeout -k 10 300 bash profiles/ab.sh $O/ab 2 base pair pair8 && python3 profiles/ab_report.py $O/ab || exit 1
timeout -k 10 200 bash profiles/ab.sh $O/ab_split 2 base pair -- --opt table_layout=2 && python3 profiles/ab_report.py $O/ab_split
