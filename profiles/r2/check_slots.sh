#!/bin/bash
# chain kernel shapes with the item stream: slots x batch, result-ring size, table layout
O=gpurun_out/slots; mkdir -p $O
timeout -k 10 600 bash profiles/ab.sh $O/ab 3 s0 s1 s1b s1c s0b s1d && python3 profiles/ab_report.py $O/ab || exit 1
timeout -k 10 200 bash profiles/ab.sh $O/ab_tl 2 s0 s1 s1b -- --opt table_layout=1 && python3 profiles/ab_report.py $O/ab_tl
