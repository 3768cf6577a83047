#!/bin/bash
# chain slots per wave: 2 (base) vs 3 (128- and 64-window batches)
O=gpurun_out/slots3; mkdir -p $O
timeout -k 10 400 bash profiles/ab.sh $O/ab 2 base sl3 sl3b64 && python3 profiles/ab_report.py $O/ab
