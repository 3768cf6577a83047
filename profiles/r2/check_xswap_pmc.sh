#!/bin/bash
# TCP / TD / SQ / TCC counters of the item-loop variants V0 (production) and V12 (paired-half loads)
V=0:12,12:12,13:12 ONLY1=1 timeout -k 10 400 bash profiles/itembench/ib_pmc.sh && python3 profiles/itembench/ib_pmc_report.py gpurun_out/ibpmc
