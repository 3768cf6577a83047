#!/bin/bash
# Round 4: the LDS-path ceiling of the item loop (itembench V14: every corner
# an LDS read, no staging cost) against the production item (V0) and the
# L2-resident fold ablation (V3), at 12 and 16 waves; PMC of V0 / V14; and the
# 1-KiB-row gather-into-LDS ceilings (profiles/calib k_rows_*).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r4lds; mkdir -p $O; cd $R
timeout -k 10 200 python3 -u profiles/itembench/run.py --reps 5 --variants 0:12,14:12,0:16,14:16,3:16 --fold 0x7f \
    --out $O/ib.json > $O/ib.txt 2>&1 || exit 1
cat $O/ib.txt
timeout -k 10 120 profiles/calib/fetch_calib > $O/calib.txt 2>&1 || exit 1
grep k_rows $O/calib.txt
cd /tmp && export TMPDIR=/tmp
for v in 0:16 14:16; do
  n=${v/:/_}
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
     --kernel-trace --output-format csv -d $O/pmc_sq_$n -o pmc -- python3 $R/profiles/itembench/run.py --reps 1 --variants $v > $O/pmc_sq_$n.txt 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE \
     --kernel-trace --output-format csv -d $O/pmc_td_$n -o pmc -- python3 $R/profiles/itembench/run.py --reps 1 --variants $v > $O/pmc_td_$n.txt 2>&1 || exit 1
done
echo done
