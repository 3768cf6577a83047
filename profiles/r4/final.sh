#!/bin/bash
# Round 4 end-of-session evidence at HEAD: the GPU suite, smoke, the default
# bench line (C2, with the CPU baseline), C1 / C4 / C5 lines, the rocprofv3
# kernel-trace summary of the default command, PMC passes of C2 / C4 / C5
# (profiles/collect_pmc_cfg.sh, each stamped with the kernel sources' sha),
# the gather-ceiling calibration and its L2 hit / miss counts.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=gpurun_out/r4final; mkdir -p $R/$O; cd $R
bash profiles/run.sh r4final pytest smoke || exit 1
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench.json'));print('C2', d['value']/1e9, d['ms_per_step'], d['kernel_ms_per_launch'], d['latency_batch1']['ms_per_frame'], d.get('cpu_baseline',{}).get('value'))"
bash profiles/run.sh r4final "bench bench_C4 --config C4" "bench bench_C5 --config C5" "rocprof trace" calib || exit 1
timeout -k 10 300 python3 bench.py --config C1 > $O/bench_C1.json 2> $O/bench_C1.err || exit 1
for c in C2 C4 C5; do bash profiles/collect_pmc_cfg.sh $O/pmc/$c --config $c || exit 1; echo "pmc $c done"; done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv \
    -d $R/$O/calib_pmc -o pmc -- $R/profiles/calib/fetch_calib > $R/$O/calib_pmc.txt 2>&1 || exit 1
echo final done
# the LDS-DMA item variant (itembench V15) against the production item
bash profiles/run.sh r4final "itembench --reps 5 --variants 0:12,15:12,0:8,15:8" || exit 1
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE --kernel-trace \
    --output-format csv -d $R/$O/ib15_td -o pmc -- python3 $R/profiles/itembench/run.py --reps 1 --variants 0:12,15:12 \
    > $R/$O/ib15_td.txt 2>&1 || exit 1
echo ib15 done
