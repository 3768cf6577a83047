#!/bin/bash
# Round 3, call 3: 16- vs 12-wave chain kernel in the product build, the
# interleaved 32-B cell layout (big levels are fabric-bound), C4 / C5.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g3
mkdir -p $O
cd $R
B="--steps 10 --warmup 2 --no-cpu --latency-steps 0 --host-steps 0"
run() { local n=$1; shift; timeout -k 10 200 python3 bench.py $B "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }; }
for r in 1 2; do
  run w16.$r && run w12.$r --opt chain_waves=12 && run il.$r --opt table_layout=1 && run il12.$r --opt table_layout=1 --opt chain_waves=12 || exit 1
done
echo "split" && timeout -k 10 300 python3 profiles/level_split.py --opt table_layout=1 > $O/split_il.json 2> $O/split_il.err &&
timeout -k 10 300 python3 profiles/level_split.py > $O/split.json 2> $O/split.err &&
run c4 --config C4 && run c5 --config C5 && run c4w12 --config C4 --opt chain_waves=12 &&
python3 - <<PY
import json,glob,os
for f in sorted(glob.glob("$O/*.json")):
    for l in open(f):
        d=json.loads(l)
        if "value" in d: print(os.path.basename(f), "%.3f Gwin/s" % (d["value"]/1e9), "chain %.3f ms" % d["kernel_ms_per_launch"]["windows"])
        elif "levels" in d: print(os.path.basename(f), d["levels"], "%.3f ms" % d["chain_ms"], "%.4f ns/win" % d["ns_per_grid_window"])
PY
