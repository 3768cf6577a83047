#!/bin/bash
# Round 6, call o: the single-frame split with one task per wave
# (SC_OPT_CHAIN_SLOTS 1: a speculative round for a second task no longer
# delays the first task's start), 4 and 8 segments per row; C2 and C4.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6o; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "shards_speculate" -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
for cfg in "C2 4" "C2 8" "C4 4"; do
  set -- $cfg
  timeout -k 10 300 python3 profiles/shard_balance.py --config $1 --opt chain_slots=1 --opt chain_segs=$2 \
    > $O/shard_$1_s$2.txt 2> $O/shard_$1_s$2.err || exit 1
  tail -1 $O/shard_$1_s$2.txt > $O/shard_$1_s$2.json
done
python3 - <<'PY'
import json
for n in ("C2_s4", "C2_s8", "C4_s4"):
    d = json.load(open("gpurun_out/r6o/shard_%s.json" % n))
    for w, v in d["worlds"].items():
        r = v["ranks"]
        print(n, w, "chain max %.4f" % max(x["chain_ms"] for x in r), "integral %.4f" % max(x["integral_ms"] for x in r),
              "eff %.3f" % v["implied_strong_efficiency"])
PY
