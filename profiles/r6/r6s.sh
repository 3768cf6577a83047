#!/bin/bash
# Round 6, call s: one-frame grid shards of 8 ranks on 8 segments per row
# (auto): shard parity, the split rank by rank (C2, C4), and 300 random
# parity cases with task slots and speculation depth among the drawn options.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6s; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "shards_speculate or one_frame or segments" -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in C2 C4; do
  timeout -k 10 300 python3 profiles/shard_balance.py --config $c > $O/shard_$c.txt 2> $O/shard_$c.err || exit 1
  tail -1 $O/shard_$c.txt > $O/shard_$c.json
done
python3 - <<'PY'
import json
for n in ("C2", "C4"):
    d = json.load(open("gpurun_out/r6s/shard_%s.json" % n))
    for w, v in d["worlds"].items():
        r = v["ranks"]
        print(n, w, "chain max %.4f" % max(x["chain_ms"] for x in r), "integral %.4f" % max(x["integral_ms"] for x in r),
              "eff %.3f" % v["implied_strong_efficiency"])
PY
timeout -k 10 600 python3 -u tests/soak_parity.py --cases 300 --seed 27000 --out $O/soak_27000.json > $O/soak_27000.log 2>&1; rc=$?
tail -2 $O/soak_27000.log | cut -c1-300
[ $rc -eq 0 ]
