#!/bin/bash
# Round 6, call i: speculative rounds per waiting task (SC_OPT_CHAIN_SPEC).
# Parity (speculation depth, one-frame grid shards at W = 2/4/8), the
# single-frame split measured rank by rank on one GPU (profiles/shard_balance.py:
# shards now speculate whole segments), and one frame per call at 1/2/4/64.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6i; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "speculat or shard" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python3 profiles/shard_balance.py --config C2 > $O/shard_c2.txt 2> $O/shard_c2.err || exit 1
tail -1 $O/shard_c2.txt > $O/shard_c2.json
timeout -k 10 300 python3 profiles/shard_balance.py --config C4 > $O/shard_c4.txt 2> $O/shard_c4.err || exit 1
tail -1 $O/shard_c4.txt > $O/shard_c4.json
bash profiles/ab_opts.sh $O/b1 3 s1:chain_spec=1 s2:chain_spec=2 s4:chain_spec=4 s64:chain_spec=64 -- --batch 1 --steps 200 || exit 1
python3 - <<'PY'
import glob, json, os, collections
for c in ("c2", "c4"):
    d = json.load(open("gpurun_out/r6i/shard_%s.json" % c))
    for w, v in d["worlds"].items():
        r = v["ranks"]
        print(c, w, "chain max %.4f" % max(x["chain_ms"] for x in r), "integral %.4f" % max(x["integral_ms"] for x in r),
              "eff %.3f" % v["implied_strong_efficiency"])
acc = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r6i/b1/*.json")):
    j = json.load(open(f))
    acc[os.path.basename(f).split(".")[0]].append((j["ms_per_step"], j["kernel_ms_per_launch"]["windows"]))
for v, xs in sorted(acc.items()):
    print("b1", v, ["%.4f/%.4f" % x for x in xs])
PY
