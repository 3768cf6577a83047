#!/bin/bash
# Round 4: C2 step with the detector on torch's stream (default) vs its own
# stream (event pair per call), and the build before the column-pass change
# (s2 = ebc6061) vs HEAD (cur); 3 interleaved runs.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r4streamab; mkdir -p $O; cd $R
B="python3 bench.py --no-cpu --host-steps 0 --latency-steps 0 --warmup 3 --steps 20"
for r in 1 2 3; do
  for v in "s2:torch" "cur:torch" "cur:own"; do
    lib=${v%%:*}; st=${v##*:}
    SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/$lib/libsurfcascade.so timeout -k 10 200 $B --detector-stream $st \
      > $O/${lib}_$st.$r.json 2> $O/${lib}_$st.$r.err || { tail -5 $O/${lib}_$st.$r.err; exit 1; }
  done
done
python3 - "$O" <<'PY'
import glob, json, os, statistics, sys, collections
res = collections.defaultdict(list)
for f in glob.glob(os.path.join(sys.argv[1], "*.json")):
    d = json.load(open(f)); res[os.path.basename(f).split(".")[0]].append((d["ms_per_step"], d["kernel_ms_per_launch"]["windows"]))
for k, v in sorted(res.items()):
    print("%-10s ms/step min %.3f med %.3f  chain min %.3f med %.3f" % (k, min(a for a, _ in v), statistics.median(a for a, _ in v), min(b for _, b in v), statistics.median(b for _, b in v)))
PY
