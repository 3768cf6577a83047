#!/bin/bash
# Round 4: address-translation counters of the chain kernel, C2 against C4
# (is C4's wide-level cost per item a UTCL1 miss cost?).  First the list of
# the counters this rocprofv3 offers, then one TCP pass per config.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4tlb; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 -L > $O/counters.txt 2>&1 || { tail -5 $O/counters.txt; exit 1; }
grep -o "UTCL[A-Z0-9_]*" $O/counters.txt | sort -u > $O/utcl.txt; cat $O/utcl.txt
for c in C2 C4; do
  timeout -s KILL 240 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_PERMISSION_MISS_sum TCP_UTCL1_REQUEST_sum \
    --kernel-trace --output-format csv -d $O/$c -o pmc -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --host-steps 0 --latency-steps 0 --config $c > $O/$c.json 2> $O/$c.err || { tail -5 $O/$c.err; exit 1; }
done
python3 - "$O" <<'PY'
import csv, glob, os, sys, collections
for c in ("C2", "C4"):
    f = glob.glob(os.path.join(sys.argv[1], c, "**", "*counter_collection.csv"), recursive=True)
    acc = collections.defaultdict(float); n = collections.Counter()
    for row in csv.DictReader(open(f[0])):
        if "chain_kernel" in row["Kernel_Name"]:
            acc[row["Counter_Name"]] += float(row["Counter_Value"]); n[row["Counter_Name"]] += 1
    print(c, {k: "%.4g" % (v / n[k]) for k, v in acc.items()})
PY
