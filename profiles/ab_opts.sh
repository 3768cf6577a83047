#!/bin/bash
# Interleaved A/B timing of detector option sets on one build.
#   bash profiles/ab_opts.sh OUTDIR ROUNDS label:name=v,name=v ... [-- extra bench args]
# (label "base" with no options: "base:"); summary: profiles/ab_report_kernels.py OUTDIR
OUT=$1; ROUNDS=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
V=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do V+=("$1"); shift; done
[ "$1" == "--" ] && shift
mkdir -p "$R/$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for spec in "${V[@]}"; do
    lab=${spec%%:*}; opts=${spec#*:}; args=()
    IFS=, read -ra kv <<< "$opts"
    for o in "${kv[@]}"; do [ -n "$o" ] && args+=(--opt "$o"); done
    timeout -k 10 200 python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu --latency-steps 0 --host-steps 0 \
      "${args[@]}" "$@" > "$R/$OUT/$lab.$r.json" 2> "$R/$OUT/$lab.$r.err" || { tail -5 "$R/$OUT/$lab.$r.err"; exit 1; }
  done
done
