#!/bin/bash
# Interleaved A/B timing of kernel variants built by build_variants.sh.
#   bash profiles/ab.sh OUTDIR ROUNDS v0 v1 ... [-- extra bench args]
OUT=$1; ROUNDS=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
V=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do V+=("$1"); shift; done
[ "$1" == "--" ] && shift
mkdir -p "$R/$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for v in "${V[@]}"; do
    SURFCASCADE_LIB="$R/surfcascade_amd/lib/variants/$v/libsurfcascade.so" timeout -k 10 200 \
      python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu --latency-steps 0 --host-steps 0 "$@" > "$R/$OUT/$v.$r.json" 2> "$R/$OUT/$v.$r.err" || { tail -5 "$R/$OUT/$v.$r.err"; exit 1; }
  done
done
