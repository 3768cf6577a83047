#!/bin/bash
# Interleaved A/B timing of (library variant, environment) pairs.
#   bash profiles/ab_env.sh OUTDIR ROUNDS "name|variant|ENV=1 ENV2=2" ... [-- extra bench args]
# variant is a directory under surfcascade_amd/lib/variants (build_variants.sh).
OUT=$1; ROUNDS=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
V=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do V+=("$1"); shift; done
[ "$1" == "--" ] && shift
mkdir -p "$R/$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for spec in "${V[@]}"; do
    IFS='|' read -r name var envs <<< "$spec"
    env $envs SURFCASCADE_LIB="$R/surfcascade_amd/lib/variants/$var/libsurfcascade.so" \
      timeout -k 10 200 python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu "$@" \
      > "$R/$OUT/$name.$r.json" 2>/dev/null || exit 1
  done
done
