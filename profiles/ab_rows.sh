#!/bin/bash
# A/B of chain-kernel row orders on the default library, interleaved rounds:
#   bash profiles/ab_rows.sh OUTDIR ROUNDS "name:ENV=V ENV2=V2" ...
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/$1; ROUNDS=$2; shift 2; mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for spec in "$@"; do
    name=${spec%%:*}; envs=${spec#*:}
    env $envs timeout -k 10 200 python3 $R/bench.py --steps 10 --warmup 2 --no-cpu > $OUT/$name.$r.json 2>/dev/null || exit 1
  done
done
