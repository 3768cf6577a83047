#!/bin/bash
# Quick PMC A/B of kernel variants: EA read requests, L2 hits/misses, VALU/VMEM counts.
#   bash profiles/pmc_variants.sh OUTDIR spec1 spec2 ... [-- bench args]
# spec: "variant" or "name|variant|ENV=1 ENV2=2" (variant: surfcascade_amd/lib/variants/<variant>)
OUT=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
V=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do V+=("$1"); shift; done
[ "$1" == "--" ] && shift
mkdir -p "$R/$OUT"
cd /tmp && export TMPDIR=/tmp
for spec in "${V[@]}"; do
  IFS='|' read -r name var envs <<< "$spec"
  [ -z "$var" ] && var=$name
  for grp in "TCC_EA0_RDREQ TCC_HIT TCC_MISS" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES" \
             "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
    tag=$(echo $grp | cut -c1-6)
    [ -n "$envs" ] && export $envs
    SURFCASCADE_LIB="$R/surfcascade_amd/lib/variants/$var/libsurfcascade.so" timeout -k 10 200 \
      rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$R/$OUT/$name.$tag" -o pmc \
      -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu "$@" > /dev/null 2>&1 || exit 1
    for e in $envs; do unset "${e%%=*}"; done
  done
done
