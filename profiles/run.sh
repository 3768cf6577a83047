#!/bin/bash
# The one GPU runner: a sequence of measurement steps, each under its own
# time limit, stopping at the first failure (no GPU step after a failed one).
# Run on the GPU box from the repo root, e.g.
#   gpurun -- 'bash profiles/run.sh r4x "pytest -k fused" "ab c2 3 old cur" "bench c4 --config C4"'
# Outputs go to gpurun_out/<OUT>/.  Steps (one quoted string each):
#   pytest [pytest args]          the GPU suite (-m gpu), or a subset (PYTEST_K="a or b": a -k
#                                 expression with spaces, which the step string cannot carry)
#   smoke                         __graft_entry__.smoke()
#   bench NAME [bench.py args]    one bench line -> NAME.json
#   ab DIR ROUNDS V... [-- args]  interleaved A/B of library variants (profiles/build_variants.sh
#                                 builds them in this container) -> DIR/, summary DIR.txt
#   abopt DIR ROUNDS L:o=v,... [-- args]  the same for detector option sets on one build
#   rocprof NAME [bench args]     rocprofv3 --kernel-trace --stats of a bench run -> NAME/
#   pmc DIR [bench args]          the PMC passes (profiles/collect_pmc_cfg.sh) -> DIR/
#   calib                         profiles/calib/fetch_calib (counter calibration, gather ceilings)
#   itembench [run.py args]       profiles/itembench/run.py (the item loop alone)
#   lib NAME                      use surfcascade_amd/lib/variants/NAME for the following steps
set -o pipefail
OUT=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=gpurun_out/$OUT
mkdir -p "$R/$O"
cd "$R" || exit 1
BENCH="python3 $R/bench.py --no-cpu --host-steps 0"
step() {
  local kind=$1; shift
  case "$kind" in
    pytest)
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        ${PYTEST_K:+-k "$PYTEST_K"} "$@" \
        > "$O/pytest.log" 2>&1; local rc=$?; tail -3 "$O/pytest.log"; return $rc ;;
    smoke)
      timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 && cat "$O/smoke.log" ;;
    bench)
      local n=$1; shift
      timeout -k 10 400 $BENCH "$@" > "$O/$n.json" 2> "$O/$n.err" || { tail -5 "$O/$n.err"; return 1; }
      python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], '%.4g G windows/s'%(d['value']/1e9), d['ms_per_step'], d['kernel_ms_per_launch'])" "$O/$n.json" ;;
    ab)
      local d=$1; shift
      bash profiles/ab.sh "$O/$d" "$@" && python3 profiles/ab_report_kernels.py "$O/$d" | tee "$O/$d.txt" ;;
    abopt)
      local d=$1; shift
      bash profiles/ab_opts.sh "$O/$d" "$@" && python3 profiles/ab_report_kernels.py "$O/$d" | tee "$O/$d.txt" ;;
    rocprof)
      local n=$1; shift
      ( cd /tmp && export TMPDIR=/tmp &&
        timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/$n" -o trace \
          -- python3 "$R/bench.py" --no-cpu --latency-steps 0 --host-steps 0 "$@" \
          > "$R/$O/$n.json" 2> "$R/$O/$n.err" ) && head -5 "$O/$n/trace_kernel_stats.csv" ;;
    pmc)
      local d=$1; shift
      bash profiles/collect_pmc_cfg.sh "$O/$d" "$@" ;;
    calib)
      timeout -k 10 180 profiles/calib/fetch_calib > "$O/calib.txt" 2>&1 && cat "$O/calib.txt" ;;
    itembench)
      timeout -k 10 300 python3 -u profiles/itembench/run.py "$@" > "$O/itembench.txt" 2>&1; local rc=$?
      grep -E "variant|items" "$O/itembench.txt"; return $rc ;;
    lib)
      export SURFCASCADE_LIB="$R/surfcascade_amd/lib/variants/$1/libsurfcascade.so"; echo "library $1" ;;
    *)
      echo "unknown step: $kind"; return 2 ;;
  esac
}
for s in "$@"; do
  echo "== $s"
  # shellcheck disable=SC2086
  step $s || { echo "step failed: $s"; exit 1; }
done
