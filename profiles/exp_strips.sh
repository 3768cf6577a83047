cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in 0 24 40 72 136; do
  SC_VARIANT=$v timeout -k 10 120 python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --batch 8 > $R/gpurun_out/exp/t$v.json 2>/dev/null || exit 1
  SC_VARIANT=$v timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ TCC_HIT TCC_MISS --kernel-trace --output-format csv -d $R/gpurun_out/exp/p$v -o pmc -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --batch 8 > /dev/null 2>&1 || exit 1
done
