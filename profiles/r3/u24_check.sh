set -o pipefail
mkdir -p gpurun_out/u1
timeout -k 10 300 python -u -m pytest tests/test_gpu_u24.py -x -v --timeout 120 --timeout-method thread > gpurun_out/u1/pytest.log 2>&1; rc=$?
tail -15 gpurun_out/u1/pytest.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for u in 1 2; do
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --latency-steps 0 --host-steps 0 --opt integral_fuse=1 --opt table_u24=$u > gpurun_out/u1/b$u.$r.json 2> gpurun_out/u1/b$u.$r.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/u1/b$u.$r.json'));print('u24=$u', d['ms_per_step'], d['kernel_ms_per_launch'], d['value']/1e9)"
done; done
