# MSM tests + bench (no CPU baseline, no extras) + kernel trace gaps of one step
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batch.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_q2.log 2>&1 || { tail -30 gpurun_out/pytest_q2.log; exit 1; }
tail -1 gpurun_out/pytest_q2.log
for i in 1 2; do
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extras --config4-log-n 0 > gpurun_out/bench_q2.log 2>&1 || { tail -5 gpurun_out/bench_q2.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_q2.log').read().strip().splitlines()[-1]);print('msm ms',d['ms_per_step'],d['breakdown_ms'], 'acc frac', d['int_mac']['kernel_frac'])"
done
