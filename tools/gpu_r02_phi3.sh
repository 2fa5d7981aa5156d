# MSM parity (incl. both GLV table layouts), 2^21 table-layout A/B, then the headline bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_host_path.py > gpurun_out/pytest_phi3.log 2>&1 || { tail -30 gpurun_out/pytest_phi3.log; exit 1; }
tail -1 gpurun_out/pytest_phi3.log
SVGPU_MSM_LEAN=1 timeout -k 10 200 python3 tools/msm_sweep_env.py 21 "SVGPU_GLV_PHI64=0" "SVGPU_GLV_PHI64=1" > gpurun_out/sweep_phi3.log 2>&1 || { tail -20 gpurun_out/sweep_phi3.log; exit 1; }
grep "2^" gpurun_out/sweep_phi3.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extras --config4-log-n 0 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms_per_step', round(d['ms_per_step'],4), d['breakdown_ms'], d['roofline']['kernel_avg_ms'])"
