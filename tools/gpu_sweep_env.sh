# MSM parity tests, then tools/msm_sweep_env.py over the given env specs.  Usage: bash tools/gpu_sweep_env.sh LOG_N SPEC...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_msm.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_sweep.log 2>&1 || { tail -30 gpurun_out/pytest_sweep.log; exit 1; }
tail -1 gpurun_out/pytest_sweep.log
timeout -k 10 400 python3 tools/msm_sweep_env.py "$@" > gpurun_out/sweep.log 2>&1; rc=$?
cat gpurun_out/sweep.log; exit $rc
