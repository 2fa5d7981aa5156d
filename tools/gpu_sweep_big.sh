# MSM tests, then tools/msm_sweep_env.py at 2^20, 2^21 and 2^24 (default settings + given specs).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_msm.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_sweep.log 2>&1 || { tail -30 gpurun_out/pytest_sweep.log; exit 1; }
tail -1 gpurun_out/pytest_sweep.log
for L in 20 21 24; do
  timeout -k 10 300 python3 tools/msm_sweep_env.py $L SVGPU_GLV=0 "$@" > gpurun_out/sweep$L.log 2>&1; rc=$?
  grep "2^" gpurun_out/sweep$L.log; [ $rc -ne 0 ] && { tail gpurun_out/sweep$L.log; exit $rc; }
done
exit 0
