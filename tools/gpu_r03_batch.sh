# Batched small MSMs (f1): parity tests, then 128 x 64 terms with the quad-form Horner vs the old
# one-wave Horner, and a rocprof kernel-time split of the two batch kernels.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_msm_batch.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_batch.log 2>&1 || { tail -30 gpurun_out/pytest_batch.log; exit 1; }
tail -2 gpurun_out/pytest_batch.log
for q in 0 1; do
  SVGPU_BATCH_QUAD=$q timeout -k 10 120 python3 tools/batch_one.py > gpurun_out/batch_q$q.log 2>&1 || { cat gpurun_out/batch_q$q.log; exit 1; }
  echo "quad=$q $(tail -1 gpurun_out/batch_q$q.log)"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/batch -o run -- python3 tools/batch_one.py > gpurun_out/prof/batch.log 2>&1 || exit 1
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof/batch/run_kernel_stats.csv")))
for r in rows:
    print("%-60s calls %5s avg %9.1f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
