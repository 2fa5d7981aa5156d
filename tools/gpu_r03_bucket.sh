# f1 bucket-wise Horner: batch parity tests, 128 x 64 per path (per-window / two kernels / fused), rocprof split.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_msm_batch.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_batch.log 2>&1 || { tail -30 gpurun_out/pytest_batch.log; exit 1; }
tail -2 gpurun_out/pytest_batch.log
for q in "SVGPU_BATCH_BUCKETS=0" "SVGPU_BATCH_FUSE=0" "SVGPU_BATCH_BW=2" "SVGPU_BATCH_BW=3" "SVGPU_BATCH_BW=4" "SVGPU_BATCH_BW=6" "SVGPU_BATCH_BW=9" "SVGPU_BATCH_BW=26"; do
  env $q timeout -k 10 120 python3 tools/batch_one.py > gpurun_out/batch_b.log 2>&1 || { cat gpurun_out/batch_b.log; exit 1; }
  echo "$q $(tail -1 gpurun_out/batch_b.log)"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/batchb -o run -- python3 tools/batch_one.py > gpurun_out/prof/batchb.log 2>&1 || exit 1
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof/batchb/run_kernel_stats.csv")))
for r in rows:
    print("%-60s calls %5s avg %9.1f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
