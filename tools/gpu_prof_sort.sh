set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/psort
SWEEP_C=16 SWEEP_K=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/psort -o run -- python3 tools/msm_sweep.py 20,24 > gpurun_out/psort/log.txt 2>&1; rc=$?
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/psort/run_kernel_stats.csv")):
    print(r["Name"].split("(")[0][:60], r["Calls"], round(float(r["AverageNs"])/1e3,1), round(float(r["TotalDurationNs"])/1e6,3))
PY
exit $rc
