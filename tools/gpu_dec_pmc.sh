set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/dpmc
for c in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_F64"; do
  tag=$(echo $c | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/dpmc/$tag -o run -- python3 tools/decider_bench.py > gpurun_out/dpmc/$tag.log 2>&1 || { tail -5 gpurun_out/dpmc/$tag.log; exit 1; }
done
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/dpmc/*/run_counter_collection.csv"):
    agg = {}
    for r in csv.DictReader(open(f)):
        if "decide" not in r["Kernel_Name"]: continue
        agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for k, v in agg.items(): print(k, len(v), v[-1])
PY
