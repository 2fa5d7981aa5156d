# Counter passes over the f1 batch kernels (128 x 64 terms): VALU instructions, wave cycles, waits.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS --output-format csv -d gpurun_out/prof/batch_pmc -o run -- python3 tools/batch_one.py > gpurun_out/prof/batch_pmc.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
rows = list(csv.DictReader(open(glob.glob("gpurun_out/prof/batch_pmc/*counter_collection.csv")[0])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    agg[r["Kernel_Name"].split("(")[0][-40:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "batch" in k or "horner" in k:
        print(k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
