#!/bin/bash
# round 4: why the 29-bit chain wins in tools/ubench_madd29 but not in k_accumulate -- one SQ
# counter pass each over the microbenchmark and over bench.py with SVGPU_ACC_R29=1 / 0
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
set -o pipefail
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES"
timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/prof/r29_ub -o run -- ./tools/ubench_madd29 24 64 > gpurun_out/prof/r29_ub.log 2>&1 || exit 1
for v in 1 0; do
  SVGPU_ACC_R29=$v timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d gpurun_out/prof/r29_b$v -o run -- python3 bench.py --no-extras --no-cpu-baseline --config4-log-n 0 --steps 5 --warmup 2 > gpurun_out/prof/r29_b$v.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, collections
for d in ["r29_ub", "r29_b1", "r29_b0"]:
    f = glob.glob(f"gpurun_out/prof/{d}/**/*counter_collection.csv", recursive=True)
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for fn in f:
        for r in csv.DictReader(open(fn)):
            k = r["Kernel_Name"]
            if "accumulate" not in k and "k_r" not in k: continue
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[(k, r["Counter_Name"])] += 1
    for k, cs in acc.items():
        m = {c: v / n[(k, c)] for c, v in cs.items()}
        print(d, k[:60], {c: f"{v:.4g}" for c, v in sorted(m.items())})
PY
