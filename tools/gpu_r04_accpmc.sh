#!/bin/bash
# round 4: SQ counters of k_accumulate (29-bit chain with its point table) -- VALU instructions per entry
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
set -o pipefail
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES"
timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d gpurun_out/prof/acc_sq -o run -- python3 bench.py --no-extras --no-cpu-baseline --config4-log-n 0 --steps 5 --warmup 2 > gpurun_out/prof/acc_sq.log 2>&1 || exit 1
C2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD"
timeout -s KILL 150 rocprofv3 --pmc $C2 --output-format csv -d gpurun_out/prof/acc_sq2 -o run -- python3 bench.py --no-extras --no-cpu-baseline --config4-log-n 0 --steps 5 --warmup 2 > gpurun_out/prof/acc_sq2.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
for d in ["acc_sq", "acc_sq2"]:
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for fn in glob.glob(f"gpurun_out/prof/{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(fn)):
            k = r["Kernel_Name"]
            if not any(x in k for x in ("accumulate", "k_bin_hist", "k_bin_scatter", "k_fine_sort", "k_wsum_tree", "k_fixup", "k_group_fin")): continue
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[(k, r["Counter_Name"])] += 1
    for k, cs in acc.items():
        m = {c: v / n[(k, c)] for c, v in cs.items()}
        print(d, k[:50], {c: f"{v:.4g}" for c, v in sorted(m.items())})
PY
