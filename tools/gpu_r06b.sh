# round 6: k_accumulate changes -- MSM parity tests, timing at 2^20 and 2^24, SQ VALU/SALU counts
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${R06B_TAG:-r06b}
mkdir -p $O
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -3 "$O/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "[$name] failed: stopping"; exit $rc; fi
}
run pytest 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_msm.py tests/test_gpu_host_path.py tests/test_gpu_msm_config4.py tests/test_gpu_crossover.py tests/test_gpu_decider.py
run sweep20 300 python3 tools/msm_sweep_env.py 20 SVGPU_GLV=1 SVGPU_GLV=1 SVGPU_GLV=1
run sweep24 300 python3 tools/msm_sweep_env.py 24 SVGPU_GLV=0
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --config4-log-n 0"
run sq_valu 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_VALU SQ_INSTS_SALU --output-format csv -d $O/sq_valu -o run -- python3 $B
python3 - "$O" <<'PY'
import csv, collections, glob, sys
f = glob.glob(f"{sys.argv[1]}/sq_valu/**/run_counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    if "k_accumulate" in r["Kernel_Name"]:
        acc[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    print(k, {c: "%.4g" % v for c, v in m.items()}, "VALU/entry-wave %.1f SALU/entry-wave %.1f" % (
        m["SQ_INSTS_VALU"] / (2**24 / 64), m["SQ_INSTS_SALU"] / (2**24 / 64)))
PY
