# round 6: k_accumulate restructured loop -- parity tests, A/B timing, SQ VALU counts (both loops)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -3 "$O/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "[$name] failed: stopping"; exit $rc; fi
}
run pytest 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_msm.py tests/test_gpu_host_path.py tests/test_gpu_msm_config4.py tests/test_gpu_crossover.py
run sweep 300 python3 tools/msm_sweep_env.py 20 SVGPU_ACC_LOOP=0 SVGPU_ACC_LOOP=1 SVGPU_ACC_LOOP=0 SVGPU_ACC_LOOP=1
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --config4-log-n 0"
for L in 0 1; do
  SVGPU_ACC_LOOP=$L run sq_valu_$L 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_VALU SQ_INSTS_SALU --output-format csv -d $O/sq_valu_$L -o run -- python3 $B
done
python3 - <<'PY'
import csv, collections, glob
for L in (0, 1):
    f = glob.glob(f"gpurun_out/r06b/sq_valu_{L}/**/run_counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].find("k_accumulate") >= 0:
            acc[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in acc.items():
        m = {c: sum(v) / len(v) for c, v in d.items()}
        print(L, k, {c: "%.4g" % v for c, v in m.items()}, "VALU/entry-wave %.1f" % (m["SQ_INSTS_VALU"] / (2**24 / 64)))
PY
