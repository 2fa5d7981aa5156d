# Round-3: the XCD-aware block map of k_bin_hist / k_bin_scatter -- MSM gpu tests, A/B bench lines,
# then one WRITE_SIZE pass per setting (HBM writes per launch of the sort kernels).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
bash tools/gpu_r03_iter.sh "test_gpu_msm or host_path or threads" "$@" || exit $?
for x in ${PMC_SET:-0 1}; do
  env ${PMC_VAR:-SVGPU_SORT_XCD}=$x timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/xcd_write$x -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --config4-log-n 0 > gpurun_out/prof/xcd_write$x.log 2>&1
  rc=$?; echo "[pmc write xcd=$x] rc=$rc"; [ $rc -ne 0 ] && exit $rc
  env ${PMC_VAR:-SVGPU_SORT_XCD}=$x timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/xcd_fetch$x -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --config4-log-n 0 > gpurun_out/prof/xcd_fetch$x.log 2>&1
  rc=$?; echo "[pmc fetch xcd=$x] rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 - <<'EOF'
import csv, glob, collections
for tag in ("write0", "write1", "fetch0", "fetch1"):
    fs = glob.glob(f"gpurun_out/prof/xcd_{tag}/**/*counter_collection.csv", recursive=True)
    acc = collections.defaultdict(list)
    for f in fs:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            for key in ("k_bin_hist", "k_bin_scatter", "k_bin_scan_chunks", "k_bin_scan_tiles", "k_fine_sort", "k_accumulate"):
                if key in k:
                    acc[key].append(float(r["Counter_Value"]))
    print(tag, {k: round(sum(v) / len(v)) for k, v in acc.items()})
EOF
