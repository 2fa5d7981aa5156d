"""Summarise a rocprofv3 run (tools/profile_*.sh) into profiles/: kernel-stats table + PMC HBM bytes.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  gfx950 correction (MI355X_MICROARCH.md, HBM):
FETCH_SIZE reads exactly half the bytes of wide (16 B/lane) coalesced streaming reads.  That x2 is
applied only to kernels that stream; k_accumulate gathers 64-B points at random and gets the factor
calibrated on that pattern (tools/calib_fetch.hip, ~1.05 from a 64 MiB table) -- the same factor
profiles/pmc_accumulate.json and bench.py's roofline.traffic use.  Each row names its factor.
usage: python3 tools/summarize_profile.py gpurun_out/prof profiles r02
"""
import csv
import json
import os
import sys
from collections import defaultdict

src, dst, tag = sys.argv[1], sys.argv[2], sys.argv[3]
os.makedirs(dst, exist_ok=True)


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "").replace("sv::", "")
    return name.split("(")[0]


rows = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
total = sum(float(r["TotalDurationNs"]) for r in rows)
lines = [f"# rocprofv3 --kernel-trace --stats, bench.py --steps 10 --warmup 2 ({tag})", "",
         "| kernel | calls | avg us | total ms | % |", "|---|---|---|---|---|"]
for r in rows:
    lines.append("| %s | %s | %.1f | %.3f | %.1f |" % (short(r["Name"]), r["Calls"], float(r["AverageNs"]) / 1e3,
                                                       float(r["TotalDurationNs"]) / 1e6, float(r["Percentage"])))
ex = os.path.join(src, "trace_extras", "run_kernel_stats.csv")
if os.path.exists(ex):
    lines += ["", "## bench.py with the next-row extras (batched MSMs, config-5 aggregation, Poseidon)", "",
              "| kernel | calls | avg us | total ms | % |", "|---|---|---|---|---|"]
    for r in csv.DictReader(open(ex)):
        lines.append("| %s | %s | %.1f | %.3f | %.1f |" % (short(r["Name"]), r["Calls"], float(r["AverageNs"]) / 1e3,
                                                           float(r["TotalDurationNs"]) / 1e6, float(r["Percentage"])))
pmc = {}
for counter, sub in (("FETCH_SIZE", "pmc_fetch"), ("WRITE_SIZE", "pmc_write")):
    acc = defaultdict(list)
    for r in csv.DictReader(open(os.path.join(src, sub, "run_counter_collection.csv"))):
        acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    pmc[counter] = {k: sum(v) / len(v) for k, v in acc.items()}
# FETCH_SIZE calibration (tools/calib_fetch.hip): known bytes / FETCH_SIZE bytes per kernel dispatch
calib = {}
cal_csv = os.path.join(src, "pmc_calib", "run_counter_collection.csv")
if os.path.exists(cal_csv):
    known = {"gather64_64MiB": 1048576 * 16 * 64, "gather64_1GiB": 1048576 * 16 * 64, "stream16": 256 << 20}
    rows_c = [r for r in csv.DictReader(open(cal_csv)) if short(r["Kernel_Name"]) in ("k_gather64", "k_stream")]
    rows_c.sort(key=lambda r: int(r["Dispatch_Id"]))
    names = [n for n, r in zip(("gather64_64MiB", "gather64_1GiB"), [r for r in rows_c if short(r["Kernel_Name"]) == "k_gather64"])]
    names += ["stream16"] if any(short(r["Kernel_Name"]) == "k_stream" for r in rows_c) else []
    for name, r in zip(names, rows_c):
        v = float(r["Counter_Value"])
        calib[name] = {"fetch_kib": v, "known_bytes": known[name], "factor": known[name] / (v * 1024) if v else None}
    lines += ["", "## FETCH_SIZE calibration (tools/calib_fetch.hip, known byte counts)", "",
              "| pattern | FETCH_SIZE KiB | known MB | factor (known / FETCH_SIZE) |", "|---|---|---|---|"]
    for k, v in calib.items():
        lines.append("| %s | %.0f | %.1f | %.3f |" % (k, v["fetch_kib"], v["known_bytes"] / 1e6, v["factor"] or 0))
GATHER_KERNELS = ("k_accumulate",)  # random 64-B point gathers (bucket entries in sorted order)


def read_factor(kernel):
    """(factor, basis) for FETCH_SIZE of one kernel: the gather calibration for the gathering
    kernels, the guide's streaming x2 (or its calibrated value) for the rest."""
    if kernel.startswith(GATHER_KERNELS):
        g = calib.get("gather64_64MiB", {}).get("factor")
        return (g, "gather64 calibrated") if g else (1.05, "gather64 (round-2 calibration)")
    st = calib.get("stream16", {}).get("factor")
    return (st, "stream16 calibrated") if st else (2.0, "streaming x2 (guide)")


lines += ["", "## HBM traffic per launch (PMC, separate passes)", "",
          "| kernel | FETCH_SIZE KiB (raw) | read factor | basis | reads MB | WRITE_SIZE KiB | MB total |",
          "|---|---|---|---|---|---|---|"]
for k in sorted(pmc["FETCH_SIZE"], key=lambda k: -pmc["FETCH_SIZE"][k]):
    f = pmc["FETCH_SIZE"][k]
    w = pmc["WRITE_SIZE"].get(k, 0.0)
    fac, basis = read_factor(k)
    lines.append("| %s | %.0f | %.3f | %s | %.1f | %.0f | %.1f |" % (k, f, fac, basis, fac * f * 1024 / 1e6, w,
                                                                   (fac * f + w) * 1024 / 1e6))
# SQ instruction / cycle counters (round 5: sq_valu, sq_wait passes), per dispatch, for the two
# dominant kernels; per-wave figures divide by SQ_WAVES
sq = {}
for sub in ("sq_valu", "sq_wait"):
    f = os.path.join(src, sub, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(f)):
        acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in acc.items():
        sq.setdefault(k, {}).update({c: sum(v) / len(v) for c, v in d.items()})
if sq:
    lines += ["", "## SQ counters per dispatch (separate --pmc passes; chip totals, per wave = / SQ_WAVES)", ""]
    for k in [k for k in sq if k.startswith("k_accumulate") or k.startswith("k_decide_wg")]:
        d = sq[k]
        waves = d.get("SQ_WAVES", 0) or 1
        lines += ["### " + k, "", "| counter | per dispatch | per wave |", "|---|---|---|"]
        for c in sorted(d):
            lines.append("| %s | %.4g | %.4g |" % (c, d[c], d[c] / waves))
        lines.append("")
    json.dump(sq, open(os.path.join(dst, f"{tag}_sq_counters.json"), "w"), indent=1)
open(os.path.join(dst, f"{tag}_kernel_stats.md"), "w").write("\n".join(lines) + "\n")
acc_key = next((k for k in pmc["FETCH_SIZE"] if k.startswith("k_accumulate")), None)  # k_accumulate<false> since r03
acc_f = pmc["FETCH_SIZE"].get(acc_key) if acc_key else None
acc_w = pmc["WRITE_SIZE"].get(acc_key) if acc_key else None
if acc_f is not None:
    g = calib.get("gather64_64MiB", {}).get("factor")
    factor = read_factor(acc_key)[0]
    json.dump({"kernel": "k_accumulate", "source": f"profiles/{tag}_kernel_stats.md",
               "fetch_kib_raw": acc_f, "write_kib": acc_w, "read_factor": factor,
               "hbm_bytes_per_launch": (factor * acc_f + (acc_w or 0)) * 1024,
               "correction": "reads scaled by the factor calibrated on k_accumulate's own access pattern "
                             "(random 64-B gathers from a 64 MiB table, tools/calib_fetch.hip) -- the "
                             "MI355X_MICROARCH.md HBM note calibrates only 16-B streaming reads (x2)"
                             if g else "reads x1.05, the round-2 gather calibration (no calibration pass in this run)"},
              open(os.path.join(dst, "pmc_accumulate.json"), "w"), indent=1)
print("\n".join(lines))
