"""Average every counter of rocprofv3 --pmc CSV passes per dispatch for the kernels whose name contains a substring,
plus the derived MFMA-busy fraction per SIMD and the wave-cycle split (MI355X_MICROARCH.md "rocprofv3 PMC slots").

  python tools/pmc_summary.py KERNEL_SUBSTRING pass_dir [pass_dir ...] [--out file.json] [--simds 1024]
"""
import argparse, collections, csv, glob, json, os

ap = argparse.ArgumentParser()
ap.add_argument("kernel")
ap.add_argument("dirs", nargs="+")
ap.add_argument("--out")
ap.add_argument("--simds", type=int, default=1024)
a = ap.parse_args()
vals = collections.defaultdict(list)
for d in a.dirs:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if a.kernel in row.get("Kernel_Name", ""):
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
avg = {k: sum(v) / len(v) for k, v in sorted(vals.items())}
res = {"kernel": a.kernel, "dispatches": max((len(v) for v in vals.values()), default=0), "avg_per_dispatch": avg}
if "GRBM_GUI_ACTIVE" in avg:
    cyc = avg["GRBM_GUI_ACTIVE"] / 8.0  # summed over the 8 XCDs
    res["kernel_cycles"] = cyc
    if "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
        res["mfma_busy_frac_per_simd"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * a.simds)
w = avg.get("SQ_WAVE_CYCLES")
if w:
    res["wave_cycle_split"] = {k: avg[k] / w for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                                       "SQ_WAIT_INST_LDS") if k in avg}
print(json.dumps(res, indent=1))
if a.out:
    json.dump(res, open(a.out, "w"), indent=1)
