"""MFMA utilisation of the Cholesky launches from a rocprofv3 --pmc pass (north star: "MFMA utilisation on the trailing
update").  Each factorisation at n = 64 nblk is nblk potrf_step_kernel dispatches (launch c = block column c); the
counters are per dispatch, so early launches (trailing-update-dominated: ~(nblk-c)^2/8 128x128 tiles beside the panel)
and late ones (panel-dominated) are reported apart.
usage: python tools/pmc_potrf.py PASS_DIR NBLK out.json"""
import csv, glob, json, os, sys
d, nblk, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
rows = {}
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "potrf_step_kernel" not in r.get("Kernel_Name", ""):
            continue
        key = int(r.get("Dispatch_Id", r.get("Correlation_Id", 0)))
        rows.setdefault(key, {})[r["Counter_Name"]] = float(r["Counter_Value"])
ids = sorted(rows)
fits = len(ids) // nblk
per_step = []
for c in range(nblk):
    acc = {}
    for fi in range(1, fits):  # skip the first (warm-up) factorisation
        for k, v in rows[ids[fi * nblk + c]].items():
            acc[k] = acc.get(k, 0.0) + v / max(fits - 1, 1)
    cyc = acc.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
    busy = acc.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
    flops = acc.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0) * 512.0
    m = nblk - c - 1
    M = (m + 1) // 2
    trail_flops = 2.0 * (128 ** 2) * 64 * (M * (M + 1) // 2) if c > 0 else 0.0
    per_step.append({"c": c, "kernel_cycles": cyc, "mfma_busy_frac_per_simd": busy / max(cyc * 1024.0, 1.0),
                     "mfma_flops": flops, "trailing_update_flops": trail_flops})
def summ(sel):
    cyc = sum(s["kernel_cycles"] for s in sel)
    busy = sum(s["mfma_busy_frac_per_simd"] * s["kernel_cycles"] for s in sel)
    return {"steps": len(sel), "kernel_cycles": cyc, "mfma_busy_frac_per_simd": busy / max(cyc, 1.0),
            "mfma_gflop": sum(s["mfma_flops"] for s in sel) / 1e9}
res = {"n": 64 * nblk, "fits_averaged": fits - 1, "dispatches_per_fit": nblk,
       "trailing_dominated_steps_1_to_22": summ(per_step[1:23]), "panel_dominated_steps_23_on": summ(per_step[23:]),
       "all_steps": summ(per_step), "per_step": per_step,
       "note": "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs) per dispatch; MOPS_F64 in units of 512 flops; "
               "trailing_update_flops = the 128x128xK=64 tiles of that launch (eager schedule)"}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "per_step"}, indent=1))
