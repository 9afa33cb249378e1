"""Per-dispatch counters of the large-n Cholesky's flush launches (every g-th potrf_step_kernel dispatch of the last
factorisation in a rocprofv3 --pmc pass over tools/fit_only.py): MFMA busy per SIMD, memory-side bytes, L2 hit rate.
usage: python tools/pmc_flush.py PASS_DIR [PASS_DIR ...] --nblk 256 --g 8"""
import argparse, csv, glob, os
ap = argparse.ArgumentParser()
ap.add_argument("dirs", nargs="+")
ap.add_argument("--nblk", type=int, default=256)
ap.add_argument("--g", type=int, default=8)
a = ap.parse_args()
rows = {}
for d in a.dirs:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "potrf_step_kernel" not in r.get("Kernel_Name", ""):
                continue
            key = (d, int(r.get("Dispatch_Id", 0)))
            rows.setdefault(key, {})[r["Counter_Name"]] = float(r["Counter_Value"])
for d in a.dirs:
    ids = sorted(k for k in rows if k[0] == d)
    last = ids[-a.nblk:]
    print(f"== {d}: {len(ids)} dispatches, last factorisation {len(last)}")
    for c in list(range(a.g, a.nblk, a.g))[:6] + [a.g + 1, a.g + 4, a.g + 7]:
        v = rows[last[c]]
        cyc = v.get("GRBM_GUI_ACTIVE", 0) / 8.0
        out = [f"c={c:3d} gui_cycles/8={cyc:9.0f}"]
        if "SQ_VALU_MFMA_BUSY_CYCLES" in v:
            out.append(f"mfma_busy/SIMD={v['SQ_VALU_MFMA_BUSY_CYCLES'] / max(cyc * 1024, 1):.3f}")
        for k in ("FETCH_SIZE", "WRITE_SIZE"):
            if k in v:
                out.append(f"{k}={v[k] / 1024 / 1024:.2f} GiB")
        if "TCC_HIT_sum" in v and "TCC_MISS_sum" in v:
            h, m = v["TCC_HIT_sum"], v["TCC_MISS_sum"]
            out.append(f"L2 hit={h / max(h + m, 1):.3f} (miss {m:.3g})")
        print("  " + "  ".join(out))
