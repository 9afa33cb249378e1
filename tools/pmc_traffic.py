"""Turn rocprofv3 --pmc CSV passes into per-launch HBM traffic for one kernel (guide: MI355X_MICROARCH.md HBM).

FETCH_SIZE on gfx950 reports half the bytes of wide coalesced streaming reads -> doubled here (uncalibrated for
other access widths: stated in the output).  WRITE_SIZE is exact for 16-B/lane stores.  Both in KiB per dispatch.
usage: python tools/pmc_traffic.py KERNEL_SUBSTRING fetch_pass_dir write_pass_dir [out.json]
"""
import csv, glob, json, os, sys

def per_dispatch(d, counter, kname):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if kname in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                vals.append(float(row["Counter_Value"]))
    return vals

k, fd, wd = sys.argv[1], sys.argv[2], sys.argv[3]
fetch = per_dispatch(fd, "FETCH_SIZE", k)
write = per_dispatch(wd, "WRITE_SIZE", k)
res = {"kernel": k, "dispatches": len(fetch),
       "fetch_kib_raw_avg": sum(fetch) / max(len(fetch), 1), "write_kib_avg": sum(write) / max(len(write), 1)}
res["hbm_bytes_per_launch"] = (2 * res["fetch_kib_raw_avg"] + res["write_kib_avg"]) * 1024
import time
res["generated_utc"] = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())
res["passes"] = [os.path.basename(os.path.normpath(fd)), os.path.basename(os.path.normpath(wd))]
res["note"] = "FETCH_SIZE doubled per the gfx950 correction for wide coalesced reads; Infinity-Cache hits are counted by these memory-side counters"
print(json.dumps(res, indent=1))
if len(sys.argv) > 4:
    json.dump(res, open(sys.argv[4], "w"), indent=1)
