"""Summarise a rocprofv3 --kernel-trace CSV of tools/fit_timing.py: per-dispatch durations of the last fit."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/trace/fit_kernel_trace.csv")))
names = [r["Kernel_Name"] for r in rows]
start = [i for i, n in enumerate(names) if "gram_kernel" in n][-1]
seq = rows[start:]
prev = int(seq[0]["Start_Timestamp"])
for r in seq:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    nm = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if "potrf_step" in nm or "mll_" in nm:
        continue
    if "gpx::" not in nm:
        if "rocclr" in nm:
            continue
        break
    print(f"{nm[:34]:34s} grid={r['Grid_Size_X']:>7}x{r['Grid_Size_Y']:>3}x{r['Grid_Size_Z']:>3} "
          f"dur={(e - s) / 1e3:8.1f}us gap={(s - prev) / 1e3:6.1f}us")
    prev = e
ps = [r for r in seq if "potrf_step" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in ps]
print(f"potrf: {len(d)} steps, {sum(d):.1f} us; per step:", " ".join(f"{x:.0f}" for x in d))
