"""Per-launch durations of the last factorisation in a rocprofv3 --kernel-trace CSV (tools/fit_only.py); with a group
size g, launches are also summed in groups of g (the lazy-flush period)."""
import csv
import glob
import sys

path = sys.argv[1]
g = int(sys.argv[2]) if len(sys.argv) > 2 else 8
if not path.endswith(".csv"):
    path = sorted(glob.glob(path + "/**/*kernel_trace.csv", recursive=True))[-1]
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "gram" in r["Kernel_Name"]][-1]
seq = [r for r in rows[idx:] if "potrf_step" in r["Kernel_Name"]]
durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in seq]
print(f"{len(durs)} launches: sum {sum(durs):.1f} us")
for c in range(0, len(durs), g):
    grp = durs[c:c + g]
    print(f"c={c:3d}: sum {sum(grp):7.1f} | " + " ".join(f"{d:5.1f}" for d in grp))
