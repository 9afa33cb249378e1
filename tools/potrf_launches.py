"""Per-launch durations and gaps of the last factorisation in a rocprofv3 --kernel-trace CSV (tools/fit_only.py)."""
import csv
import glob
import sys

path = sys.argv[1]
if not path.endswith(".csv"):
    path = sorted(glob.glob(path + "/**/*kernel_trace.csv", recursive=True))[-1]
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "gram_kernel" in r["Kernel_Name"]][-1]
seq = [r for r in rows[idx:] if "potrf_step" in r["Kernel_Name"]]
prev = None
durs, gaps = [], []
for r in seq:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    durs.append((e - s) / 1e3)
    gaps.append(0.0 if prev is None else (s - prev) / 1e3)
    prev = e
print(f"{len(durs)} launches: sum dur {sum(durs):.1f} us, sum gaps {sum(gaps):.1f} us")
for c in range(0, len(durs), 8):
    print(f"c={c:2d}: " + " ".join(f"{d:5.1f}/{g:3.1f}" for d, g in zip(durs[c:c + 8], gaps[c:c + 8])))
