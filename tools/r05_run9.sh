set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/trace9
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace9 -o fit -- python3 $R/tools/fit_only.py --n 4096 --reps 3 > $R/gpurun_out/trace9.log 2>&1 || exit $?
cd $R
python3 tools/potrf_launches.py gpurun_out/trace9 8 > gpurun_out/r05_potrf_launches_4096.log 2>&1
python3 - >> gpurun_out/r05_potrf_launches_4096.log <<'PY'
import csv, glob
p = sorted(glob.glob("gpurun_out/trace9/**/*kernel_trace.csv", recursive=True))[-1]
rows = sorted(csv.DictReader(open(p)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "gram" in r["Kernel_Name"]][-1]
seq = rows[idx:]
t0 = int(seq[0]["Start_Timestamp"])
for r in seq:
    if "potrf_step" in r["Kernel_Name"]:
        continue
    print(f"{r['Kernel_Name'][:60]:60s} start {(int(r['Start_Timestamp'])-t0)/1e3:9.1f} us dur {(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3:7.1f} us")
print(f"whole update {(int(seq[-1]['End_Timestamp'])-t0)/1e3:.1f} us")
PY
timeout -k 10 300 python -u tools/opt_ab.py --n 4096 --batch 4 --rounds 3 --reps 5 --arms "" "potrf_switch=0" > gpurun_out/r05_sched_b4_check.log 2>&1
