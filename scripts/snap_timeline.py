"""Kernel timeline of one snapshot reload from a kernel trace (scripts/gpu_session.sh):
python scripts/snap_timeline.py <kernel_trace.csv> [reload index, default: the second to last]
A reload starts at k_snap_walk; kernels of both stores' streams are listed in start order."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
walks = [i for i, r in enumerate(rows) if "k_snap_walk" in r["Kernel_Name"]]
k = int(sys.argv[2]) if len(sys.argv) > 2 else len(walks) - 2
i0 = walks[k]
i1 = walks[k + 1] if k + 1 < len(walks) else len(rows)
t0 = int(rows[i0]["Start_Timestamp"])
end = max(int(r["End_Timestamp"]) for r in rows[i0:i1])
print(f"--- reload {k} of {len(walks)}: first kernel start to last kernel end {(end - t0) / 1e3:.1f} us")
busy, prev = 0, t0
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    print(f"{(s - t0) / 1e3:8.1f} gap {(s - prev) / 1e3:7.1f} dur {(e - s) / 1e3:7.1f}  {r['Kernel_Name'][:90]}")
    prev = max(prev, e)
print(f"kernel time {busy / 1e3:.1f} us")
