"""Per-batch kernel timeline of a config5 kernel trace (scripts/gpu_session.sh):
python scripts/c5_timeline.py gpurun_out/c5t/c5_kernel_trace.csv [batch ...]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
# a batch starts at its key sort's histogram pass (round 3 on: the sort runs before the lift, queued behind the
# previous batch's result copy); older traces start it at the lift
mark = "k_cs_hist<" if any("k_cs_hist<" in r["Kernel_Name"] for r in rows) and any(
    "k_lift_search<" in r["Kernel_Name"] for r in rows) else "k_lift<"
lifts = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"] and int(r["Grid_Size_X"]) < 2_000_000]
# "longest": the two batches with the longest spans (the compacting ones), then the arguments
args = sys.argv[2:]
if args and args[0] == "longest":
    spans = sorted(range(len(lifts) - 1), key=lambda b: int(rows[lifts[b + 1]]["Start_Timestamp"]) - int(rows[lifts[b]]["Start_Timestamp"]))
    args = [str(b) for b in sorted(spans[-2:])] + args[1:]
batches = [int(b) for b in args] or [len(lifts) - 3]
for b in batches:
    i0, i1 = lifts[b], lifts[b + 1]
    t0 = int(rows[i0]["Start_Timestamp"])
    busy, prev = 0, t0
    print(f"--- batch {b}: span {(int(rows[i1]['Start_Timestamp']) - t0) / 1e3:.1f} us")
    for r in rows[i0:i1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += e - s
        print(f"{(s - t0) / 1e3:8.1f} gap {(s - prev) / 1e3:6.1f} dur {(e - s) / 1e3:7.1f}  {r['Kernel_Name'][:90]}")
        prev = e
    print(f"kernels {busy / 1e3:.1f} us, idle after the last {(int(rows[i1]['Start_Timestamp']) - prev) / 1e3:.1f} us")
