"""Print the kernel sequence of the last solve (from k_chol_prep on) in a rocprofv3 kernel trace.
    python tools/kt_summary.py TRACE.csv [FIRST_KERNEL_SUBSTRING] [COUNT]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
key = sys.argv[2] if len(sys.argv) > 2 else "k_chol_prep"
cnt = int(sys.argv[3]) if len(sys.argv) > 3 else 40
rows.sort(key=lambda x: int(x["Start_Timestamp"]))
idx = [i for i, x in enumerate(rows) if key in x["Kernel_Name"]]
s = idx[-1]
prev = None
t0 = int(rows[s]["Start_Timestamp"])
for x in rows[s:s + cnt]:
    st, en = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    name = x["Kernel_Name"].split("(")[0].split("::")[-1]
    gap = (st - prev) / 1000 if prev else 0.0
    print(f"{name:28s} grid={int(x['Grid_Size_X']) // int(x['Workgroup_Size_X']):6d} dur={(en - st) / 1000:8.2f} gap={gap:6.2f} t={(en - t0) / 1000:8.1f}")
    prev = en
