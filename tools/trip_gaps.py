"""Per-trip idle time of the one-GPU LM loop from a rocprofv3 kernel trace: for every trip, the
gaps between its kernels (evaluation -> [copy] -> next FD launch and the in-trip boundaries),
medians over the trips.  Usage: python tools/trip_gaps.py <run_kernel_trace.csv> [label]"""
import csv
import re
import statistics
import sys


def short(name):
    m = re.search(r"(k_\w+|__amd_\w+)", name)
    return m.group(1) if m else name[:30]


rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ks = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
fd = [i for i, k in enumerate(ks) if k[0] == "k_linres_fdP"]
eval_to_fd, trip_gaps, trip_span, eval_us = [], [], [], []
for a, b in zip(fd, fd[1:]):
    seg = ks[a:b + 1]
    ev = max(i for i, k in enumerate(seg) if k[0] in ("k_linres_evalP", "k_linres_evalS"))
    eval_to_fd.append((seg[-1][1] - seg[ev][2]) / 1e3)
    eval_us.append((seg[ev][2] - seg[ev][1]) / 1e3)
    trip_gaps.append(sum(max(0, seg[i][1] - seg[i - 1][2]) for i in range(1, len(seg))) / 1e3)
    trip_span.append((seg[-1][1] - seg[0][1]) / 1e3)
label = sys.argv[2] if len(sys.argv) > 2 else ""
print(f"{label} trips {len(trip_span)}: span {statistics.median(trip_span):.1f} us, idle {statistics.median(trip_gaps):.1f} us, "
      f"evaluation {statistics.median(eval_us):.1f} us, its end -> next FD start {statistics.median(eval_to_fd):.1f} us (medians)")
