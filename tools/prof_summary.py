"""Print the top kernels of a rocprofv3 --stats CSV and the bench line's headline numbers."""
import csv
import json
import sys

stats = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_stats.csv"
bench = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/bench.json"
try:
    b = json.loads(open(bench).read().strip().splitlines()[-1])
    print("value", round(b["value"], 2), b["unit"], "| per-step ms", {k: round(v, 3) for k, v in b["kernel_ms_per_step"].items()})
except Exception as e:  # noqa: BLE001
    print("bench:", e)
rows = list(csv.DictReader(open(stats)))
for x in sorted(rows, key=lambda x: -float(x["TotalDurationNs"]))[:14]:
    print(f"{x['Name'][:66]:66s} calls={x['Calls']:>6} avg_us={float(x['AverageNs'])/1e3:9.2f} tot_ms={float(x['TotalDurationNs'])/1e6:8.2f}")
