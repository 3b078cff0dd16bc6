"""Summarise a rocprofv3 --kernel-trace --stats directory: the top kernels of the stats CSV, and
the same kernels split by grid size from the kernel trace (the bench launches H.g and the fused
BFGS pass at three sizes each, which the stats CSV folds into one row).

    python3 tools/prof_summary.py gpurun_out/<dir> [bench.json] [--csv out_by_grid.csv]
"""
import csv
import glob
import json
import os
import statistics
import sys


def short(name):
    for p in ("pnol::(anonymous namespace)::", "(anonymous namespace)::", "pnol::"):
        name = name.replace(p, "")
    if name.startswith("void "):
        name = name[5:]
    return name.split("(")[0]


def by_grid(trace_csv):
    """{(kernel, grid_x, wg_x): [durations ns]} from a kernel-trace CSV"""
    out = {}
    for r in csv.DictReader(open(trace_csv)):
        k = (short(r["Kernel_Name"]), int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))
        out.setdefault(k, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    out_csv = sys.argv[sys.argv.index("--csv") + 1] if "--csv" in sys.argv else None
    if out_csv in args:
        args.remove(out_csv)
    d = args[0] if args else "gpurun_out/prof"
    stats = (glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True) or [d])[0]
    traces = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if len(args) > 1:
        try:
            b = json.loads(open(args[1]).read().strip().splitlines()[-1])
            print("value", round(b["value"], 2), b["unit"])
        except Exception as e:  # noqa: BLE001
            print("bench:", e)
    if os.path.isfile(stats):
        rows = list(csv.DictReader(open(stats)))
        print("== kernel stats (all launches, warmup included)")
        for x in sorted(rows, key=lambda x: -float(x["TotalDurationNs"]))[:16]:
            print(f"{short(x['Name'])[:48]:48s} calls={x['Calls']:>6} avg_us={float(x['AverageNs'])/1e3:9.2f} "
                  f"tot_ms={float(x['TotalDurationNs'])/1e6:8.2f}")
    if not traces:
        return
    g = by_grid(traces[0])
    print("== by kernel and grid size (kernel trace)")
    rows = []
    for (k, gx, wx), v in sorted(g.items(), key=lambda kv: -sum(kv[1])):
        rows.append({"kernel": k, "grid_x": gx, "workgroup_x": wx, "workgroups": gx // max(wx, 1), "calls": len(v),
                     "avg_us": statistics.mean(v) / 1e3, "median_us": statistics.median(v) / 1e3,
                     "min_us": min(v) / 1e3, "max_us": max(v) / 1e3, "total_ms": sum(v) / 1e6})
    for r in rows[:30]:
        print(f"{r['kernel'][:40]:40s} wgs={r['workgroups']:>7} calls={r['calls']:>6} avg_us={r['avg_us']:9.2f} "
              f"med_us={r['median_us']:9.2f} min_us={r['min_us']:9.2f} tot_ms={r['total_ms']:8.2f}")
    if out_csv:
        with open(out_csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
            w.writeheader()
            for r in rows:
                w.writerow({k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()})


if __name__ == "__main__":
    main()
