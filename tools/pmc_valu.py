"""Summarise a rocprofv3 --pmc pass of SQ_INSTS_VALU / SQ_ACTIVE_INST_VALU / GRBM_GUI_ACTIVE (+ the
SQ wait buckets) per kernel: VALU busy fraction = 4 * SQ_ACTIVE_INST_VALU (quad-cycles -> cycles)
/ (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs), the effective clock = GRBM_GUI_ACTIVE / 8 / wall.

    python tools/pmc_valu.py gpurun_out/pmc_fdp profiles/r01_pmc_fd_valu.json [kernel-substring ...]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

src, out = sys.argv[1], sys.argv[2]
keys = sys.argv[3:] or ["k_linres_fdP", "k_linres_evalP", "k_syrk_tile"]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "?")
        if any(k in name for k in keys):
            vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {"source": "rocprofv3 --pmc " + src, "simds": 1024, "xcds": 8, "kernels": {}}
for name, d in vals.items():
    avg = {c: sum(v) / len(v) for c, v in d.items()}
    e = {"counters_per_launch": avg, "launches": len(next(iter(d.values())))}
    if "SQ_ACTIVE_INST_VALU" in avg and "GRBM_GUI_ACTIVE" in avg:
        e["valu_busy_frac"] = 4 * avg["SQ_ACTIVE_INST_VALU"] / (avg["GRBM_GUI_ACTIVE"] / 8 * 1024)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg:
        e["mfma_busy_frac"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (avg["GRBM_GUI_ACTIVE"] / 8 * 1024)
    if "SQ_WAVE_CYCLES" in avg:
        w = avg["SQ_WAVE_CYCLES"]
        e["wave_cycle_split"] = {k: avg[k] / w for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY")
                                 if k in avg}
    res["kernels"][name[:120]] = e
json.dump(res, open(out, "w"), indent=1)
for k, e in res["kernels"].items():
    print(k[:70], {kk: (round(v, 3) if isinstance(v, float) else v) for kk, v in e.items() if kk != "counters_per_launch"})
