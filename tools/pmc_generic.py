"""Per-kernel means of every counter in rocprofv3 --pmc CSV output under a directory.

    python tools/pmc_generic.py gpurun_out/pmc_x [kernel-substring]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

src = sys.argv[1]
key = sys.argv[2] if len(sys.argv) > 2 else ""
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "?")
        if key in name:
            vals[name[:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {k: {c: sum(v) / len(v) for c, v in d.items()} | {"launches": max(len(v) for v in d.values())}
       for k, d in vals.items()}
print(json.dumps(out, indent=1))
