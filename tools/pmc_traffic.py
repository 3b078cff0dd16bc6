"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch L2<->fabric bytes.

MI355X_MICROARCH.md (HBM section): FETCH_SIZE / WRITE_SIZE derive from TCC_EA0_RDREQ/_WRREQ
(Infinity-Cache hits are counted, not excluded); on gfx950 FETCH_SIZE reports exactly half of
the bytes of 16-B-per-lane coalesced reads, so it is doubled here (every hot kernel of this
library reads with 16-B lanes); WRITE_SIZE is exact for 16-B-per-lane stores.  Units: kB.
The two counters need separate passes (TCC slots), so each comes from its own run.

    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write profiles/r01_pmc_traffic.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(dirname, counter):
    files = glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(list)
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            name = row.get("Kernel_Name", "?")
            per[name].append(float(row["Counter_Value"]))
    return per


def short(name):
    for key in ("k_syrk_tile<0, 128", "k_syrk_tile<1, 64", "k_linres_fdP", "k_linres_evalP", "k_linres_fd2",
                "k_linres_fd", "k_linres_eval",
                "k_gemv_neg_wg<2, true>", "k_gemv_neg<2>", "k_gemv_neg<1>", "k_bfgs_pass<", "k_trsv_fwd", "k_trsv_bwd",
                "k_potrf_diag", "k_trsm_panel", "k_syrk_reduce", "k_chol_dag"):
        if key in name:
            return key.rstrip("<").replace("k_syrk_tile<0, 128", "k_syrk_tile<0, 128>").replace(
                "k_syrk_tile<1, 64", "k_syrk_tile<1, 64>")
    return None


def main():
    fdir, wdir, out = sys.argv[1], sys.argv[2], sys.argv[3]
    fetch, write = load(fdir, "FETCH_SIZE"), load(wdir, "WRITE_SIZE")
    res = {}
    for name in set(fetch) | set(write):
        k = short(name)
        if not k:
            continue
        fv, wv = fetch.get(name, []), write.get(name, [])
        if not fv or not wv:
            continue
        fb = 2.0 * 1e3 * sum(fv) / len(fv)      # kB -> B, x2 gfx950 wide-read correction
        wb = 1e3 * sum(wv) / len(wv)
        e = res.setdefault(k, {"fetch_bytes_per_launch": 0.0, "write_bytes_per_launch": 0.0, "launches": 0,
                               "kernel": name[:120]})
        e["fetch_bytes_per_launch"] = fb
        e["write_bytes_per_launch"] = wb
        e["traffic_bytes_per_launch"] = fb + wb
        e["launches"] = len(fv)
    json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), "
                         "FETCH doubled per MI355X_MICROARCH.md gfx950 correction",
               "kernels": res}, open(out, "w"), indent=1)
    for k, v in sorted(res.items()):
        print(f"{k:24s} fetch {v['fetch_bytes_per_launch']/1e6:10.2f} MB  write {v['write_bytes_per_launch']/1e6:10.2f} MB"
              f"  launches {v['launches']}")


if __name__ == "__main__":
    main()
