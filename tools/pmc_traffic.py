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
            per[(name, int(row.get("Grid_Size") or 0))].append(float(row["Counter_Value"]))
    return per


def short(name):
    for key in ("k_syrk_red", "k_syrk_tile<0, 128", "k_syrk_tile<1, 64", "k_syrk_tile<4, 64", "k_linres_fdP", "k_linres_evalP", "k_linres_fd2",
                "k_linres_fd", "k_linres_eval",
                "k_gemv_neg_wg<2, true>", "k_gemv_neg<2>", "k_gemv_neg<1>", "k_bfgs_pass<", "k_trsv_fwd", "k_trsv_bwd",
                "k_potrf_diag", "k_trsm_panel", "k_syrk_reduce", "k_chol_dag", "k_chol_persist", "k_chol_bwd",
                "k_gemv_neg_slices"):
        if key in name:
            return key.rstrip("<").replace("k_syrk_tile<0, 128", "k_syrk_tile<0, 128>").replace(
                "k_syrk_tile<1, 64", "k_syrk_tile<1, 64>").replace("k_syrk_tile<4, 64", "k_syrk_tile<4, 64>")
    return None


def main():
    fdir, wdir, out = sys.argv[1], sys.argv[2], sys.argv[3]
    fetch, write = load(fdir, "FETCH_SIZE"), load(wdir, "WRITE_SIZE")
    # one entry per kernel and grid size (the bench launches H.g and the fused pass at n = 8192
    # and 4096: averaging them would mix two problem sizes); the plain kernel key holds the
    # largest grid, the bench's headline size
    res = {}
    for key in sorted(set(fetch) | set(write), key=lambda kg: kg[1]):
        name, grid = key
        k = short(name)
        if not k:
            continue
        fv, wv = fetch.get(key, []), write.get(key, [])
        if not fv or not wv:
            continue
        fb = 2.0 * 1e3 * sum(fv) / len(fv)      # kB -> B, x2 gfx950 wide-read correction
        wb = 1e3 * sum(wv) / len(wv)
        e = {"fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb, "traffic_bytes_per_launch": fb + wb,
             "launches": len(fv), "grid_size": grid, "kernel": name[:120]}
        res[f"{k}@grid{grid}"] = e
        res[k] = e   # ascending grids: the largest wins
    json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), "
                         "FETCH doubled per MI355X_MICROARCH.md gfx950 correction; per kernel and grid size",
               "kernels": res}, open(out, "w"), indent=1)
    for k, v in sorted(res.items()):
        if "@" in k:
            print(f"{k:40s} fetch {v['fetch_bytes_per_launch']/1e6:10.2f} MB  write {v['write_bytes_per_launch']/1e6:10.2f} MB"
                  f"  launches {v['launches']}")


if __name__ == "__main__":
    main()
