"""Kernel timeline from a rocprofv3 results database (rocpd sqlite): per dispatch the kernel
name, start / end relative to the first listed dispatch (us) and duration.  argv: db [name
substring filter ...] [--last N]."""
import glob
import sqlite3
import sys


def main():
    args = sys.argv[1:]
    last = None
    if "--last" in args:
        i = args.index("--last")
        last = int(args[i + 1])
        del args[i:i + 2]
    db, filt = args[0], args[1:]
    con = sqlite3.connect(db)
    tabs = [r[0] for r in con.execute("select name from sqlite_master where type='table'")]
    kd = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
    ks = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
    cols = [r[1] for r in con.execute(f"pragma table_info({kd})")]
    scol = [r[1] for r in con.execute(f"pragma table_info({ks})")]
    name_col = "kernel_name" if "kernel_name" in scol else ("display_name" if "display_name" in scol else scol[1])
    rows = con.execute(f"select d.start, d.end, s.{name_col}, d.queue_id from {kd} d join {ks} s on d.kernel_id = s.id "
                       f"order by d.start").fetchall() if "queue_id" in cols else \
        [(a, b, c, 0) for a, b, c in con.execute(f"select d.start, d.end, s.{name_col} from {kd} d join {ks} s "
                                                  f"on d.kernel_id = s.id order by d.start")]
    if filt:
        rows = [r for r in rows if any(f in r[2] for f in filt)]
    if last:
        rows = rows[-last:]
    t0 = rows[0][0]
    for s, e, n, q in rows:
        print(f"{(s - t0) / 1e3:10.1f} {(e - t0) / 1e3:10.1f} {(e - s) / 1e3:9.1f}  q{q}  {n[:70]}")


if __name__ == "__main__":
    main()
