"""Summarise tools/microbench/chol_timeline output (persistent form): mean shader cycles per
diagonal-chain step in each phase (wait for the two tiles, prepare, factor, publish) and how
many steps used the look-ahead (lookahead_used = 1) or found the tiles staged only (2).  Usage: python tools/chol_tl_summary.py < timeline.json"""
import json
import sys

for line in sys.stdin:
    line = line.strip()
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    st = d["steps_us"][1:]
    ph = {"wait": [], "prepare": [], "factor": [], "publish": []}
    used = staged = 0
    for s in st:
        c = s["stamps"]   # staged, L strip, factor start, factor done, end, wait end
        wait_end = c[5]
        ph["wait"].append(wait_end)
        ph["prepare"].append(c[2] - wait_end)
        ph["factor"].append(c[3] - c[2])
        ph["publish"].append(c[4] - c[3])
        used += int(s.get("lookahead_used", 0)) == 1
        staged += int(s.get("lookahead_used", 0)) == 2
    out = {k: round(sum(v) / max(len(v), 1)) for k, v in ph.items()}
    out.update({"steps": len(st), "lookahead_used": used, "staged_only": staged, "ms_events": d["ms_events"], "lookahead": d.get("lookahead")})
    print(json.dumps(out))
