#!/bin/bash
# Sweep the persistent Cholesky's knobs with the per-step timeline tool (one JSON line each).
set -u
mkdir -p gpurun_out
B=tools/microbench/chol_timeline
out=gpurun_out/chol5_sweep.jsonl
: > $out
run() { timeout -k 10 60 env "$@" $B >> $out || exit $?; }
run PNOL_CHOL_PERSIST=0
for solo in 0; do
  for w in 64 128 192 255; do
    run PNOL_CHOL_PERSIST=1 PNOL_CHOL5_SOLO=$solo PNOL_CHOL5_WORKERS=$w
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/chol5_sweep.jsonl"):
    d = json.loads(l)
    ev = sorted(d["ms_events"][1:])
    st = d["steps_us"]
    fac = [s["stamps"][3] - s["stamps"][2] for s in st[1:]]
    wait = [s["stamps"][5] for s in st[1:]]
    stage = [s["stamps"][0] - s["stamps"][5] for s in st[1:]]
    pub = [s["stamps"][4] - s["stamps"][3] for s in st[1:]]
    print(d["persist"], d["solo"], d["workers"], "median_ms %.4f" % ev[len(ev)//2], "diag_us %.1f" % d["sum_diag_us"],
          "gap_us %.1f" % d["sum_gap_us"], "factor_cycles_mean %.0f" % (sum(fac)/len(fac)),
          "wait %.0f stage %.0f publish %.0f" % (sum(wait)/len(wait), sum(stage)/len(stage), sum(pub)/len(pub)))
PY
