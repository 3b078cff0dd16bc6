#!/bin/bash
# Same-box sweep of SYRK launch knobs (env) with tools/microbench/syrk_timeline: every config
# runs once per round, 4 rounds, then the median of each config's per-launch medians.
set -e
CONFIGS=("" "PNOL_SYRK_FIRST=70" "PNOL_SYRK_FIRST=80" "PNOL_SYRK_FIRST=85" "PNOL_SYRK_SUB=3" "PNOL_SYRK_SUB=3 PNOL_SYRK_FIRST=60" "PNOL_SYRK_SUB=4 PNOL_SYRK_FIRST=70")
out=gpurun_out/syrk_env_ab.txt
mkdir -p gpurun_out
: > $out
for r in 1 2 3 4; do
  for c in "${CONFIGS[@]}"; do
    v=$(timeout -k 10 60 env $c tools/microbench/syrk_timeline 16384 2048 10 | python3 -c "import json,sys; d=json.load(sys.stdin); e=sorted(d['ms_events'][2:]); print('%.4f %.1f' % (e[len(e)//2], d['tail_us']))")
    echo "[$c] $v" >> $out
  done
done
python3 - <<'PY'
from collections import defaultdict
d = defaultdict(list)
for l in open("gpurun_out/syrk_env_ab.txt"):
    k, v = l.rsplit("]", 1)
    ms, tail = v.split()
    d[k + "]"].append((float(ms), float(tail)))
for k, v in d.items():
    ms = sorted(x[0] for x in v); tl = sorted(x[1] for x in v)
    print(f"{k:45s} median_ms {ms[len(ms)//2]:.4f}  runs {' '.join('%.4f' % x for x in ms)}  tail_us {tl[len(tl)//2]:.0f}")
PY
