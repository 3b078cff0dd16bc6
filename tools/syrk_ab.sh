#!/bin/bash
# Same-box A/B of two syrk_timeline builds (tools/microbench/syrk_timeline.hip, e.g. one with
# -DPNOL_SYRK_NO_DIAG_SKIP): alternating runs, median / min of the HIP-event times per launch.
#   tools/syrk_ab.sh tools/microbench/syrk_timeline tools/microbench/syrk_timeline_b
set -e
for i in 1 2 3 4; do
  for b in "$@"; do
    timeout -k 10 60 "$b" 16384 2048 12 | python3 -c "import json,sys; d=json.load(sys.stdin); e=sorted(d['ms_events'][2:]); print('$b', 'min %.4f med %.4f' % (e[0], e[len(e)//2]), 'span', d['span_us'])"
  done
done
