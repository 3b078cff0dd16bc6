#!/bin/bash
# Same-box A/B of a persistent-Cholesky knob (KNOB, default PNOL_CHOL_SPLIT): the Cholesky / trip / LM GPU tests first, then alternating standalone
# timelines at n = 2048 (tools/microbench/chol_timeline: per-step cycles, look-ahead count, the
# critical tile's publish after W), then the LM bench (tools/env_ab.sh).
set -u
mkdir -p gpurun_out
KNOB=${KNOB:-PNOL_CHOL_SPLIT}
timeout -k 10 700 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_solvers.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "chol or trip or lm_ or solve" > gpurun_out/sp_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/sp_pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in 1 0; do
    env $KNOB=$v timeout -k 5 60 ./tools/microbench/chol_timeline 2048 > gpurun_out/sp_tl_${v}_$rep.json || exit 7
    echo "$KNOB=$v $(python3 tools/chol_tl_summary.py < gpurun_out/sp_tl_${v}_$rep.json)"
    python3 -c "
import json,statistics; d=json.loads(open('gpurun_out/sp_tl_${v}_$rep.json').readline()); c=[r[6] for r in d['critical_us_after_W'] if r[6]>-1]; print('  crit publish median us after W', round(statistics.median(c),2), ' per step:', ' '.join(str(s['lookahead_used']) for s in d['steps_us'][1:]))"
  done
done
VAR=$KNOB VALS="1 0" KEY=syrk bash tools/env_ab.sh
