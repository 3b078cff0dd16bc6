set -u
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_solvers.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "chol or trip or lm_ or solve" > gpurun_out/sp_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/sp_pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for sp in 1 0; do
    PNOL_CHOL_SPLIT=$sp timeout -k 5 60 ./tools/microbench/chol_timeline 2048 > gpurun_out/sp_tl_${sp}_$rep.json || exit 7
    echo "split=$sp $(python3 tools/chol_tl_summary.py < gpurun_out/sp_tl_${sp}_$rep.json)"
    python3 -c "
import json,statistics; d=json.loads(open('gpurun_out/sp_tl_${sp}_$rep.json').readline()); c=[r[6] for r in d['critical_us_after_W'] if r[6]>-1]; print('  crit publish median us after W', round(statistics.median(c),2))"
  done
done
VAR=PNOL_CHOL_SPLIT VALS="1 0" KEY=syrk bash tools/env_ab.sh
