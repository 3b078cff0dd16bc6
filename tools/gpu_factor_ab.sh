# The diagonal factor before / after a change: W's checksum and stamps (diag_factor_probe), the
# persistent solve's per-step timeline (chol_timeline), alternating; then the solve / LM tests.
set -u
mkdir -p gpurun_out
for r in 1 2; do
  for v in old new; do
    timeout -k 5 30 ./tools/microbench/diag_factor_probe_$v > gpurun_out/fp_$v.json || exit 1
    echo "probe $v $(cat gpurun_out/fp_$v.json)"
    timeout -k 5 60 ./tools/microbench/chol_timeline_$v 2048 > gpurun_out/tl_$v.json || exit 1
    echo "timeline $v $(python3 tools/chol_tl_summary.py < gpurun_out/tl_$v.json)"
  done
done
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    -k "chol or solve or lm_trip or levmarq or fused_trip or cfg3" > gpurun_out/fa_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/fa_tests.log; exit $rc
