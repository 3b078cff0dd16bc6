# Round 5, first GPU session: the multi-process Cholesky contention probe, then the whole GPU suite + smoke.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/chol_contention_probe.py --procs 3 --trips 300 --m 1000 --n 700 \
    --out gpurun_out/r05_chol_contention_3p.json > gpurun_out/r05_chol_contention.log 2>&1
rc=$?; echo "probe rc=$rc"; tail -30 gpurun_out/r05_chol_contention.log; [ "$rc" -eq 0 ] || exit $rc
bash tools/gpu_full_tests.sh
