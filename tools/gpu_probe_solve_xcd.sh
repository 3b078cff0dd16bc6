# The damped solve (method 5, n = 2048) on the whole chip vs confined to one XCD (PNOL_CHOL_XCD).
set -u
mkdir -p gpurun_out
for x in -1 0 5 -1 0; do
  if [ "$x" = "-1" ]; then unset PNOL_CHOL_XCD; else export PNOL_CHOL_XCD=$x; fi
  timeout -k 10 120 python tools/solve_bench.py 2048 5 5 || exit $?
done
