set -u
mkdir -p gpurun_out
for mp in 0 1; do
  for la in 64 0; do
    PNOL_CHOL_LOOKAHEAD=$la timeout -k 5 60 ./tools/microbench/chol_timeline_mp$mp 2048 > gpurun_out/tl_mp${mp}_la$la.json || exit 1
    echo "mp=$mp la=$la $(python3 tools/chol_tl_summary.py < gpurun_out/tl_mp${mp}_la$la.json)"
  done
done
