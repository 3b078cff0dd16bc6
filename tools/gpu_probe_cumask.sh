set -u
mkdir -p gpurun_out
timeout -k 10 60 ./tools/microbench/cumask_probe > gpurun_out/cumask.json 2>&1; echo "cumask rc=$?"; cat gpurun_out/cumask.json
timeout -k 10 240 ./tools/microbench/overlap_probe > gpurun_out/overlap.json 2> gpurun_out/overlap.err; echo "overlap rc=$?"; cat gpurun_out/overlap.json
