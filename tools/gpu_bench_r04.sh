# The default bench line, its rocprofv3 kernel stats, and the N > 1 host-communicator rehearsals
# (columns mode headline + rows-mode extra) at 2 / 4 / 8 ranks on the one GPU.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/bench.json; [ "$rc" -eq 0 ] || exit $rc
# what outlives bench.py (the round-end lease reports one process left): this user's processes
ps -o pid,ppid,etime,stat,cmd -u "$(id -u)" > gpurun_out/ps_after_bench.txt 2>&1 || true
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-bfgs > gpurun_out/bench_prof.json 2> gpurun_out/prof.err
rc=$?; echo "rocprof rc=$rc"; [ "$rc" -eq 0 ] || exit $rc
for w in 2 4 8; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $w --master-addr 127.0.0.1 \
      --master-port $((29500 + w)) bench.py --gpus $w --host-comm --steps 5 --warmup 2 --no-cpu-baseline --no-bfgs \
      > gpurun_out/bench_hostcomm$w.json 2> gpurun_out/bench_hostcomm$w.err
  rc=$?; echo "hostcomm$w rc=$rc"; [ "$rc" -eq 0 ] || exit $rc
done
exit 0
