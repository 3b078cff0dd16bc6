#!/bin/bash
# The N > 1 bench line rehearsed on one GPU: bench.py --gpus N --host-comm (bench.py starts its
# N rank processes itself; gloo + the host communicator; the ranks share the box's GPU), for
# N in NS (default 2 4 8).  Each run has its own limit; the first failure ends the session.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in ${NS:-2 4 8}; do
  timeout -k 10 400 python bench.py --gpus $n --host-comm --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --no-bfgs \
      > gpurun_out/bench_hostcomm$n.json 2> gpurun_out/bench_hostcomm$n.err
  rc=$?; echo "hostcomm$n rc=$rc"; tail -c 400 gpurun_out/bench_hostcomm$n.json; echo
  [ "$rc" -eq 0 ] || exit $rc
done
exit 0
