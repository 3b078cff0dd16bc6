set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 400 --timeout-method thread -k "cfg2 or cfg4 or disagree or multi_rank or gpus_flag or rccl or quadratic_fast" > gpurun_out/pytest_r04c.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_r04c.log | tail -40; exit $rc
