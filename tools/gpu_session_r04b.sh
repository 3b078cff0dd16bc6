set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/fd_phase_probe.py 5 > gpurun_out/fd_phase_probe_pw.json 2> gpurun_out/fd_phase_probe_pw.err || exit $?
echo probe done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "fd_jacobian or fd_tiles or cfg2 or fd_modes or cfg4 or disagree or multi_rank or gpus_flag or rccl or quadratic_fast" > gpurun_out/pytest_r04b.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_r04b.log | tail -60; exit $rc
