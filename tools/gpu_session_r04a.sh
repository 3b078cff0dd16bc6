set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/fd_phase_probe.py 5 > gpurun_out/fd_phase_probe.json 2> gpurun_out/fd_phase_probe.err || exit $?
echo probe1 done
timeout -k 10 300 python -u tools/cfg2_traj_probe.py > gpurun_out/cfg2_traj.json 2> gpurun_out/cfg2_traj.err || exit $?
echo probe2 done
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "bnd or recur or Recur" > gpurun_out/pytest_bnd.log 2>&1 || exit $?
tail -3 gpurun_out/pytest_bnd.log
