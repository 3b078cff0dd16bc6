# Round-4 PMC passes of the damped solve: the standalone solve (tools/solve_bench.py, n = 2048)
# and the LM trip's reducing persistent Cholesky (bench.py trips); wave-cycle buckets, then MFMA.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -s KILL "$lim" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
MF="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
B="bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-bfgs --no-hg"
step sq_solve 120 rocprofv3 --pmc $SQ -d /tmp/c_sq_s -o pmc --output-format csv -- python3 tools/solve_bench.py 2048 5
step mf_solve 120 rocprofv3 --pmc $MF -d /tmp/c_mf_s -o pmc --output-format csv -- python3 tools/solve_bench.py 2048 5
step sq_trip 240 rocprofv3 --pmc $SQ -d /tmp/c_sq_t -o pmc --output-format csv -- python3 $B
step mf_trip 240 rocprofv3 --pmc $MF -d /tmp/c_mf_t -o pmc --output-format csv -- python3 $B
python3 tools/pmc_valu.py /tmp/c_sq_s gpurun_out/r04_pmc_chol_solve_sq.json k_chol_persist k_chol_bwd &&
python3 tools/pmc_valu.py /tmp/c_mf_s gpurun_out/r04_pmc_chol_solve_mfma.json k_chol_persist k_chol_bwd &&
python3 tools/pmc_valu.py /tmp/c_sq_t gpurun_out/r04_pmc_chol_trip_sq.json k_chol_persist k_chol_bwd &&
python3 tools/pmc_valu.py /tmp/c_mf_t gpurun_out/r04_pmc_chol_trip_mfma.json k_chol_persist k_chol_bwd
