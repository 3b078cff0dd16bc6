#!/bin/bash
# PMC passes of the damped solve's kernels (prep / persistent / backward) on tools/solve_bench.py
# (n = 2048, method 5): SQ wave-cycle buckets + VALU, then MFMA busy; summarised per kernel.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -s KILL "$lim" "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
step pmc_sq 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
    SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d /tmp/pmc_chol_sq -o pmc --output-format csv -- \
    python tools/solve_bench.py 2048 5
step pmc_mfma 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
    -d /tmp/pmc_chol_mfma -o pmc --output-format csv -- python tools/solve_bench.py 2048 5
python3 tools/pmc_valu.py /tmp/pmc_chol_sq gpurun_out/pmc_chol_sq.json k_chol_persist k_chol_bwd k_chol_step
python3 tools/pmc_valu.py /tmp/pmc_chol_mfma gpurun_out/pmc_chol_mfma.json k_chol_persist k_chol_bwd k_chol_step
