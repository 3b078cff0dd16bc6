# PMC passes on the timed build (one counter group per run, no trace domains): the bench's
# FETCH_SIZE / WRITE_SIZE, the SYRK's MFMA busy, the FD's VALU busy, and the trip's persistent
# Cholesky wave-cycle buckets and MFMA busy; summaries to gpurun_out/${TAG}_pmc_*.json (TAG=r06).
set -u
T=${TAG:-r06}
mkdir -p gpurun_out
export TMPDIR=/tmp
B="bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-bfgs"
run() { local name=$1; shift; timeout -s KILL 300 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
MF="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
run pmc_fetch rocprofv3 --pmc FETCH_SIZE -d /tmp/pmc_fetch -o pmc --output-format csv -- python3 $B &&
run pmc_write rocprofv3 --pmc WRITE_SIZE -d /tmp/pmc_write -o pmc --output-format csv -- python3 $B &&
run pmc_mfma rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d /tmp/pmc_mfma -o pmc --output-format csv -- python3 $B --no-hg &&
run pmc_valu rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d /tmp/pmc_valu -o pmc --output-format csv -- python3 $B --no-hg &&
run pmc_csq rocprofv3 --pmc $SQ -d /tmp/c_sq_t -o pmc --output-format csv -- python3 $B --no-hg &&
run pmc_cmf rocprofv3 --pmc $MF -d /tmp/c_mf_t -o pmc --output-format csv -- python3 $B --no-hg || exit 1
python3 tools/pmc_traffic.py /tmp/pmc_fetch /tmp/pmc_write gpurun_out/${T}_pmc_traffic.json &&
python3 tools/pmc_valu.py /tmp/pmc_mfma gpurun_out/${T}_pmc_syrk_mfma.json k_syrk_red k_syrk_tile &&
python3 tools/pmc_valu.py /tmp/pmc_valu gpurun_out/${T}_pmc_fd_valu.json k_linres_fdP k_linres_evalP &&
python3 tools/pmc_valu.py /tmp/c_sq_t gpurun_out/${T}_pmc_chol_trip_sq.json k_chol_persist k_chol_bwd &&
python3 tools/pmc_valu.py /tmp/c_mf_t gpurun_out/${T}_pmc_chol_trip_mfma.json k_chol_persist k_chol_bwd
