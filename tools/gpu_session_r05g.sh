#!/bin/bash
# r05f (-J^T F in the SYRK: tests + library A/B + kernel trace) and r05e (fused pass prefetch sweep).
set -u
bash tools/gpu_session_r05f.sh || exit $?
bash tools/gpu_session_r05e.sh
