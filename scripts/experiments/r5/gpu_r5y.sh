#!/bin/bash
# Round 5, batch Y: the WRMF pipeline and side-stream HH against the serial path, bit for bit
# (experiments build; scripts/check_wrmf_pipe_identity.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
(
    export MML_LIB_PATH=variants/exp/libmml_hip.so MML_WRMF_PIPE=1 MML_WRMF_HH_SIDE=0
    step r5y_serial 300 python -u scripts/check_wrmf_pipe_identity.py save gpurun_out/wrmf_serial.npz
) || exit $?
(
    export MML_LIB_PATH=variants/exp/libmml_hip.so MML_WRMF_PIPE=4
    step r5y_pipe 300 python -u scripts/check_wrmf_pipe_identity.py save gpurun_out/wrmf_pipe.npz
) || exit $?
step r5y_compare 120 python -u scripts/check_wrmf_pipe_identity.py compare gpurun_out/wrmf_serial.npz gpurun_out/wrmf_pipe.npz
rm -f gpurun_out/wrmf_serial.npz gpurun_out/wrmf_pipe.npz
