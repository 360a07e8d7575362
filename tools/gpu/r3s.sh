#!/bin/bash
# K3 at cfg5: rocprof stats + PMC passes of the merged kernel (shipped) and of the two-launch
# variant (seq1), which separates the camera waves from the observation stream.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 bash tools/pmc_k3.sh r3s_k3_merged "ba_jtj_kernel|ba_finish_kernel" > gpurun_out/r3s_merged.log 2>&1 && \
SFMCORE_LIB=$PWD/sfm-project_amd/lib/libsfmcore_seq1.so timeout -k 10 600 bash tools/pmc_k3.sh r3s_k3_seq1 "ba_cam_kernel|ba_obs_kernel|ba_finish_kernel" > gpurun_out/r3s_seq1.log 2>&1
