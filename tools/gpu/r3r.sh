#!/bin/bash
# K3 A/B: the camera waves and the observation blocks as two launches (each at its own register
# budget), 1/2/4/8 camera splits, interleaved with the merged kernel; then the bit check of the
# BA solve change (previous library vs this one).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 bash tools/gpu/ba_ab.sh 3 base seq1 seq2 seq4 seq8 > gpurun_out/r3r_k3ab.txt 2>&1 && \
SFMCORE_LIB=$PWD/sfm-project_amd/lib/libsfmcore_baprev.so timeout -k 10 200 python tests/perf/ba_bits.py gpurun_out/r3r_bits_prev.npz && \
timeout -k 10 200 python tests/perf/ba_bits.py gpurun_out/r3r_bits_new.npz
