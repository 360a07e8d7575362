#!/bin/bash
# Builds lib/libsfmcore_<name>.so with extra -D flags (kernel-variant A/B timing via SFMCORE_LIB).
set -e -o pipefail
NAME=$1; shift
cd "$(dirname "$0")/../sfm-project_amd"
OUT=lib/variant_$NAME; mkdir -p $OUT
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-gpu-rdc -Wno-unused-function"
for f in capi match_mfma match_l2fr match_hamming ransac ba ba_solve graph tracks triangulate register orb calib; do
  X=""; [ $f = ransac ] && X="-fno-slp-vectorize"
  /opt/rocm/bin/hipcc $FL $X "$@" -c csrc/$f.hip -o $OUT/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/libsfmcore_$NAME.so $OUT/*.o
rm -rf $OUT
echo lib/libsfmcore_$NAME.so
