#!/bin/bash
# K1 compiled with the LLVM AMDGPU scheduler strategies (max-ilp, max-memory-clause, iterative-ilp)
# against the default: interleaved k1_time (bench rule, parity sample vs the oracle) at cfg3 and at
# K = 4096 (40 images).
set -o pipefail
mkdir -p gpurun_out/r5l
export PYTHONUNBUFFERED=1 TMPDIR=/tmp K1_ONLY_BENCH_RULE=1
for r in 1 2 3; do
  for v in base ilp memclause itilp; do
    L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
    echo -n "cfg3 $v "; SFMCORE_LIB=$L timeout -k 10 120 python tests/perf/k1_time.py 2>&1 | grep "xc=" || exit 1
    echo -n "k4096 $v "; N_IMG=40 K=4096 SFMCORE_LIB=$L timeout -k 10 120 python tests/perf/k1_time.py 2>&1 | grep "xc=" || exit 1
  done
done | tee gpurun_out/r5l/ab.txt
