#!/bin/bash
# Interleaved A/B timing of K1 library variants: tools/ab_k1.sh ROUNDS name1 name2 ...
# ("base" = lib/libsfmcore.so, otherwise lib/libsfmcore_<name>.so).
set -o pipefail
R=$1; shift
for r in $(seq $R); do
  for v in "$@"; do
    L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
    SFMCORE_LIB=$L timeout -k 10 120 python tests/perf/k1_time.py 2>&1 | grep "xc=" | sed "s/^/$v /" || exit 1
  done
done
