#!/bin/bash
# CPU test suite against the ASan + UBSan build of the oracle (SURVEY.md §5 "sanitizers").
# Host code only (GPU sanitizers are not available on the pool).
set -euo pipefail
cd "$(dirname "$0")/.."
make -s -C oracle sanitize
export SFM_ORACLE_LIB=$PWD/oracle/lib/liboracle_san.so
export LD_PRELOAD=$(gcc -print-file-name=libasan.so)
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
python -m pytest tests -q -m "not gpu" -x -p no:cacheprovider "$@"
