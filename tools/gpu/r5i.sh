#!/bin/bash
# Tracks: CAS-retry hooking (one joining round + one confirming round) vs the atomicMin rounds
# (tkold); tracks GPU tests, then the 500 x 4096 graph's build_tracks timing for both builds.
set -o pipefail
mkdir -p gpurun_out/r5i
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_recon.py tests/test_gpu_incremental.py > gpurun_out/r5i/pytest.log 2>&1 || { tail -30 gpurun_out/r5i/pytest.log; exit 1; }
tail -2 gpurun_out/r5i/pytest.log
for v in tkold base base tkold; do
  L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
  echo -n "$v "; SFMCORE_LIB=$L timeout -k 10 300 python tests/perf/tracks_time.py | tee -a gpurun_out/r5i/tracks_$v.jsonl || exit 1
done
