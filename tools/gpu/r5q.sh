#!/bin/bash
# Round-3 PMC traffic records (FETCH_SIZE / WRITE_SIZE passes) of the bench's kernels at cfg4 and cfg3.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash tools/pmc_traffic.sh r5q_traffic_cfg4 cfg4 && bash tools/pmc_traffic.sh r5q_traffic_cfg3 cfg3
