#!/bin/bash
# bench smoke at cfg3 with the measured K2 executed share + the box's CPU-share evidence
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
(cat /sys/fs/cgroup/cpu.max 2>&1; cat /sys/fs/cgroup/cpuset.cpus.effective 2>&1; nproc; echo OMP=$OMP_NUM_THREADS) > gpurun_out/r3f_cpu.txt
timeout -k 10 600 python bench.py --config cfg3 --steps 10 --warmup 3 --cpu-seconds 8 > gpurun_out/r3f_bench_cfg3.json 2> gpurun_out/r3f_bench.err
