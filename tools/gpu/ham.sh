set -o pipefail
bash tools/gpu/k1.sh ham1 || exit 1
timeout -k 10 200 python tests/perf/hamming_time.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/hamming_k500.json
K=2048 timeout -k 10 300 python tests/perf/hamming_time.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/hamming_k2048.json
