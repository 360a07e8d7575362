set -o pipefail
# Round 4: PMC HBM traffic of the bench kernels on this round's code (cfg4, cfg3), one counter per pass.
export TMPDIR=/tmp
timeout -k 10 600 bash tools/pmc_traffic.sh r6x_t4 cfg4 > gpurun_out/r6x_t4.log 2>&1 || { tail -8 gpurun_out/r6x_t4.log; exit 1; }
timeout -k 10 400 bash tools/pmc_traffic.sh r6x_t3 cfg3 > gpurun_out/r6x_t3.log 2>&1 || { tail -8 gpurun_out/r6x_t3.log; exit 1; }
python3 -c "import json; [print(c, {k: round(v['hbm_bytes_per_step']/1e9,2) for k,v in json.load(open(f'gpurun_out/r6x_{t}/traffic.json'))['kernels'].items()}) for c,t in (('cfg4','t4'),('cfg3','t3'))]"
