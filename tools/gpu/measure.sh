set -o pipefail
# PMC traffic (cfg4, cfg3), rocprofv3 kernel stats of the default bench command, and a 2-rank
# gloo same-GPU rehearsal of the strong-scaling path.  Results under gpurun_out/meas_TAG.
TAG=${1:-m}
O=gpurun_out/meas_$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 bash tools/pmc_traffic.sh meas_$TAG/traffic_cfg4 cfg4 > $O/t4.log 2>&1 || { tail -5 $O/t4.log; exit 1; }
timeout -k 10 300 bash tools/pmc_traffic.sh meas_$TAG/traffic_cfg3 cfg3 > $O/t3.log 2>&1 || { tail -5 $O/t3.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || { tail -5 $O/prof_bench.err; exit 1; }
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/prof/run_kernel_stats.csv')))[:12]: print(r['Name'][:60], r['Calls'], r['AverageNs'], r['Percentage'])"
timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --device 0 --steps 2 --warmup 1 > $O/n2_gloo.json 2> $O/n2_gloo.err || { tail -5 $O/n2_gloo.err; exit 1; }
cat $O/n2_gloo.json
