set -o pipefail
# Round 5 K1 A/B (interleaved): the group kernel with the LDS column reduction (default library),
# with the reduction consumed one tile later (-DMU_GRP_PIPE), and with round 4's transpose
# (-DMU_GRP_XPOSE), each against round 4's kernel (SFM_K1_GRP=0) in the same process; outputs
# compared bit for bit.
OUT=gpurun_out/q5e; mkdir -p $OUT
L=$PWD/sfm-project_amd/lib
for r in 1 2; do
  timeout -k 10 240 python -u tests/perf/k1_grp_ab.py 2 > $OUT/base_$r.txt 2>&1 || { tail -5 $OUT/base_$r.txt; exit 1; }
  SFMCORE_LIB=$L/libsfmcore_grpp.so timeout -k 10 240 python -u tests/perf/k1_grp_ab.py 2 > $OUT/grpp_$r.txt 2>&1 || { tail -5 $OUT/grpp_$r.txt; exit 1; }
  SFMCORE_LIB=$L/libsfmcore_grpx.so timeout -k 10 240 python -u tests/perf/k1_grp_ab.py 2 > $OUT/grpx_$r.txt 2>&1 || { tail -5 $OUT/grpx_$r.txt; exit 1; }
done
grep -H "median\|identical" $OUT/*.txt
