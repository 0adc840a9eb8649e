# round 6 pass d: the product library (sources of this commit) bit for bit
# against the round-5 library (1-, 8- and 16-lane kernels); the G = 2 experiment
# (scripts/bin/variants/lib_g2.so: two lanes per env, group objects at two waves
# per SIMD): teacher-forced parity, Push timing at 65 536 and 131 072 envs
# against the product's one-lane kernel, and its SQ_WAVES / busy-cycle counters
set -o pipefail
mkdir -p gpurun_out
V=scripts/bin/variants
P=panda-lang-manip_amd/pandasim/libpandasim.so
: > gpurun_out/r06d_compare.log
timeout -k 10 600 python scripts/compare_libs.py $V/lib_r05.so $P 1024 20 >> gpurun_out/r06d_compare.log 2>&1 && LANES=8 timeout -k 10 600 python scripts/compare_libs.py $V/lib_r05.so $P 512 10 >> gpurun_out/r06d_compare.log 2>&1 && LANES=16 timeout -k 10 600 python scripts/compare_libs.py $V/lib_r05.so $P 256 10 >> gpurun_out/r06d_compare.log 2>&1 || exit $?
PANDASIM_LIB=$V/lib_g2.so timeout -k 10 300 python -u scripts/lanes_parity.py 2 push ee > gpurun_out/r06d_g2_parity.log 2>&1
PANDASIM_LIB=$V/lib_g2.so timeout -k 10 300 python -u scripts/lanes_parity.py 2 reach joints >> gpurun_out/r06d_g2_parity.log 2>&1
: > gpurun_out/r06d_g2_ab.log
for B in 65536 131072; do
  for r in 1 2; do
    echo "== B=$B round $r: product one-lane, then G=2" >> gpurun_out/r06d_g2_ab.log
    B=$B TASKS=push LANES=1 timeout -k 10 300 python scripts/time_variants.py $P >> gpurun_out/r06d_g2_ab.log 2>&1 || exit $?
    B=$B TASKS=push LANES=2 timeout -k 10 300 python scripts/time_variants.py $V/lib_g2.so >> gpurun_out/r06d_g2_ab.log 2>&1 || exit $?
  done
done
cd /tmp
for B in 65536 131072; do
  PANDASIM_LIB=$GRAFT_REPO_ROOT/$V/lib_g2.so timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -o run -d $GRAFT_REPO_ROOT/gpurun_out/r06d_g2_sq_$B -- python $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline --batch $B --lanes 2 > $GRAFT_REPO_ROOT/gpurun_out/r06d_g2_sq_$B.log 2>&1 || exit $?
done
echo "done rc=$?"
