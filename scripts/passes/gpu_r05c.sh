# round 5 pass c: the two-waves-per-SIMD experiment build (one-lane Reach and
# Push kernels with M^-1 J^T, candidate records and stash in global memory,
# register-allocated for two waves per SIMD): parity first, then timing
# against the product at 65 536 envs (one wave per SIMD either way) and at
# 131 072 envs (two waves per SIMD where the registers allow), then a kernel
# trace for the resource dump
set -o pipefail
mkdir -p gpurun_out
TW=$PWD/scripts/bin/variants/lib_two_waves.so
PROD=panda-lang-manip_amd/pandasim/libpandasim.so
PANDASIM_LIB=$TW timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -s -k "teacher_forced and (push-ee-1 or reach-ee-1 or push-joints-1)" --timeout 200 --timeout-method thread > gpurun_out/pytest_two_waves.log 2>&1; rc=$?; echo "two-waves pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for b in 65536 131072; do
    echo "== round $r, $b envs" >> gpurun_out/ab_c.log
    B=$b TASKS=push,reach timeout -k 10 300 python scripts/time_variants.py $PROD $TW >> gpurun_out/ab_c.log 2>&1 || exit $?
  done
done
cd /tmp
PANDASIM_LIB=$TW timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -o run -d $GRAFT_REPO_ROOT/gpurun_out/tw_trace -- python $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --batch 131072 > $GRAFT_REPO_ROOT/gpurun_out/tw_trace.log 2>&1 || exit $?
PANDASIM_LIB=$TW timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -o run -d $GRAFT_REPO_ROOT/gpurun_out/tw_sq -- python $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --batch 131072 > $GRAFT_REPO_ROOT/gpurun_out/tw_sq.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -o run -d $GRAFT_REPO_ROOT/gpurun_out/prod_sq -- python $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --batch 131072 > $GRAFT_REPO_ROOT/gpurun_out/prod_sq.log 2>&1 || exit $?
echo "done rc=0"
