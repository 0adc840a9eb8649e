# GPU pass for group-kernel experiments: the group parity tests on the product
# library, then scripts/time_variants.py over the product and every build in
# scripts/bin/variants/ at the small-batch configs with 16 and 8 lanes per env
# -> gpurun_out/group_variants.log
set -o pipefail
mkdir -p gpurun_out
LIBS="panda-lang-manip_amd/pandasim/libpandasim.so $(ls scripts/bin/variants/*.so 2>/dev/null)"
[ -n "$NO_TESTS" ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -rf --timeout 120 --timeout-method thread \
  -k "group_kernels_match or ragged or teacher_forced" > gpurun_out/pytest_group.log 2>&1 || exit $?
for lanes in 16 8; do
  echo "== lanes $lanes, 4096 envs" >> gpurun_out/group_variants.log
  B=4096 LANES=$lanes TASKS=reach,push timeout -k 10 300 python scripts/time_variants.py $LIBS >> gpurun_out/group_variants.log 2>&1 || exit $?
  echo "== lanes $lanes, 8192 envs" >> gpurun_out/group_variants.log
  B=8192 LANES=$lanes TASKS=push,pick_and_place timeout -k 10 300 python scripts/time_variants.py $LIBS >> gpurun_out/group_variants.log 2>&1 || exit $?
done
echo "done rc=0"
