# round 5 pass g: group kernels with one LDS column per env (shared by the
# group's lanes), at the product's register budget and at two waves per SIMD:
# parity (group tests), then timings at the small-batch configs
set -o pipefail
mkdir -p gpurun_out
V=$PWD/scripts/bin/variants
PROD=panda-lang-manip_amd/pandasim/libpandasim.so
for lib in groups_shared groups_shared_2w; do
  PANDASIM_LIB=$V/lib_$lib.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_contacts.py -q -s -k "group_kernels or (teacher_forced and (-16] or -8])) or ragged or work_lists or config_size" --timeout 300 --timeout-method thread > gpurun_out/pytest_$lib.log 2>&1; rc=$?; echo "$lib pytest rc=$rc"
  [ $rc -le 1 ] || exit $rc
done
for r in 1 2; do
  for lanes in 16 8; do
    echo "== round $r, lanes $lanes" >> gpurun_out/ab_g.log
    LANES=$lanes B=4096 TASKS=reach timeout -k 10 300 python scripts/time_variants.py $PROD $V/lib_groups_shared.so $V/lib_groups_shared_2w.so >> gpurun_out/ab_g.log 2>&1 || exit $?
    LANES=$lanes B=8192 TASKS=push,pick_and_place timeout -k 10 300 python scripts/time_variants.py $PROD $V/lib_groups_shared.so $V/lib_groups_shared_2w.so >> gpurun_out/ab_g.log 2>&1 || exit $?
  done
done
echo "done rc=0"
