# round 5 pass b: the contact-state group test and the group kernels' parity
# on the product (motor-row chain), the Stack tiled-stash variant's parity,
# and interleaved A/B timings of the experiment builds against the baseline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_contacts.py -q -s -k "group_kernels or free_running or teacher_forced or config_size" --timeout 300 --timeout-method thread > gpurun_out/pytest_b.log 2>&1; rc=$?; echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
PANDASIM_LIB=$PWD/scripts/bin/variants/lib_stack_tiled.so timeout -k 10 600 python -u -m pytest tests -q -s -m gpu -k "stack or box_on_box or airborne" --timeout 300 --timeout-method thread > gpurun_out/pytest_tiled.log 2>&1; rc=$?; echo "tiled pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
BASE=scripts/bin/variants/lib_base.so
PROD=panda-lang-manip_amd/pandasim/libpandasim.so
for r in 1 2; do
  echo "== round $r, 65536 envs" >> gpurun_out/ab.log
  B=65536 TASKS=stack,push,reach timeout -k 10 300 python scripts/time_variants.py $BASE $PROD scripts/bin/variants/lib_stack_tiled.so scripts/bin/variants/lib_two_waves.so >> gpurun_out/ab.log 2>&1 || exit $?
  echo "== round $r, small batches (auto lanes)" >> gpurun_out/ab.log
  B=4096 TASKS=reach timeout -k 10 300 python scripts/time_variants.py $BASE $PROD >> gpurun_out/ab.log 2>&1 || exit $?
  B=8192 TASKS=push,pick_and_place timeout -k 10 300 python scripts/time_variants.py $BASE $PROD >> gpurun_out/ab.log 2>&1 || exit $?
done
echo "done rc=0"
