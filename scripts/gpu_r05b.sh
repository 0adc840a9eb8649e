# round 5 pass b: the contact-state group test, the Stack tiled-stash variant's
# parity (Stack tests) and an interleaved A/B of it against the product
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_contacts.py -q -s -k "in_contact or free_running" --timeout 300 --timeout-method thread > gpurun_out/pytest_b.log 2>&1; rc=$?; echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
PANDASIM_LIB=$PWD/scripts/bin/variants/lib_stack_tiled.so timeout -k 10 600 python -u -m pytest tests -q -s -m gpu -k "stack or box_on_box or airborne" --timeout 300 --timeout-method thread > gpurun_out/pytest_tiled.log 2>&1; rc=$?; echo "tiled pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
LIBS="panda-lang-manip_amd/pandasim/libpandasim.so scripts/bin/variants/lib_stack_tiled.so scripts/bin/variants/lib_two_waves.so" timeout -k 10 600 bash -c 'for r in 1 2; do B=65536 TASKS=stack,push,reach python scripts/time_variants.py $LIBS >> gpurun_out/ab.log 2>&1 || exit $?; done'
echo "done rc=$?"
