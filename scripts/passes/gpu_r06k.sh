# round 6 pass k: group solver motor sweep with the next row's product formed from a pre-update broadcast (bit-identical expected at 1, 8 and 16 lanes), C2-C4 A/B
set -o pipefail
mkdir -p gpurun_out
V=scripts/bin/variants
P=panda-lang-manip_amd/pandasim/libpandasim.so
: > gpurun_out/r06k_compare.log
timeout -k 10 600 python scripts/compare_libs.py $V/lib_r05.so $P 1024 10 >> gpurun_out/r06k_compare.log 2>&1 && LANES=16 timeout -k 10 600 python scripts/compare_libs.py $V/lib_r05.so $P 256 10 >> gpurun_out/r06k_compare.log 2>&1 && LANES=8 timeout -k 10 600 python scripts/compare_libs.py $V/lib_r05.so $P 512 10 >> gpurun_out/r06k_compare.log 2>&1 || exit $?
: > gpurun_out/r06k_ab.log
for r in 1 2 3; do
  B=8192 TASKS=push,pick_and_place timeout -k 10 300 python scripts/time_variants.py $V/lib_r05.so $P >> gpurun_out/r06k_ab.log 2>&1 || exit $?
  B=4096 TASKS=reach timeout -k 10 300 python scripts/time_variants.py $V/lib_r05.so $P >> gpurun_out/r06k_ab.log 2>&1 || exit $?
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_envs.py tests/test_gpu_contacts.py -v -s -k "group or lanes or ragged or config_size or teacher_forced or work_lists" --timeout 300 --timeout-method thread > gpurun_out/r06k_pytest.log 2>&1
echo "done rc=$?"
