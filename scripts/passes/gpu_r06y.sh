# round 6 pass y: contact-aware env packing of the one-lane kernel (k_pack):
# bits against round 5 (1 024 and 8 192 envs, one lane; 16 and 8 lanes
# unchanged), timing at 65 536 envs against round 5 (rotating order)
set -o pipefail
mkdir -p gpurun_out
V=scripts/bin/variants
P=panda-lang-manip_amd/pandasim/libpandasim.so
: > gpurun_out/r06y_compare.log
LANES=1 timeout -k 10 600 python scripts/compare_libs.py $V/lib_r05.so $P 1024 10 >> gpurun_out/r06y_compare.log 2>&1 && LANES=1 timeout -k 10 600 python scripts/compare_libs.py $V/lib_r05.so $P 8000 12 >> gpurun_out/r06y_compare.log 2>&1 && LANES=8 timeout -k 10 600 python scripts/compare_libs.py $V/lib_r05.so $P 1000 10 >> gpurun_out/r06y_compare.log 2>&1 || exit $?
: > gpurun_out/r06y_ab.log
for order in "$V/lib_r05.so $P" "$P $V/lib_r05.so" "$V/lib_r05.so $P"; do
  B=65536 TASKS=push,pick_and_place,stack,slide,flip,reach timeout -k 10 400 python scripts/time_variants.py $order >> gpurun_out/r06y_ab.log 2>&1 || exit $?
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -v -s -k "packing or ragged or teacher_forced" --timeout 300 --timeout-method thread > gpurun_out/r06y_pytest.log 2>&1
echo "done rc=$?"
