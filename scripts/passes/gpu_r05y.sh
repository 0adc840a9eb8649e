# round 5 pass y: the ground contacts' friction rows as f32x2 pairs and the
# gripper rows' object velocity updates as v_pk_fma_f32 -- bit-for-bit against
# the previous build (56c1ea7; 1-, 8- and 16-lane kernels), then A/B timings
set -o pipefail
mkdir -p gpurun_out
V=scripts/bin/variants
P=panda-lang-manip_amd/pandasim/libpandasim.so
: > gpurun_out/compare_y.log
timeout -k 10 600 python scripts/compare_libs.py $V/lib_base.so $P 1024 20 >> gpurun_out/compare_y.log 2>&1 && LANES=8 timeout -k 10 600 python scripts/compare_libs.py $V/lib_base.so $P 512 10 >> gpurun_out/compare_y.log 2>&1 && LANES=16 timeout -k 10 600 python scripts/compare_libs.py $V/lib_base.so $P 256 10 >> gpurun_out/compare_y.log 2>&1 || exit $?
rm -f gpurun_out/ab.log
ROUNDS=3 TASKS=push,pick_and_place,slide,flip,reach,stack LIBS="$V/lib_base.so $P" bash scripts/gpu_ab.sh
