# round 5 pass x: the gripper rows' velocity updates as v_pk_fma_f32 pairs
# (pk_apply) and the friction limits without max(lam_n, 0) -- bit-for-bit
# against the previous build (1-, 8- and 16-lane kernels), then A/B timings of
# the previous build, the limit change alone (variant no_pk) and the product
set -o pipefail
mkdir -p gpurun_out
V=scripts/bin/variants
P=panda-lang-manip_amd/pandasim/libpandasim.so
: > gpurun_out/compare_x.log
timeout -k 10 600 python scripts/compare_libs.py $V/lib_base.so $P 1024 20 >> gpurun_out/compare_x.log 2>&1 && LANES=8 timeout -k 10 600 python scripts/compare_libs.py $V/lib_base.so $P 512 10 >> gpurun_out/compare_x.log 2>&1 && LANES=16 timeout -k 10 600 python scripts/compare_libs.py $V/lib_base.so $P 256 10 >> gpurun_out/compare_x.log 2>&1 || exit $?
rm -f gpurun_out/ab.log
ROUNDS=3 TASKS=push,pick_and_place,slide,flip,reach,stack LIBS="$V/lib_base.so $V/lib_no_pk.so $P" bash scripts/gpu_ab.sh
