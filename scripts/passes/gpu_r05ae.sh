# round 5 pass ae: the joint rows' velocity update (and Stack's M^-1 products, column by column) over the lower part of
# M^-1's column as v_pk_fma_f32 pairs -- bit-for-bit against the ceffab0
# library (lib_prev: 1-, 8-, 16-lane kernels), then A/B timings
set -o pipefail
mkdir -p gpurun_out
V=scripts/bin/variants
P=panda-lang-manip_amd/pandasim/libpandasim.so
: > gpurun_out/compare_ae.log
timeout -k 10 600 python scripts/compare_libs.py $V/lib_prev.so $P 1024 20 >> gpurun_out/compare_ae.log 2>&1 && LANES=8 timeout -k 10 600 python scripts/compare_libs.py $V/lib_prev.so $P 512 10 >> gpurun_out/compare_ae.log 2>&1 && LANES=16 timeout -k 10 600 python scripts/compare_libs.py $V/lib_prev.so $P 256 10 >> gpurun_out/compare_ae.log 2>&1 || exit $?
rm -f gpurun_out/ab.log
ROUNDS=3 TASKS=push,pick_and_place,slide,flip,reach,stack LIBS="$V/lib_prev.so $P" bash scripts/gpu_ab.sh
