# round 5 pass aa: the group kernels' (8 and 16 lanes per env) updates of a
# lane's two DoFs as v_pk_fma_f32 and their friction-cone rows as f32x2 pairs
# -- bit-for-bit against 56c1ea7 (1-, 8-, 16-lane kernels), then A/B timings
set -o pipefail
mkdir -p gpurun_out
V=scripts/bin/variants
P=panda-lang-manip_amd/pandasim/libpandasim.so
: > gpurun_out/compare_aa.log
LANES=8 timeout -k 10 600 python scripts/compare_libs.py $V/lib_base.so $P 512 10 >> gpurun_out/compare_aa.log 2>&1 && LANES=16 timeout -k 10 600 python scripts/compare_libs.py $V/lib_base.so $P 256 10 >> gpurun_out/compare_aa.log 2>&1 && timeout -k 10 600 python scripts/compare_libs.py $V/lib_base.so $P 1024 20 >> gpurun_out/compare_aa.log 2>&1 || exit $?
rm -f gpurun_out/ab.log
ROUNDS=3 TASKS=push,reach LIBS="$V/lib_base.so $P" bash scripts/gpu_ab.sh
