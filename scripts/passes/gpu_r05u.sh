# round 5 pass u: the solver's residual max as llvm.maximum and its clamps as
# v_med3 -- bit-for-bit against the previous build (scripts/compare_libs.py,
# one-lane and 8-lane kernels), then A/B timings
set -o pipefail
mkdir -p gpurun_out
V=scripts/bin/variants
P=panda-lang-manip_amd/pandasim/libpandasim.so
: > gpurun_out/compare_u2.log
LANES=8 timeout -k 10 600 python scripts/compare_libs.py $V/lib_base.so $P 512 10 >> gpurun_out/compare_u2.log 2>&1 && LANES=16 timeout -k 10 600 python scripts/compare_libs.py $V/lib_base.so $P 256 10 >> gpurun_out/compare_u2.log 2>&1 || exit $?
rm -f gpurun_out/ab.log
ROUNDS=2 TASKS=push,pick_and_place,slide,flip,reach,stack LIBS="$V/lib_base.so $P" bash scripts/gpu_ab.sh
