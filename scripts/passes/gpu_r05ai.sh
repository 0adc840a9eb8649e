# round 5 pass ai: the one-lane solver's velocity change as f32x2 pairs
# (VelChange), the gripper friction rows' two dot products side by side and
# the cylinder's inverse inertia product with rows x, y paired (mul_pk)
# -- bit-for-bit against the a5ca20b library (the product; the experiment built as scripts/bin/variants/lib_new.so: 1-, 8-, 16-lane
# kernels), then A/B timings
set -o pipefail
mkdir -p gpurun_out
V=scripts/bin/variants
P=panda-lang-manip_amd/pandasim/libpandasim.so
: > gpurun_out/compare_ai.log
timeout -k 10 600 python scripts/compare_libs.py $P $V/lib_new.so 1024 20 >> gpurun_out/compare_ai.log 2>&1 && LANES=8 timeout -k 10 600 python scripts/compare_libs.py $P $V/lib_new.so 512 10 >> gpurun_out/compare_ai.log 2>&1 && LANES=16 timeout -k 10 600 python scripts/compare_libs.py $P $V/lib_new.so 256 10 >> gpurun_out/compare_ai.log 2>&1 || exit $?
rm -f gpurun_out/ab.log
ROUNDS=3 TASKS=push,pick_and_place,slide,flip,reach,stack LIBS="$P $V/lib_new.so" bash scripts/gpu_ab.sh
