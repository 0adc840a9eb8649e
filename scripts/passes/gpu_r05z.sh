# round 5 pass z: the one-object kernels' ground friction rows as f32x2 pairs
# and the gripper rows' object velocity updates as v_pk_fma_f32 (Stack keeps
# its scalar rows) -- bit-for-bit against 56c1ea7 (1-, 8-, 16-lane kernels),
# A/B timings, then every -m gpu test, smoke, bench, trace and PMC passes
set -o pipefail
mkdir -p gpurun_out
V=scripts/bin/variants
P=panda-lang-manip_amd/pandasim/libpandasim.so
: > gpurun_out/compare_z.log
timeout -k 10 600 python scripts/compare_libs.py $V/lib_base.so $P 1024 20 >> gpurun_out/compare_z.log 2>&1 && LANES=8 timeout -k 10 600 python scripts/compare_libs.py $V/lib_base.so $P 512 10 >> gpurun_out/compare_z.log 2>&1 && LANES=16 timeout -k 10 600 python scripts/compare_libs.py $V/lib_base.so $P 256 10 >> gpurun_out/compare_z.log 2>&1 || exit $?
grep -q "bit-identical lib_base.so libpandasim.so B=1024" gpurun_out/compare_z.log || { echo "not bit-identical"; exit 1; }
rm -f gpurun_out/ab.log
ROUNDS=2 TASKS=push,pick_and_place,slide,flip,reach,stack LIBS="$V/lib_base.so $P" bash scripts/gpu_ab.sh || exit $?
STAGES="tests smoke bench trace pmc" bash scripts/gpu_round.sh
