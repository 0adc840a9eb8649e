# round 5 pass an: experiment -- the gripper rows' J.dv dot products as two
# partial sums (even, odd DoFs; -DPS_EXPERIMENT_SPLIT_DOTS, built from 17471bd
# as scripts/bin/variants/lib_split.so): not bit-identical by design, so only
# A/B timings against the product here
set -o pipefail
mkdir -p gpurun_out
V=scripts/bin/variants
P=panda-lang-manip_amd/pandasim/libpandasim.so
rm -f gpurun_out/ab.log
ROUNDS=3 TASKS=push,pick_and_place,slide,flip,reach LIBS="$P $V/lib_split.so" bash scripts/gpu_ab.sh
