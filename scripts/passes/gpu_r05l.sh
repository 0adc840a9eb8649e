# round 5 pass l: A/B of the previous build, the Slide-only change and the
# product (Slide change + rsq Cholesky pivots) on the tasks the pivots touch
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/ab.log
V=scripts/bin/variants
ROUNDS=3 TASKS=push,pick_and_place,flip,reach LIBS="$V/lib_head.so $V/lib_slideonly.so panda-lang-manip_amd/pandasim/libpandasim.so" bash scripts/gpu_ab.sh
