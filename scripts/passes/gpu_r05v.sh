# round 5 pass v: which half of the max/med3 change moves Push -- the previous
# build, residual max only, clamps only, both (the product); Push and the
# small-batch configs, three interleaved rounds
set -o pipefail
mkdir -p gpurun_out
V=scripts/bin/variants
rm -f gpurun_out/ab.log
ROUNDS=3 TASKS=push,pick_and_place,flip LIBS="$V/lib_base.so $V/lib_resmax_only.so $V/lib_clamp_only.so panda-lang-manip_amd/pandasim/libpandasim.so" bash scripts/gpu_ab.sh
