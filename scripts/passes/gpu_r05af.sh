# round 5 pass af: Stack's pair rows' velocity updates (x, y paired) and its
# gripper normals' M^-1 J^T update as v_pk_fma_f32 -- bit-for-bit against
# the 1509ab9 library (lib_prev), then A/B timings of Stack
set -o pipefail
mkdir -p gpurun_out
V=scripts/bin/variants
P=panda-lang-manip_amd/pandasim/libpandasim.so
: > gpurun_out/compare_af.log
timeout -k 10 600 python scripts/compare_libs.py $V/lib_prev.so $P 1024 20 >> gpurun_out/compare_af.log 2>&1 || exit $?
rm -f gpurun_out/ab.log
for r in 1 2 3; do B=65536 TASKS=stack timeout -k 10 300 python scripts/time_variants.py $V/lib_prev.so $P >> gpurun_out/ab.log 2>&1 || exit $?; done
echo "done rc=0"
