# round 5 pass ao: Slide's inverse-inertia product packed only in the solver
# loop's velocity updates (inv_inertia_pk; setup keeps the scalar product) --
# bit-for-bit against the product (variant scripts/bin/variants/lib_new.so),
# then A/B timings of Slide and Push
set -o pipefail
mkdir -p gpurun_out
V=scripts/bin/variants
P=panda-lang-manip_amd/pandasim/libpandasim.so
: > gpurun_out/compare_ao.log
timeout -k 10 600 python scripts/compare_libs.py $P $V/lib_new.so 1024 20 >> gpurun_out/compare_ao.log 2>&1 && LANES=8 timeout -k 10 600 python scripts/compare_libs.py $P $V/lib_new.so 512 10 >> gpurun_out/compare_ao.log 2>&1 && LANES=16 timeout -k 10 600 python scripts/compare_libs.py $P $V/lib_new.so 256 10 >> gpurun_out/compare_ao.log 2>&1 || exit $?
rm -f gpurun_out/ab.log
for r in 1 2 3; do B=65536 TASKS=slide,push timeout -k 10 300 python scripts/time_variants.py $P $V/lib_new.so >> gpurun_out/ab.log 2>&1 || exit $?; done
echo "done rc=0"
