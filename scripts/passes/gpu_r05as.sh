# round 5 pass as: Stack's ground friction rows as f32x2 pairs with |f|^2
# contracted as Stack's scalar rows had it (fma(a, a, b b)) -- bit-for-bit
# against the product (variant scripts/bin/variants/lib_new.so), then A/B
# timings of Stack
set -o pipefail
mkdir -p gpurun_out
V=scripts/bin/variants
P=panda-lang-manip_amd/pandasim/libpandasim.so
: > gpurun_out/compare_as.log
timeout -k 10 600 python scripts/compare_libs.py $P $V/lib_new.so 1024 20 >> gpurun_out/compare_as.log 2>&1 || exit $?
rm -f gpurun_out/ab.log
for r in 1 2 3; do B=65536 TASKS=stack timeout -k 10 300 python scripts/time_variants.py $P $V/lib_new.so >> gpurun_out/ab.log 2>&1 || exit $?; done
echo "done rc=0"
