# round 5 pass n: rim-point culling in Slide's box-cylinder stream, 1-ulp
# damping norms in the bias forces, (the rsq IK pivots dropped again) -- the whole GPU suite on
# the product (classifier counts printed), then A/B timings of the round-5
# head, the previous commit and the product
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -q -s -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/pytest_n.log 2>&1; rc=$?; echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
rm -f gpurun_out/ab.log
V=scripts/bin/variants
ROUNDS=2 TASKS=push,pick_and_place,slide,flip,reach,stack LIBS="$V/lib_head.so $V/lib_de178e8.so panda-lang-manip_amd/pandasim/libpandasim.so" bash scripts/gpu_ab.sh
