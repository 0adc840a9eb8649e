# round 5 pass k: fast sqrt / reciprocal in Slide's candidate stream and
# reciprocal-sqrt pivots in the mass-matrix inverse -- the whole GPU suite on
# the product, then interleaved A/B timings against the previous build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/pytest_k.log 2>&1; rc=$?; echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
rm -f gpurun_out/ab.log
ROUNDS=2 TASKS=push,pick_and_place,slide,flip,reach,stack LIBS="scripts/bin/variants/lib_base.so panda-lang-manip_amd/pandasim/libpandasim.so" bash scripts/gpu_ab.sh
