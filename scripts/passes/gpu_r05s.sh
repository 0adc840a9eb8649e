# round 5 pass s: IEEE mode off (-fno-honor-nans -mno-amdgpu-ieee, variant
# ieee_off) -- the whole GPU suite on it, then A/B timings against the product
set -o pipefail
mkdir -p gpurun_out
V=scripts/bin/variants
PANDASIM_LIB=$PWD/$V/lib_ieee_off.so timeout -k 10 1000 python -u -m pytest tests -q -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_s.log 2>&1; rc=$?; echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
rm -f gpurun_out/ab.log
ROUNDS=2 TASKS=push,pick_and_place,slide,flip,reach,stack LIBS="panda-lang-manip_amd/pandasim/libpandasim.so $V/lib_ieee_off.so" bash scripts/gpu_ab.sh
