# round 5 pass j: Slide's box-cylinder pick in the cylinder's frame -- the
# Slide GPU tests on the product, then interleaved A/B timings against the
# previous build (scripts/bin/variants/lib_base.so)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -s -m gpu -k "slide" --timeout 300 --timeout-method thread > gpurun_out/pytest_j.log 2>&1; rc=$?; echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
BASE=scripts/bin/variants/lib_base.so
PROD=panda-lang-manip_amd/pandasim/libpandasim.so
rm -f gpurun_out/ab.log
for r in 1 2; do
  echo "== round $r, 65536 envs" >> gpurun_out/ab.log
  B=65536 TASKS=slide,push timeout -k 10 300 python scripts/time_variants.py $BASE $PROD >> gpurun_out/ab.log 2>&1 || exit $?
done
echo "done rc=0"
