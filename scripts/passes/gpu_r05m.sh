# round 5 pass m: the box-box clipping polygons in registers (Stack scratch
# 544 B -> 0 B) -- Stack's GPU tests on the product, then A/B timings
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -s -m gpu -k "stack or box_on_box or airborne" --timeout 300 --timeout-method thread > gpurun_out/pytest_m.log 2>&1; rc=$?; echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
rm -f gpurun_out/ab.log
V=scripts/bin/variants
for r in 1 2 3; do
  echo "== round $r, 65536 envs" >> gpurun_out/ab.log
  B=65536 TASKS=stack,push timeout -k 10 300 python scripts/time_variants.py $V/lib_head.so panda-lang-manip_amd/pandasim/libpandasim.so >> gpurun_out/ab.log 2>&1 || exit $?
done
echo "done rc=0"
