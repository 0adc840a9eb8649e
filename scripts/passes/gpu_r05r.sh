# round 5 pass r: Stack with the gripper friction rows' M^-1 J^T in the global
# stash (variant stack_fric_mj) -- Stack's GPU tests on it, then A/B timings
set -o pipefail
mkdir -p gpurun_out
V=scripts/bin/variants
PANDASIM_LIB=$PWD/$V/lib_stack_fric_mj.so timeout -k 10 900 python -u -m pytest tests -q -s -m gpu -k "stack or box_on_box or airborne" --timeout 300 --timeout-method thread > gpurun_out/pytest_r.log 2>&1; rc=$?; echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
rm -f gpurun_out/ab.log
for r in 1 2 3; do
  echo "== round $r, 65536 envs" >> gpurun_out/ab.log
  B=65536 TASKS=stack timeout -k 10 300 python scripts/time_variants.py panda-lang-manip_amd/pandasim/libpandasim.so $V/lib_stack_fric_mj.so >> gpurun_out/ab.log 2>&1 || exit $?
done
echo "done rc=0"
