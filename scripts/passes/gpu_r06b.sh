# round 6 pass b: Stack's solver reads a shared zero block for the pair and
# gripper slots an env does not use (no zero rows written or read per env);
# bit-for-bit against the round-5 library, Stack/Push A/B, Stack PMC at
# 65 536 envs, the judged contact workloads, and the 200-step teacher forcing
# with its beyond samples printed and dumped (gpurun_out/tf200/)
set -o pipefail
mkdir -p gpurun_out
V=scripts/bin/variants
P=panda-lang-manip_amd/pandasim/libpandasim.so
: > gpurun_out/r06b_compare.log
timeout -k 10 600 python scripts/compare_libs.py $V/lib_r05.so $P 1024 20 >> gpurun_out/r06b_compare.log 2>&1 || exit $?
rm -f gpurun_out/ab.log
for r in 1 2; do
  B=65536 TASKS=stack,push timeout -k 10 300 python scripts/time_variants.py $V/lib_r05.so $P >> gpurun_out/ab.log 2>&1 || exit $?
done
cp gpurun_out/ab.log gpurun_out/r06b_ab.log
PMC_CONFIGS="PandaStack-v3:65536" bash scripts/gpu_pmc_configs.sh || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k judged_contact -v -s --timeout 300 --timeout-method thread > gpurun_out/r06b_pytest_judged.log 2>&1
rm -rf gpurun_out/tf200
timeout -k 10 900 python -u -m pytest tests/test_gpu_contacts.py -k teacher_forced_200 -v -s --timeout 300 --timeout-method thread > gpurun_out/r06b_pytest_tf200.log 2>&1
echo "done rc=$?"
