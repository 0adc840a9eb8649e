# round 6 pass a: Stack's global stash without rewritten zero rows (pair and
# gripper slots past the env's dirty counts) and without the split rows;
# bit-for-bit against the round-5 library (lib_r05 = 3f1eb78's sources),
# Stack/Push timing A/B, Stack PMC at 65 536 envs, the reference's own
# seed_test.py / envs_test.py on the GPU, the judged contact workloads
# (Stack stack_push, Flip push), and the box's counter list
set -o pipefail
mkdir -p gpurun_out
V=scripts/bin/variants
P=panda-lang-manip_amd/pandasim/libpandasim.so
: > gpurun_out/r06a_compare.log
timeout -k 10 600 python scripts/compare_libs.py $V/lib_r05.so $P 1024 20 >> gpurun_out/r06a_compare.log 2>&1 && LANES=8 timeout -k 10 600 python scripts/compare_libs.py $V/lib_r05.so $P 512 10 >> gpurun_out/r06a_compare.log 2>&1 || exit $?
rm -f gpurun_out/ab.log
for r in 1 2; do
  B=65536 TASKS=stack,push timeout -k 10 300 python scripts/time_variants.py $V/lib_r05.so $P >> gpurun_out/ab.log 2>&1 || exit $?
done
cp gpurun_out/ab.log gpurun_out/r06a_ab.log
PMC_CONFIGS="PandaStack-v3:65536" bash scripts/gpu_pmc_configs.sh || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_reference_suite.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r06a_pytest_refsuite.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k judged_contact -v -s --timeout 300 --timeout-method thread > gpurun_out/r06a_pytest_judged.log 2>&1
cd /tmp && timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/r06a_counters.txt 2>&1
echo "done rc=$?"
