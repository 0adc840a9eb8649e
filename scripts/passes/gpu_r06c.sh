# round 6 pass c: the judged contact workloads again (beyond samples dumped to
# gpurun_out/judged/), the substep-by-substep replay of the two 200-step
# 'beyond' samples of pass b (scratch_samples/), and the FLOPS counter
# calibration probe (scripts/flops_probe.hip)
set -o pipefail
mkdir -p gpurun_out
rm -rf gpurun_out/judged
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k judged_contact -v -s --timeout 300 --timeout-method thread > gpurun_out/r06c_pytest_judged.log 2>&1
timeout -k 10 300 python -u scripts/substep_compare.py scratch_samples/pick_and_place_ee_87_15.npz scratch_samples/stack_joints_64_44.npz > gpurun_out/r06c_substep_compare.log 2>&1 || exit $?
cd /tmp && timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU --output-format csv -o run -d $GRAFT_REPO_ROOT/gpurun_out/flops_probe -- $GRAFT_REPO_ROOT/scripts/bin/flops_probe > $GRAFT_REPO_ROOT/gpurun_out/flops_probe.log 2>&1
echo "done rc=$?"
