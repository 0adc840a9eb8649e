# GPU diagnostic pass: per-phase cycle split (diagnostic build) for several
# tasks, then SQ stall counters of the bench command for Push and Stack.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P="--output-format csv -o run"
for t in Push Stack PickAndPlace Reach; do
  timeout -k 10 300 python scripts/phase_profile.py Panda$t-v3 65536 20 >> gpurun_out/phase.log 2>&1 || exit $?
done
cd /tmp
for t in Push Stack; do
  B="$R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --env-id Panda$t-v3"
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VALU $P -d $R/gpurun_out/diag_sq_$t -- python $B > $R/gpurun_out/diag_sq_$t.log 2>&1 || exit $?
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats $P -d $R/gpurun_out/diag_trace_$t -- python $B > $R/gpurun_out/diag_trace_$t.log 2>&1 || exit $?
done
echo "done"
