# rocprofv3 kernel trace + PMC passes (FETCH_SIZE, WRITE_SIZE, SQ counters,
# FP32 instruction counters) of the bench at each config of $PMC_CONFIGS
# (default: the BASELINE small-batch configs C2-C4 and Stack at 65 536 envs),
# each into gpurun_out/pmc_<env>_<batch>_{trace,fetch,write,valu,fp32}/; run
# through gpurun from the repo root, then on the CPU
#   python scripts/summarize_profiles.py <tag> "<env> x<batch>/gpu" --prefix pmc_<env>_<batch> --steps 40
# Every pass has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
DEFAULT="PandaPush-v3:8192 PandaPickAndPlace-v3:8192 PandaReach-v3:4096 PandaStack-v3:65536"
P="--output-format csv -o run"
run() { echo "[pmc] $*" >&2; "$@" || { rc=$?; echo "[pmc] failed rc=$rc: $*"; exit $rc; }; }
cd /tmp
for cfg in ${PMC_CONFIGS:-$DEFAULT}; do
  id=${cfg%%:*}; b=${cfg##*:}; d=$R/gpurun_out/pmc_${id}_${b}
  BENCH="$R/bench.py --steps 40 --warmup 5 --no-cpu-baseline --env-id $id --batch $b"
  run timeout -k 10 300 rocprofv3 --kernel-trace --stats $P -d ${d}_trace -- python $BENCH > ${d}_trace.log 2>&1
  run timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE $P -d ${d}_fetch -- python $BENCH > ${d}_fetch.log 2>&1
  run timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE $P -d ${d}_write -- python $BENCH > ${d}_write.log 2>&1
  run timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES $P -d ${d}_valu -- python $BENCH > ${d}_valu.log 2>&1
  run timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 $P -d ${d}_fp32 -- python $BENCH > ${d}_fp32.log 2>&1
done
cd $R
echo "done rc=0"
