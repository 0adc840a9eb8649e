# where a step kernel's wave-cycles go (issue vs waits) and its instruction-
# cache behaviour: two PMC passes over a short bench of ENV_ID x BATCH
# -> gpurun_out/stall_{sq,sqc}/ (scripts/summarize_stalls.py reads them)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
ENV_ID=${ENV_ID:-PandaPush-v3}
BATCH=${BATCH:-65536}
TAG=${TAG:-push}
BENCH="$R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --env-id $ENV_ID --batch $BATCH"
P="--output-format csv -o run"
cd /tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_IFETCH $P -d $R/gpurun_out/stall_sq_$TAG -- python $BENCH > $R/gpurun_out/stall_sq_$TAG.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES $P -d $R/gpurun_out/stall_sqc_$TAG -- python $BENCH > $R/gpurun_out/stall_sqc_$TAG.log 2>&1 || exit $?
echo "done rc=0"
