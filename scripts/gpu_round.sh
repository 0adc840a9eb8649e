# GPU pass for a round checkpoint: GPU parity tests, the default bench line
# (with cpu_baseline), then rocprofv3 kernel-trace/stats and separate PMC
# passes (FETCH_SIZE, WRITE_SIZE, SQ counters) of the same bench command.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
ENV_ID=${ENV_ID:-PandaPush-v3}
P="--output-format csv -o run"
BENCH="$R/bench.py --steps 100 --warmup 10 --no-cpu-baseline --env-id $ENV_ID"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -s --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --env-id $ENV_ID > gpurun_out/bench.log 2>&1 && \
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats $P -d $R/gpurun_out/prof_trace -- python $BENCH > $R/gpurun_out/prof_trace.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE $P -d $R/gpurun_out/prof_fetch -- python $BENCH > $R/gpurun_out/prof_fetch.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE $P -d $R/gpurun_out/prof_write -- python $BENCH > $R/gpurun_out/prof_write.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES $P -d $R/gpurun_out/prof_valu -- python $BENCH > $R/gpurun_out/prof_valu.log 2>&1
echo "done rc=$?"
