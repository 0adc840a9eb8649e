# GPU pass: every GPU test, the Push bench line, and the HBM-traffic PMC
# passes (FETCH_SIZE, WRITE_SIZE) of the same bench command
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P="--output-format csv -o run"
BENCH="$R/bench.py --steps 100 --warmup 10 --no-cpu-baseline"
timeout -k 10 900 python -u -m pytest tests -q -m gpu -s -rf --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_push.log 2>&1 && \
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats $P -d $R/gpurun_out/prof_trace -- python $BENCH > $R/gpurun_out/prof_trace.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE $P -d $R/gpurun_out/prof_fetch -- python $BENCH > $R/gpurun_out/prof_fetch.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE $P -d $R/gpurun_out/prof_write -- python $BENCH > $R/gpurun_out/prof_write.log 2>&1
echo "done rc=$?"
