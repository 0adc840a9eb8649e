# GPU pass after a kernel change: GPU parity tests, then bench lines of the
# headline config, Stack, and the small-batch BASELINE configs, and a kernel
# trace of the headline bench.  Each GPU step has its own time limit; a
# crash, abort or time limit ends the call.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${TAG:-perf}
timeout -k 10 600 python -u -m pytest tests -q -m gpu -s -rf --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
for cfg in "PandaPush-v3 65536" "PandaStack-v3 65536" "PandaPickAndPlace-v3 65536" "PandaReach-v3 4096" \
           "PandaPush-v3 8192" "PandaPickAndPlace-v3 8192"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --no-cpu-baseline --env-id $1 --batch $2 >> gpurun_out/${TAG}_configs.jsonl 2>>gpurun_out/${TAG}_bench.err || exit $?
done
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -o run -d $R/gpurun_out/${TAG}_trace -- python $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline > $R/gpurun_out/${TAG}_trace.log 2>&1
echo "done rc=$?"
