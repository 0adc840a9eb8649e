# GPU pass: the parity tests of the 8-lane kernel (and the group-kernel
# tests), then the lanes sweep at the BASELINE small-batch configs
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu -s -rf --timeout 300 --timeout-method thread -k "lanes or ragged or group or -8" > gpurun_out/pytest_lanes8.log 2>&1
rc=$?; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for cfg in "PandaPush-v3 8192 1" "PandaPush-v3 8192 8" "PandaPush-v3 8192 16" "PandaPickAndPlace-v3 8192 8" \
           "PandaReach-v3 4096 8" "PandaReach-v3 4096 16" "PandaPush-v3 4096 8" "PandaPush-v3 4096 16" \
           "PandaPush-v3 16384 8" "PandaPush-v3 16384 1"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --no-cpu-baseline --env-id $1 --batch $2 --lanes $3 >> gpurun_out/lanes8.jsonl 2>/dev/null || exit $?
done
echo "done rc=$?"
