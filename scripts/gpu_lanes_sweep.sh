# GPU pass: bench lines of the step kernel with 1 and 16 lanes per env over
# the small-batch BASELINE configs and around the auto threshold.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "PandaReach-v3 4096" "PandaReachJoints-v3 4096" "PandaPush-v3 8192" "PandaPickAndPlace-v3 8192" \
           "PandaPush-v3 2048" "PandaPush-v3 16384" "PandaPush-v3 32768"; do
  set -- $cfg
  for lanes in 1 16; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-40} --warmup 5 --env-id $1 --batch $2 \
      --lanes $lanes >> gpurun_out/lanes.jsonl 2>>gpurun_out/lanes.err || exit $?
  done
done
echo "done rc=$?"
