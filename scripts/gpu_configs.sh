# GPU pass: the bench line at every BASELINE config that fits one GPU
# (SURVEY.md §8(d)), plus the default bench line with its CPU baseline.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
for cfg in "PandaReach-v3 4096" "PandaReachJoints-v3 4096" "PandaPush-v3 8192" "PandaPickAndPlace-v3 8192" \
           "PandaPush-v3 65536" "PandaReachDense-v3 65536" "PandaReachJoints-v3 65536" "PandaPickAndPlace-v3 65536" \
           "PandaSlide-v3 65536" "PandaStack-v3 65536" "PandaFlip-v3 65536"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --no-cpu-baseline --env-id $1 --batch $2 >> gpurun_out/configs.jsonl 2>/dev/null || exit $?
done
echo "done rc=$?"
