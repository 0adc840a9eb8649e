# GPU pass: the bench line at every BASELINE config that fits one GPU
#  and every task at 65 536 envs -> gpurun_out/configs.jsonl;
# LANES="1 8 16" adds a sweep of the step kernel's lanes per env over the
# small-batch configs -> gpurun_out/lanes.jsonl;
# VARIANTS=1 times the experimental builds of scripts/build_variants.py.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
# (a quoted default inside ${CONFIGS:-"..."} would be one word: one run)
ALL="PandaReach-v3:4096 PandaReachJoints-v3:4096 PandaPush-v3:8192 PandaPickAndPlace-v3:8192
     PandaPush-v3:65536 PandaReachDense-v3:65536 PandaReachJoints-v3:65536 PandaPickAndPlace-v3:65536
     PandaSlide-v3:65536 PandaStack-v3:65536 PandaFlip-v3:65536"
for cfg in ${CONFIGS:-$ALL}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --env-id ${cfg%%:*} --batch ${cfg##*:} >> gpurun_out/configs.jsonl 2>>gpurun_out/configs.err || exit $?
done
for lanes in $LANES; do
  for cfg in PandaReach-v3:4096 PandaPush-v3:8192 PandaPickAndPlace-v3:8192 PandaPush-v3:16384; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 --warmup 5 --env-id ${cfg%%:*} --batch ${cfg##*:} \
      --lanes $lanes >> gpurun_out/lanes.jsonl 2>>gpurun_out/lanes.err || exit $?
  done
done
if [ -n "$VARIANTS" ]; then
  TASKS=reach,push,pick_and_place timeout -k 10 600 python scripts/time_variants.py scripts/bin/variants/*.so > gpurun_out/variants.log 2>&1 || exit $?
fi
echo "done rc=0"
