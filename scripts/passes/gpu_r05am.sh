# round 5 pass am: C2 (Reach and ReachJoints at 4 096 envs) at 8 and 16 lanes
# per env on the f1d930c library (the 8-lane kernels gained the most from
# the packed pairs) -> gpurun_out/lanes.jsonl
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/lanes.jsonl
for r in 1 2; do
  for cfg in PandaReach-v3:4096 PandaReachJoints-v3:4096; do
    for lanes in 16 8; do
      timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 --warmup 10 --env-id ${cfg%%:*} --batch ${cfg##*:} \
        --lanes $lanes >> gpurun_out/lanes.jsonl 2>>gpurun_out/lanes.err || exit $?
    done
  done
done
echo "done rc=0"
