# round 6 final pass (library f03ef581), part 2: per-config PMC passes (trace, FETCH_SIZE,
# WRITE_SIZE, SQ, FLOPS) of the BASELINE small-batch configs and of every
# task at 65 536 envs but Push (part 1), in two halves (CONFIG_HALF=1|2)
set -o pipefail
mkdir -p gpurun_out
if [ "$CONFIG_HALF" = 1 ]; then
  PMC_CONFIGS="PandaReach-v3:4096 PandaReachJoints-v3:4096 PandaPush-v3:8192 PandaPickAndPlace-v3:8192 PandaStack-v3:65536" bash scripts/gpu_pmc_configs.sh
else
  PMC_CONFIGS="PandaPickAndPlace-v3:65536 PandaSlide-v3:65536 PandaFlip-v3:65536 PandaReachDense-v3:65536 PandaReachJoints-v3:65536" bash scripts/gpu_pmc_configs.sh
fi
