# round 5 final pass, per-config PMC (library of d54809d): C2-C4, Slide and
# Stack at 65 536 envs (scripts/gpu_pmc_configs.sh)
set -o pipefail
mkdir -p gpurun_out
PMC_CONFIGS="PandaPush-v3:8192 PandaPickAndPlace-v3:8192 PandaReach-v3:4096 PandaSlide-v3:65536 PandaStack-v3:65536" bash scripts/gpu_pmc_configs.sh
