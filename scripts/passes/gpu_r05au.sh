# round 5 final pass (library of 37ec464), part 2: per-config PMC passes
# (C2-C4, Slide and Stack at 65 536 envs) and the phase split of k_step
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/phase.log
PMC_CONFIGS="PandaPush-v3:8192 PandaPickAndPlace-v3:8192 PandaReach-v3:4096 PandaSlide-v3:65536 PandaStack-v3:65536" bash scripts/gpu_pmc_configs.sh || exit $?
STAGES="phase" PHASE_IDS="PandaPush-v3:65536 PandaSlide-v3:65536 PandaStack-v3:65536 PandaPush-v3:8192" bash scripts/gpu_round.sh
