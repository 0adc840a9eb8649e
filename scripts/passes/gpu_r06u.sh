# round 6 final pass (library f03ef581), part 3b: the phase split of k_step
# (the diagnostic build rebuilt for these sources)
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/phase.log
STAGES="phase" PHASE_IDS="PandaPush-v3:65536 PandaStack-v3:65536 PandaPush-v3:8192 PandaReach-v3:4096" bash scripts/gpu_round.sh
