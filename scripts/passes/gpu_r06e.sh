# round 6 pass e: phase split of the small-batch group kernels (C2 Reach and
# ReachJoints 4 096 / 16 lanes, C3 Push 8 192 / 8 lanes) and Push 65 536, with
# the mass matrix and its inverse forced out of the candidate code in the
# diagnostic build (so their cycles land in their own phases)
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/phase.log
STAGES="phase" PHASE_IDS="PandaReach-v3:4096 PandaReachJoints-v3:4096 PandaPush-v3:8192 PandaPush-v3:65536" bash scripts/gpu_round.sh
