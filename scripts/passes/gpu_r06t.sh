# round 6 final pass (library f03ef581), part 3 (after profiles/pmc_traffic.json holds every
# config's PMC for this library): the bench at every config (pmc "current" in
# each line), the default bench line again, and the phase split of k_step
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/configs.jsonl gpurun_out/configs.err gpurun_out/phase.log
bash scripts/gpu_configs.sh || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || exit $?
STAGES="phase" PHASE_IDS="PandaPush-v3:65536 PandaStack-v3:65536 PandaPush-v3:8192 PandaReach-v3:4096" bash scripts/gpu_round.sh
