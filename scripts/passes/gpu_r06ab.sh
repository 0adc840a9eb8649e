# round 6 pass ab: the final tree (library f03ef581, stamp 3bab6899): every
# -m gpu test, smoke, the default bench line
set -o pipefail
mkdir -p gpurun_out
rm -rf gpurun_out/tf200 gpurun_out/judged
STAGES="tests smoke bench" bash scripts/gpu_round.sh
