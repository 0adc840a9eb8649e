# round 6 pass l: the final tree (library e62ece47, source stamp 43beaf54):
# every -m gpu test, smoke, the default bench line
STAGES="tests smoke bench" bash scripts/gpu_round.sh
