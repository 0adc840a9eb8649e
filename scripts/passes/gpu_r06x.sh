# round 6 pass x: per-env PGS iterations and contact slots (diagnostic build):
# would dealing envs to waves by last step's contact slots cut the solve?
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r06x_iter_dump.log
for id in PandaPush-v3 PandaStack-v3; do
  timeout -k 10 300 python scripts/iter_dump.py $id 65536 16 >> gpurun_out/r06x_iter_dump.log 2>&1 || exit $?
done
echo "done rc=0"
