# round 6 pass j: per-env PGS iteration counts of the one-lane kernel
# (diagnostic build) -- would sorting envs into waves by last step's
# iterations cut the wave's PGS cost?
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r06j_iter_dump.log
for id in PandaPush-v3 PandaPickAndPlace-v3 PandaStack-v3; do
  timeout -k 10 300 python scripts/iter_dump.py $id 65536 24 >> gpurun_out/r06j_iter_dump.log 2>&1 || exit $?
done
echo "done rc=0"
