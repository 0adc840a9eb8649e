# round 6 pass w: what the gripper rows cost in the solve -- the phase split of
# the diagnostic build with and without them (timing only, the second is wrong
# physics: scripts/build_variants.py prof_norobot)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r06w_phase.log
for id in PandaPush-v3 PandaPickAndPlace-v3; do
  timeout -k 10 300 python scripts/phase_profile.py $id 65536 20 >> gpurun_out/r06w_phase.log 2>&1 || exit $?
  PANDASIM_PROF_LIB=$GRAFT_REPO_ROOT/scripts/bin/variants/lib_prof_norobot.so timeout -k 10 300 python scripts/phase_profile.py $id 65536 20 >> gpurun_out/r06w_phase.log 2>&1 || exit $?
done
echo "done rc=0"
