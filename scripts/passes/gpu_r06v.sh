# round 6 pass v: what Stack's box-box rows cost -- the phase split of the
# diagnostic build with and without them (timing only, the second is wrong
# physics: scripts/build_variants.py prof_nopair)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r06v_phase.log
timeout -k 10 300 python scripts/phase_profile.py PandaStack-v3 65536 20 >> gpurun_out/r06v_phase.log 2>&1 || exit $?
PANDASIM_PROF_LIB=$GRAFT_REPO_ROOT/scripts/bin/variants/lib_prof_nopair.so timeout -k 10 300 python scripts/phase_profile.py PandaStack-v3 65536 20 >> gpurun_out/r06v_phase.log 2>&1 || exit $?
echo "done rc=0"
