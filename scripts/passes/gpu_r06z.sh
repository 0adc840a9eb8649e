# round 6 pass z: env packing on and off in the same library -- the open row
# gates per wave (diagnostic build) and the step time (product)
set -o pipefail
mkdir -p gpurun_out
P=panda-lang-manip_amd/pandasim/libpandasim.so
: > gpurun_out/r06z_phase.log
for id in PandaStack-v3 PandaPush-v3; do
  for pk in 1 0; do
    echo "== $id packing $pk" >> gpurun_out/r06z_phase.log
    PACKING=$pk timeout -k 10 300 python scripts/phase_profile.py $id 65536 20 >> gpurun_out/r06z_phase.log 2>&1 || exit $?
  done
done
: > gpurun_out/r06z_ab.log
for r in 1 2; do
  for pk in 1 0; do
    echo "== packing $pk" >> gpurun_out/r06z_ab.log
    PACKING=$pk B=65536 TASKS=push,stack,slide timeout -k 10 400 python scripts/time_variants.py $P >> gpurun_out/r06z_ab.log 2>&1 || exit $?
  done
done
echo "done rc=0"
