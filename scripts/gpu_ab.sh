# Interleaved A/B timing of library builds (scripts/time_variants.py) for the
# scheduler-option decisions of pandasim/build.py: ROUNDS passes over LIBS at
# 65 536 envs per task (TASKS), then the small-batch configs -> gpurun_out/ab.log
set -o pipefail
mkdir -p gpurun_out
LIBS=${LIBS:-"panda-lang-manip_amd/pandasim/libpandasim.so $(ls scripts/bin/variants/*.so 2>/dev/null)"}
for r in $(seq ${ROUNDS:-2}); do
  echo "== round $r, 65536 envs" >> gpurun_out/ab.log
  B=65536 TASKS=${TASKS:-push,pick_and_place,slide,flip,reach,stack} timeout -k 10 300 python scripts/time_variants.py $LIBS >> gpurun_out/ab.log 2>&1 || exit $?
  echo "== round $r, C2 reach 4096 / C3-C4 8192 (auto lanes)" >> gpurun_out/ab.log
  B=4096 TASKS=reach timeout -k 10 300 python scripts/time_variants.py $LIBS >> gpurun_out/ab.log 2>&1 || exit $?
  B=8192 TASKS=push,pick_and_place timeout -k 10 300 python scripts/time_variants.py $LIBS >> gpurun_out/ab.log 2>&1 || exit $?
done
echo "done rc=0"
