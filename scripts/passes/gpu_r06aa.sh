# round 6 pass aa: env packing on and off at batches of more waves than SIMDs
# (131 072 and 262 144 envs: two and four waves per SIMD in turn)
set -o pipefail
mkdir -p gpurun_out
P=panda-lang-manip_amd/pandasim/libpandasim.so
: > gpurun_out/r06aa_ab.log
for B in 131072 262144; do
  for r in 1 2; do
    for pk in 1 0; do
      echo "== B $B packing $pk" >> gpurun_out/r06aa_ab.log
      PACKING=$pk B=$B TASKS=push,stack timeout -k 10 400 python scripts/time_variants.py $P >> gpurun_out/r06aa_ab.log 2>&1 || exit $?
    done
  done
done
echo "done rc=0"
