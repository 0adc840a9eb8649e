# round 6 pass o: the XCD-aware block order's timing, three builds of the same
# sources: no remap (the round-5 order), remap at 16 lanes only, remap at 8
# and 16 (the product); the order of the builds rotates between rounds
set -o pipefail
mkdir -p gpurun_out
V=scripts/bin/variants
P=panda-lang-manip_amd/pandasim/libpandasim.so
: > gpurun_out/r06o_ab.log
for order in "$V/lib_noremap.so $V/lib_remap16.so $P" "$P $V/lib_noremap.so $V/lib_remap16.so" "$V/lib_remap16.so $P $V/lib_noremap.so"; do
  B=8192 TASKS=push,pick_and_place timeout -k 10 300 python scripts/time_variants.py $order >> gpurun_out/r06o_ab.log 2>&1 || exit $?
  B=4096 TASKS=reach timeout -k 10 300 python scripts/time_variants.py $order >> gpurun_out/r06o_ab.log 2>&1 || exit $?
done
echo "done rc=0"
