# The -O3 group-kernel probe: group kernels at -O3 against
# the one-lane kernel, then the row dumps of the -O1 and -O3 group solvers
# for the Slide and Push pairs -> gpurun_out/groups_o3_*.log
set -o pipefail
mkdir -p gpurun_out
V=scripts/bin/variants
PANDASIM_LIB=$V/lib_groups_o3.so timeout -k 10 200 python scripts/group_vs_one_lane.py > gpurun_out/groups_o3_vs_one_lane.log 2>&1 || exit $?
for cfg in "slide joints 16" "slide joints 8" "slide ee 16" "slide ee 8" "push ee 8" "pick_and_place ee 16"; do
  timeout -k 10 200 python scripts/row_dump.py $cfg $V/lib_dump.so $V/lib_groups_o3_dump.so >> gpurun_out/groups_o3_row_dump.log 2>&1 || exit $?
done
echo "done rc=0"
