# round 6 pass ac: the group-vs-one-lane test at 1 000 envs too (the XCD
# block order's tiles and its ragged tail)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -s -k "group_kernels_match_one_lane" --timeout 300 --timeout-method thread > gpurun_out/r06ac_pytest.log 2>&1
echo "done rc=$?"
