set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -s -m gpu -rf --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
PANDASIM_LIB=$PWD/scripts/bin/variants/lib_group_contract.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -s -k "group_kernels_match_one_lane" --timeout 120 --timeout-method thread > gpurun_out/pytest_contract.log 2>&1; rc=$?; echo "contract rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
bash scripts/gpu_pmc_configs.sh
