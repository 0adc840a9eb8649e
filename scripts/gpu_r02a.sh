# GPU pass: the whole GPU suite on the product library, the teacher-forced
# parity tests again on the IEEE-mode-off build, then the
# bench line.  A failing test still lets the next steps run; a crash, abort or
# time limit ends the call there.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
PY="python -u -m pytest -q -s -rf --timeout 300 --timeout-method thread"
timeout -k 10 900 $PY tests -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
PANDASIM_LIB=$PWD/panda-lang-manip_amd/pandasim/libpandasim_ieee_off.so timeout -k 10 600 $PY tests/test_gpu_parity.py -m gpu -k "teacher_forced or sim_step" > gpurun_out/pytest_ieee_off.log 2>&1
rc=$?; echo "pytest ieee_off rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
echo "done rc=$?"
