# round 5 pass o: which change moves the in-contact Push sample env 62 --
# the in-contact scenario on four builds (scripts/incontact_probe.py)
set -o pipefail
mkdir -p gpurun_out
V=scripts/bin/variants
for lib in $V/lib_de178e8.so $V/lib_noikrsq.so $V/lib_nobiasfast.so panda-lang-manip_amd/pandasim/libpandasim.so; do
  PANDASIM_LIB=$PWD/$lib timeout -k 10 300 python scripts/incontact_probe.py push ee >> gpurun_out/incontact.log 2>&1 || exit $?
done
echo "done rc=0"
