set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_suite.sh r04b tests/test_gpu_parity.py tests/test_gpu_scale.py; rc=$?
[ $rc -le 1 ] || exit $rc
BRAX_AMD_LIB=brax_amd/_lib_stamps/libbrax_amd.so timeout -k 10 120 python tools/stamps.py ant > gpurun_out/stamps_r04b_ant.log 2>&1 || exit 5
BRAX_AMD_LIB=brax_amd/_lib_stamps/libbrax_amd.so timeout -k 10 120 python tools/stamps.py humanoid > gpurun_out/stamps_r04b_humanoid.log 2>&1 || exit 5
BRAX_AMD_LIB=brax_amd/_lib_mstamps/libbrax_amd.so timeout -k 10 120 python tools/mstamps.py 0 > gpurun_out/mstamps_r04b_0.log 2>&1 || exit 6
BRAX_AMD_LIB=brax_amd/_lib_mstamps/libbrax_amd.so timeout -k 10 120 python tools/mstamps.py 36 > gpurun_out/mstamps_r04b_36.log 2>&1 || exit 6
bash tools/run_prof.sh r04b || exit 7
exit $rc
