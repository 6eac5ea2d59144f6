set -u
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -2 gpurun_out/gpu_tests.log; if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/gpu_tests.log | head -20; exit $rc; fi
bash tools/ab_bench.sh cur base || exit $?
FFC_LIB_PATH=fastfourierconvolution_amd/libffc_amd_trace.so timeout -k 10 200 python tools/trace_spectral.py > gpurun_out/trace_sp.log 2>&1; grep -v amdgpu.ids gpurun_out/trace_sp.log
