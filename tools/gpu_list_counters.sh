cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/r03t; timeout -k 10 120 rocprofv3 -L > gpurun_out/r03t/counters.txt 2>&1; echo rc=$?; grep -c . gpurun_out/r03t/counters.txt
