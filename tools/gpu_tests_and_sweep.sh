R=${GRAFT_REPO_ROOT:-$PWD}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_hdr.log 2>&1 &&
NO_TESTS=1 WORKLOADS="cfg3 cfg2" REPS=2 bash tools/gpu_ab_env.sh s4 base: ch32:TONK_AMD_CHUNK=32 ch128:TONK_AMD_CHUNK=128 in1:TONK_AMD_INLINE_SEG=1 in8:TONK_AMD_INLINE_SEG=8
