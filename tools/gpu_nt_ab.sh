R=${GRAFT_REPO_ROOT:-$PWD}; cd $R; mkdir -p gpurun_out
TONK_AMD_LIB=libtonk_amd_nt.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/nt_tests.log 2>&1 &&
NO_TESTS=1 WORKLOADS="cfg3 cfg2" REPS=3 bash tools/gpu_ab_env.sh s13 base: nt:TONK_AMD_LIB=libtonk_amd_nt.so
