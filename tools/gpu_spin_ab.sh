REPS=3 bash tools/gpu_tonk_rep.sh spin8 &&
for s in 8 64; do TONK_AMD_SPINNERS=$s timeout -k 10 400 python bench.py --workload capi > gpurun_out/capi_spin$s.json 2> gpurun_out/capi_spin$s.err || exit 1; done
