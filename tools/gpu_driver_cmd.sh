# The round-end driver's bench command, run REPS times back to back on one box (its spread).
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R; mkdir -p gpurun_out
TAG=${TAG:-drv}
for i in $(seq 1 ${REPS:-3}); do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || exit $?
  tail -c 300 gpurun_out/${TAG}_$i.json
done
