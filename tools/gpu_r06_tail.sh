# tail (in-launch PH update) on / off by shard size, plus the final wave's stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06_tail CASES="--scen 10000;--scen 5000;--scen 2500;--scen 1250" ENVS="PHG_TAIL=0;PHG_TAIL=1" REPS=2 bash tools/gpu_run.sh || exit 1
for sc in 10000 1250; do
  PHG_TAIL=1 PHG_TAIL_PROF=1 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --conv-iters 0 --cpu-seconds 0 --scen $sc > gpurun_out/r06_tail/prof_$sc.json 2> gpurun_out/r06_tail/prof_$sc.err || exit 1
  grep PHG_TAIL_PROF gpurun_out/r06_tail/prof_$sc.err | tail -4
done
