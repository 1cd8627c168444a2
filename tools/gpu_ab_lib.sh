# A/B of two builds of libphg.so on one bench case, alternating runs in one call:
#   CASE_ARGS="--case hydro --scen 100000" OLD=tools/ab/libphg_old.so bash tools/gpu_ab_lib.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab; mkdir -p $O
for rep in 1 2; do
  for v in old new; do
    if [ $v = old ]; then L=$OLD; else L=mpi-sppy_amd/libphg.so; fi
    PHG_LIB=$PWD/$L timeout -k 10 240 python bench.py --steps 20 --warmup 5 --conv-iters 0 --cpu-seconds 0 $CASE_ARGS > $O/$v$rep.json 2> $O/$v$rep.err || exit 1
    python3 -c "import json,sys; d=json.loads(open('$O/$v$rep.json').read()); r=d['per_rank']; print('$v$rep', d['value'], d['ms_per_step'], r['pdhg_ms_per_step'][0], r['pdhg_iters_per_scen'][0], 1000*r['pdhg_ms_per_step'][0]/r['pdhg_iters_per_scen'][0])"
  done
done
