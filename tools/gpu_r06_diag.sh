# round-6 diagnostic: old vs new library at 10k / 5k, and the new library's per-wave split at 10k
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06c; mkdir -p $O
for sc in 10000 5000; do
  for v in old new; do
    if [ $v = old ]; then L=tools/ab/libphg_old.so; else L=mpi-sppy_amd/libphg.so; fi
    PHG_LIB=$PWD/$L timeout -k 10 240 python bench.py --steps 20 --warmup 5 --conv-iters 0 --cpu-seconds 0 --scen $sc > $O/${v}_$sc.json 2> $O/${v}_$sc.err || exit 1
    python3 -c "import json,sys; d=json.loads(open('$O/${v}_$sc.json').read()); r=d['per_rank']; print('$v $sc', d['value'], d['ms_per_step'], r['pdhg_ms_per_step'][0], r['pdhg_iters_per_scen'][0])"
  done
done
PHG_LOCAL_PROF=1 timeout -k 10 240 python bench.py --steps 3 --warmup 1 --conv-iters 0 --cpu-seconds 0 > $O/prof_new.json 2> $O/prof_new.err || exit 1
grep PHG_LOCAL_PROF $O/prof_new.err | tail -3
PHG_LIB=$PWD/tools/ab/libphg_old.so PHG_LOCAL_PROF=1 timeout -k 10 240 python bench.py --steps 3 --warmup 1 --conv-iters 0 --cpu-seconds 0 > $O/prof_old.json 2> $O/prof_old.err || exit 1
grep PHG_LOCAL_PROF $O/prof_old.err | tail -3
