# round-6 diagnostic 2: the new library's launch time vs scenarios, and a kernel trace at 10k
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06d; mkdir -p $O
for sc in 6000 8000 10000 12000; do
  timeout -k 10 240 python bench.py --steps 10 --warmup 3 --conv-iters 0 --cpu-seconds 0 --scen $sc > $O/new_$sc.json 2> $O/new_$sc.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('$O/new_$sc.json').read()); r=d['per_rank']; print('new $sc', d['value'], d['ms_per_step'], r['pdhg_ms_per_step'][0], r['pdhg_iters_per_scen'][0])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 3 --conv-iters 0 --cpu-seconds 0 > $O/prof.log 2>&1 || exit 1
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
head -12 $O/kernel_stats.csv
