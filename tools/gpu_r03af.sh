# Round 3: farmer launch time vs check interval (the restart / termination check's share of the kernel)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03af
mkdir -p $O
for c in 32 64 128 256; do
  timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 3 --conv-iters 0 --cpu-seconds 0 --check-every $c > $O/f_$c.json 2> $O/f_$c.err || { tail -3 $O/f_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/f_$c.json')); r=d['roofline']; it=r['pdhg_iters_per_scen_per_step']; ms=r['avg_launch_ms']; print('check_every=$c', d['value'], ms, it, r['max_pdhg_iters'], 'us/iter(avg)', round(ms*1e3/it, 4))"
done
