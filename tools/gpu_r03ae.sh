# Round 3: UC workgroups per scenario (PHG_STREAM_K) at the new theta default
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03ae
mkdir -p $O
for k in 22 20 26 32 22; do
  PHG_COOP=0 PHG_STREAM_K=$k timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --conv-iters 0 --cpu-seconds 0 --case uc > $O/uc_$k.json 2> $O/uc_$k.err || { tail -3 $O/uc_$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/uc_$k.json')); r=d['roofline']; c=d['config']; print('uc K=$k', d['value'], d['ms_per_step'], r.get('pdhg_iters_per_scen_per_step'), r.get('max_pdhg_iters'), c.get('lanes_per_scenario'), r.get('kernel','')[:40])"
done
