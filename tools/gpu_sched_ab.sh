# time to PH conv (farmer 10k headline) vs the launch-schedule cadence (PHG_SCHED_EVERY)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/sched; mkdir -p $O
for rep in 1 2; do
  for k in ${KS:-4 8 16}; do
    PHG_SCHED_EVERY=$k timeout -k 10 240 python bench.py --cpu-seconds 0 > $O/k$k.$rep.json 2> $O/k$k.$rep.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/k$k.$rep.json').read()); t=d['time_to_conv']; print('every $k rep $rep', d['value'], d['ms_per_step'], t['seconds'], t['ph_iters'])"
  done
done
