# Whole GPU suite, then one bench line per argument set in $AB (';'-separated), with time-to-conv.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/gpu_all.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -15 gpurun_out/gpu_all.log
[ $rc -eq 0 ] || exit $rc
i=0
IFS=';' read -ra SETS <<< "$AB"
for A in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --conv-iters ${CONV_ITERS:-20000} --cpu-seconds 0 $A > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err
  rc=$?; echo "== [$A] exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/ab_$i.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$i.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],r['pdhg_iters_per_scen_per_step'],r['max_pdhg_iters'],d.get('time_to_conv'))"
done
