# Whole GPU suite, then the M3 hydro-tree bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cases
timeout -k 10 700 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/gpu_all.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/gpu_all.log | tail -8; [ $rc -eq 0 ] || exit $rc
for S in 2000 500; do
  timeout -k 10 300 python -u bench.py --case hydro --scen $S --conv-time 60 --cpu-seconds 6 > gpurun_out/cases/hydro$S.json 2> gpurun_out/cases/hydro$S.err
  rc=$?; echo "hydro$S exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/cases/hydro$S.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/cases/hydro$S.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],d['config']['pdhg_layout'],r['avg_launch_ms'],r['frac'],r['pdhg_iters_per_scen_per_step'],d.get('time_to_conv'))"
done
