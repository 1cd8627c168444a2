# hydro non-uniform trees: bench lines of the MFMA vs the gather layout at several sizes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for S in ${SIZES:-2000 20000}; do
for L in ${LAYOUTS:-mfma gather}; do
  timeout -k 10 200 python -u bench.py --case hydro --scen $S --layout $L --conv-iters ${CONV_ITERS:-0} --cpu-seconds 0 > gpurun_out/hydro_${L}_$S.json 2> gpurun_out/hydro_${L}_$S.err
  rc=$?; [ $rc -eq 0 ] || { echo "$L $S exit $rc"; tail -5 gpurun_out/hydro_${L}_$S.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/hydro_${L}_$S.json')); r=d['roofline']; print('$L', $S, d['value'], d['ms_per_step'], r['avg_launch_ms'], r['bound'], r['frac'], r.get('executed_tflops'), r['pdhg_iters_per_scen_per_step'], r['max_pdhg_iters'], d.get('time_to_conv',{}).get('seconds'), d.get('time_to_conv',{}).get('ph_iters'))"
done
done
