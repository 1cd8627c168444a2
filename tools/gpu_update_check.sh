# PH-update change check: parity tests, the HBM sweep of the update kernels, one default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ph_update_sweep.py gpurun_out/ph_update_sweep.json > gpurun_out/sweep.log 2>&1
rc=$?; echo "sweep exit $rc"; cat gpurun_out/sweep.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --cpu-seconds 0 > gpurun_out/bench_upd.json 2> gpurun_out/bench_upd.err
rc=$?; echo "bench exit $rc"; cut -c1-300 gpurun_out/bench_upd.json; python -c "import json;d=json.load(open('gpurun_out/bench_upd.json'));print(d['roofline_ph_update'], d['roofline']['avg_launch_ms'])"
exit $rc
