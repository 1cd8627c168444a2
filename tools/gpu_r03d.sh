# Round 3: the full -m gpu suite, the default bench line, the PH-update sweep (incl. the folded
# update), then the UC run under rocprofv3 with faulthandler (the r02 profiler-teardown segfault).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03d
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/r03d/tests.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03d/tests.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --cpu-seconds 10 > gpurun_out/r03d/bench.json 2> gpurun_out/r03d/bench.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/r03d/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac']); print(json.dumps(d['roofline_ph_update'])); print(json.dumps(d['time_to_conv']))"
timeout -k 10 400 python -u tools/ph_update_sweep.py gpurun_out/r03d/sweep.json > gpurun_out/r03d/sweep.log 2>&1 || exit $?
cat gpurun_out/r03d/sweep.log
export PYTHONFAULTHANDLER=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03d/uc_trace -o run -- python3 -X faulthandler bench.py --case uc --steps 3 --warmup 1 --conv-iters 0 --cpu-seconds 0 > gpurun_out/r03d/uc_trace.log 2>&1
echo "uc rocprof exit $?"; tail -30 gpurun_out/r03d/uc_trace.log
