# Round profile: kernel-trace stats + FETCH/WRITE PMC passes of the default bench workload,
# traffic per launch from the PMC passes, then the full default bench line using that traffic.
set -o pipefail
cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof
PMC=1 bash tools/gpu_profile.sh || exit $?
F=$(find gpurun_out/prof/fetch -name "*counter_collection.csv" | head -1)
W=$(find gpurun_out/prof/write -name "*counter_collection.csv" | head -1)
python tools/trace_summary.py gpurun_out/prof/trace/run_kernel_trace.csv ${STEPS:-20} gpurun_out/trace_summary.json ${WARMUP:-5} || exit $?
python tools/traffic_from_pmc.py "$F" "$W" ${LAYOUT:-local} gpurun_out/traffic.json || exit $?
timeout -k 10 600 python -u bench.py --traffic-json gpurun_out/traffic.json ${BENCH_ARGS:-} > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc=$?; echo "bench exit $rc"; tail -3 gpurun_out/bench_full.err; cat gpurun_out/bench_full.json; exit $rc
