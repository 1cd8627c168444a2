# rocprofv3 kernel-trace summary + separate PMC passes (FETCH_SIZE, WRITE_SIZE) of a short bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
B="python3 bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} --conv-iters 0 --cpu-seconds 0 ${BENCH_ARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- $B > gpurun_out/prof/trace.log 2>&1
rc=$?; echo "trace exit $rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/prof/trace.log; exit $rc; }
if [ -n "${PMC:-}" ]; then
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/fetch -o run -- $B > gpurun_out/prof/fetch.log 2>&1
rc=$?; echo "fetch exit $rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/prof/fetch.log; exit $rc; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/write -o run -- $B > gpurun_out/prof/write.log 2>&1
rc=$?; echo "write exit $rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/prof/write.log; exit $rc; }
fi
find gpurun_out/prof -name "*.csv" | head -20
