# UC (configs[4]) bench line, kernel trace and HBM traffic passes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/uc
export TMPDIR=/tmp
B="bench.py --case uc --steps 3 --warmup 1 --conv-iters 0 --cpu-seconds ${CPU_S:-0}"
timeout -k 10 240 python3 -u $B > gpurun_out/uc/bench.json 2> gpurun_out/uc/bench.err || exit 1
echo bench ok
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/uc/trace -o run -- python3 $B > gpurun_out/uc/trace.log 2>&1 || exit 1
echo trace ok
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/uc/fetch -o run -- python3 $B > gpurun_out/uc/fetch.log 2>&1 || exit 1
echo fetch ok
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/uc/write -o run -- python3 $B > gpurun_out/uc/write.log 2>&1 || exit 1
echo write ok
find gpurun_out/uc -name "*.csv"
