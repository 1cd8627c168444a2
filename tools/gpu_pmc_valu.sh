# VALU issue profile of the default bench workload: one rocprofv3 PMC pass (SQ + GRBM counters),
# per-dispatch CSV under gpurun_out/prof/valu
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
B="python3 bench.py --steps ${STEPS:-10} --warmup ${WARMUP:-3} --conv-iters 0 --cpu-seconds 0 ${BENCH_ARGS:-}"
timeout -s KILL 200 rocprofv3 --pmc ${COUNTERS:-SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 GRBM_GUI_ACTIVE GRBM_COUNT} --output-format csv -d gpurun_out/prof/valu -o run -- $B > gpurun_out/prof/valu.log 2>&1
rc=$?; echo "pmc exit $rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/prof/valu.log; exit $rc; }
find gpurun_out/prof/valu -name "*.csv"
