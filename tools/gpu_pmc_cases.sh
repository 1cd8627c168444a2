# PMC passes for the secondary workloads (one counter group per rocprofv3 run):
#   * MFMA utilisation of the shared-matrix kernel (hydro tree, MFMA layout)
#   * VALU / issue counters of the farmer lane-local kernel
#   * FETCH_SIZE / WRITE_SIZE of the block-kernel cases (sslp, netdes)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
run() {   # name counters bench-args...
  local name=$1; shift; local ctr=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc/$name -o run -- python3 bench.py --steps 5 --warmup 2 --conv-iters 0 --cpu-seconds 0 "$@" > gpurun_out/pmc/$name.log 2>&1
  local rc=$?; echo "$name exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc/$name.log; exit $rc; }
}
run mfma_hydro "SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE" --case hydro --scen 20000 --layout mfma
run valu_farmer "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for c in "sslp --scen 4096" "netdes --scen 1024"; do
  set -- $c
  run fetch_$1 FETCH_SIZE --case $c
  run write_$1 WRITE_SIZE --case $c
done
find gpurun_out/pmc -name "*counter_collection.csv"
