# the headline kernel's VALU instruction mix by class (PMC), one rocprofv3 pass
# per counter group (<= 8 SQ + GRBM_GUI_ACTIVE), after listing which of the wanted counters exist
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmc_mix; mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
B="python3 bench.py --steps 10 --warmup 3 --conv-iters 0 --cpu-seconds 0"
pass=0
for grp in "SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_SALU" \
           "SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_ACTIVE_INST_VALU"; do
  pass=$((pass+1)); ok=""
  for c in $grp; do grep -qw "$c" $O/avail.txt && ok="$ok $c"; done
  echo "pass $pass:$ok"
  timeout -s KILL 200 rocprofv3 --pmc $ok GRBM_GUI_ACTIVE --output-format csv -d $O/p$pass -o run -- $B > $O/p$pass.log 2>&1
  rc=$?; echo "pmc pass $pass exit $rc"; [ $rc -eq 0 ] || { tail -5 $O/p$pass.log; exit $rc; }
done
find $O -name "*counter_collection*.csv"
