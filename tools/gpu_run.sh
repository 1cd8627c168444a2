# One parameterised GPU runner (replaces round 3's ~40 one-off gpu_r03*.sh scripts).  Run it on the
# box:   gpurun -- 'OUT=gpurun_out/r04x TESTS="tests/test_gpu_parity.py" CASES="farmer;sslp --scen 4096" bash tools/gpu_run.sh'
#
#   OUT     output directory (default gpurun_out/run)
#   TESTS   pytest targets run first (-m gpu); a failure stops the run
#   TESTK   optional pytest -k expression
#   CASES   ';'-separated bench.py argument sets, e.g. "farmer;netdes --scen 1024 --conv-time 60"
#   ENVS    ';'-separated env assignments for an A/B (each CASE runs under each ENV), e.g.
#           "PHG_FOLD=0;PHG_FOLD=1"; empty: one plain run per case
#   REPS    repetitions of each (case, env) pair, interleaved (default 1)
#   BENCH   extra bench.py arguments for every run (default "--conv-iters 0 --cpu-seconds 0")
#   TLIM    time limit per bench run in seconds (default 300)
#   PROF    1: rocprofv3 --kernel-trace --stats of the first case (plain env) into $OUT/prof
# Every step runs under its own timeout; the first failing step ends the run (nothing retried).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/run}
mkdir -p "$OUT"
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TLIM:-900} python -u -m pytest $TESTS -v --timeout 300 --timeout-method thread -m gpu \
      ${TESTK:+-k "$TESTK"} > "$OUT/tests.log" 2>&1
  rc=$?; echo "pytest exit $rc"; grep -E "FAILED|ERROR|passed|failed" "$OUT/tests.log" | tail -20
  [ $rc -eq 0 ] || exit $rc
fi
BENCH=${BENCH:---conv-iters 0 --cpu-seconds 0}
IFS=';' read -ra CS <<< "$CASES"
IFS=';' read -ra ES <<< "${ENVS:-}"
[ ${#ES[@]} -eq 0 ] && ES=("PHG_NONE=0")
for rep in $(seq 1 ${REPS:-1}); do
  ci=0
  for C in "${CS[@]}"; do
    ci=$((ci+1)); ei=0
    for E in "${ES[@]}"; do
      ei=$((ei+1))
      tag="c${ci}_e${ei}_r${rep}"
      env $E timeout -k 10 ${TLIM:-300} python -u bench.py $BENCH $C > "$OUT/$tag.json" 2> "$OUT/$tag.err"
      rc=$?; [ $rc -eq 0 ] || { echo "[$C | $E] exit $rc"; tail -5 "$OUT/$tag.err"; exit $rc; }
      python - "$OUT/$tag.json" "$C" "$E" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline", {})
t = d.get("time_to_conv") or {}
print(f"[{sys.argv[2]} | {sys.argv[3]}] value={d['value']:.6g} ms/step={d['ms_per_step']:.4f} "
      f"launch_ms={r.get('avg_launch_ms')} frac={r.get('frac')} iters={r.get('pdhg_iters_per_scen_per_step')} "
      f"max_iters={r.get('max_pdhg_iters')} conv_s={t.get('seconds')} conv={t.get('conv')}")
PY
    done
  done
done
if [ "${PROF:-0}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 -u bench.py $BENCH ${CS[0]} \
      > "$OUT/prof.log" 2>&1
  rc=$?; echo "rocprofv3 exit $rc"; [ $rc -eq 0 ] || exit $rc
fi
