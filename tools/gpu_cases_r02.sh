# Round-2 secondary workloads (SURVEY 8(d) M2 sslp, M3 hydro, M4 netdes; M5 uc separately: its
# rocprofv3 runs end in a profiler-teardown segfault): per case FETCH_SIZE and WRITE_SIZE passes
# (separate rocprofv3 runs), traffic per launch, then the bench line that reads it.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/cases_r02
mkdir -p $O
one() {   # name layout args...
  local nm=$1 lay=$2; shift 2
  local B="bench.py --steps 5 --warmup 2 --conv-iters 0 --cpu-seconds 0 $*"
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/$nm/fetch -o run -- python3 $B > $O/$nm.fetch.log 2>&1 || { echo "$nm fetch failed"; tail -5 $O/$nm.fetch.log; return 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/$nm/write -o run -- python3 $B > $O/$nm.write.log 2>&1 || { echo "$nm write failed"; tail -5 $O/$nm.write.log; return 1; }
  python3 tools/traffic_from_pmc.py $O/$nm/fetch/run_counter_collection.csv $O/$nm/write/run_counter_collection.csv $lay $O/${nm}_traffic.json $nm "$*" > /dev/null || return 1
  timeout -k 10 400 python3 -u bench.py --traffic-json $O/${nm}_traffic.json --conv-time 60 --cpu-seconds 6 $* > $O/$nm.json 2> $O/$nm.err || { echo "$nm bench failed"; tail -5 $O/$nm.err; return 1; }
  echo "$nm ok"; head -c 400 $O/$nm.json; echo
}
case "${CASES:-all}" in
  sslp) one sslp block --case sslp --scen 4096 ;;
  *) one sslp block --case sslp --scen 4096 && \
     one netdes block --case netdes --scen 1024 && \
     one hydro mfma --case hydro --scen 20000 ;;
esac
