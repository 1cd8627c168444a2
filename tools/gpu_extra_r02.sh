# Round-2 bench lines for the remaining SURVEY 8(d) inputs: M1 rho = 0.1, M2 sslp 8 192, M4 netdes
# 4 096, M3 hydro non-uniform trees of 500 and 2 000 leaves (no PMC passes: the kernels' PMC traffic
# is in profiles/cases_r02 for the main sizes).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/extra
mkdir -p $O
run() {  # name args...
  local nm=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > $O/$nm.json 2> $O/$nm.err || { echo "$nm failed"; tail -5 $O/$nm.err; return 1; }
  echo "$nm ok"; head -c 250 $O/$nm.json; echo
}
run farmer_rho01 --rho 0.1 --cpu-seconds 6 && \
run sslp8192 --case sslp --scen 8192 --conv-iters 0 --cpu-seconds 0 && \
run netdes4096 --case netdes --scen 4096 --conv-iters 0 --cpu-seconds 0 && \
run hydro500 --case hydro --scen 500 --cpu-seconds 6 && \
run hydro2000 --case hydro --scen 2000 --cpu-seconds 6
