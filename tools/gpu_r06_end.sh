# round 6 end (after the coupling-row change): VALU class-mix passes, the whole GPU suite, the round profile
set -o pipefail
cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/pmc_mix
bash tools/gpu_pmc_mix.sh || exit $?
bash tools/gpu_r06_final.sh
