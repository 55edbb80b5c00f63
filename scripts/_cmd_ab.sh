set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/ab_env.sh gpurun_out/colwg SDP_ES_COL_WG "3 4 6 8 12" 2 || exit $?
echo done
