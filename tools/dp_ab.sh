set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
echo "== early side stream"; NOPROF=1 bash tools/dp_check.sh dp2 || exit 1
echo "== late side stream"; U2GNN_EARLY_SIDE=0 MODES="none" bash tools/dp_check.sh dp2late || exit 1
echo "== early + 8 HW queues"; GPU_MAX_HW_QUEUES=8 MODES="none overlap" bash tools/dp_check.sh dp2q8 || exit 1
