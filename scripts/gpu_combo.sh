cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/diag_impact.sh; rc=$?; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_agent.sh
