#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/gpu_tests_agent.sh || exit $?
bash scripts/gpu_sync_nb.sh
