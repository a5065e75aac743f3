cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/diag
DIAG_IMPACT=1 timeout -k 10 300 python -u tools/diag_merge.py tools/_variants/libcorro_diag256.so tools/_variants/libcorro_diag1280.so > gpurun_out/diag/impact.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/diag_merge.py tools/_variants/libcorro_diag64.so > gpurun_out/diag/plain.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/diag/impact.log | sort | uniq -c | sort -rn | head; grep -v amdgpu.ids gpurun_out/diag/plain.log | sort | uniq -c | sort -rn | head
