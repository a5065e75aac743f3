#!/bin/bash
# Host-side helper (runs here, not on the GPU box): submit one gpurun command, and resubmit it only
# while the pool reports that no box was free (status "transient" with nothing run: no GPU time was
# used). Any call that ran -- passed, failed, timed out -- ends the loop.
#   tools/gpurun_retry.sh TIMEOUT 'OUT=x bash scripts/gpu.sh tests bench' [ATTEMPTS]
cd "$(dirname "$0")/.." || exit 1
T=$1; CMD=$2; N=${3:-8}
for k in $(seq 1 "$N"); do
  timeout $((T + 1500)) /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD"
  rc=$?
  if python3 - <<'EOF'
import json, sys
v = json.load(open("gpurun_out/.last_call.json"))
sys.exit(0 if v.get("status") == "transient" and not v.get("run_s") else 1)
EOF
  then
    echo "[retry $k/$N] no box ran the command; waiting"
    sleep 240
  else
    exit $rc
  fi
done
exit 3
