#!/bin/bash
# r5 session U: host cost of the driver-shape timed region (tools/host_sync_probe.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 300 python -u tools/host_sync_probe.py --jsonl $O/u_host_sync.jsonl > $O/u_host_sync.txt 2>&1
echo "exit $?"
