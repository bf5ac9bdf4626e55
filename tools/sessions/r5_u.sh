#!/bin/bash
# r5 session U2: host cost of the driver-shape timed region (tools/host_sync_probe.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 300 python -u tools/host_sync_probe.py --jsonl $O/u2_host_sync.jsonl > $O/u2_host_sync.txt 2>&1
echo "exit $?"
