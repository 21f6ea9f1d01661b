#!/bin/bash
# Secondary legs only (reference timeouts, ring, C2) + ring parity tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u - > gpurun_out/legs.json 2> gpurun_out/legs.err <<'PY'
import json, sys
sys.path.insert(0, "p2p-file-system-with-gossip-detect-failure-management_amd"); sys.path.insert(0, ".")
import bench, gossipsim as gs
print(json.dumps(bench.secondary_legs(gs)))
PY
