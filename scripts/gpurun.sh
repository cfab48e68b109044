#!/bin/bash
# rebuild the in-tree library (so the snapshot never carries a stale .so), then gpurun
# usage: scripts/gpurun.sh TIMEOUT 'command'
set -e
cd "$(dirname "$0")/.."
python -c "import shadow_amd.build as b; b.build()"
exec /usr/local/graft/bin/gpurun --timeout "$1" -- "$2"
