#!/bin/bash
# round-4 GPU call J: full GPU suite + smoke + default bench after the late round-4 changes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LIMIT=800 tools/gpu.sh tests tests/ || exit 1
tools/gpu.sh smoke || exit 1
LIMIT=300 tools/gpu.sh bench || exit 1
