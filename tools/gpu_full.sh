#!/bin/bash
# tests + smoke + bench + kernel-stats profile + FETCH/WRITE PMC passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_check.sh || exit $?
GROUPS_LIST="${GROUPS_LIST:-FETCH_SIZE;WRITE_SIZE}" bash tools/pmc.sh
