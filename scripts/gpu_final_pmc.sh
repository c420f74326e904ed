#!/bin/bash
# The writer's PMC passes on the WGS line, final tree (profiles/pmc_k_emit_tiles_r04_wgs.json).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_pmc.sh r04final k_emit_tiles r04_wgs wgs 150 3095693981 || exit $?
echo done
