#!/bin/bash
# GPU box, round 5 (o): native SD engine tests (incl. img2img), then the SDXL step kernel table.
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r5_l.sh || exit 1
bash scripts/gpu_r5_k.sh
