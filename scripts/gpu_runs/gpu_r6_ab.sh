#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
./scripts/gpu_r6_b.sh && ./scripts/gpu_r6_a.sh
