#!/bin/bash
# one optimisation iteration: GPU suite, race benches, actor-driven phase profile (timing build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_quick.sh
bash tools/gpu_phases_c3p.sh
