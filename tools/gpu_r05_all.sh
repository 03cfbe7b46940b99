#!/bin/bash
# Round-5 final session: validation + drop-in trace (gpu_r05.sh), then the profiling
# session (gpu_round.sh, TAG) on the two bench configs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r05.sh && TAG=${TAG:-r05v2} NOTEST=1 BENCH_CONFIGS="deit_base dit_xl2" bash tools/gpu_round.sh
