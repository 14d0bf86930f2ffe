#!/bin/bash
# walk batching with row slots: slots (NB_SK) and entries (NB_NE) per lane per round
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && STEPS=2 WARMUP=1 bash tools/sweep_walks.sh r06ae "main sk1 sk4 ne4 ne1 main" || exit 1
