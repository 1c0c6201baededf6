#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
args=()
for c in 8192 32768 131072; do for r in 0.5 1 2 4; do args+=("c${c}_r$r" "DT_SG_CELLS=$c DT_SG_REACH=$r"); done; done
bash $R/tools/ab_env.sh "${args[@]}"
