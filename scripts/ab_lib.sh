#!/bin/bash
# A/B of library builds (scripts/variant_lib.sh) on the config-2 bench,
# alternating runs: scripts/ab_lib.sh OUT ROUNDS "dir_a dir_b ..." [bench args]
OUT=$1; ROUNDS=$2; DIRS=$3; shift 3
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 scripts/ab_env.sh "$OUT" SKA_SDP_FUNC_LIB_DIR "$DIRS" "$ROUNDS" "$@"
