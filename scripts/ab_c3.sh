#!/bin/bash
# A/B of library builds on config 3 (10 M rows x 64 channels, one GPU),
# alternating runs: scripts/ab_c3.sh OUT ROUNDS "dir_a dir_b ..."
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=$1; ROUNDS=$2; DIRS=$3; shift 3
timeout -k 10 900 scripts/ab_env.sh "$OUT" SKA_SDP_FUNC_LIB_DIR "$DIRS" "$ROUNDS" \
    --rows 100000 --steps 2 --warmup 1 --no-degrid --no-wstack --c3-steps 3 "$@"
