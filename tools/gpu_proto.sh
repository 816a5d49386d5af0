#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}/tools/proto_bin" || exit 1
for b in *; do timeout -k 5 60 ./$b ${REPS:-24} ${GRID:-256} || { echo "fail $b"; exit 1; }; done
