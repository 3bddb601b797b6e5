#!/bin/bash
# Build libba3c.so of a git revision (default HEAD) into the working tree as
# distributed-ba3c_amd/ba3c_amd/libba3c_<name>.so, for same-box A/B runs (BA3C_LIB=...).
# usage: scripts/build_prev.sh [REV] [NAME]
set -e
REV=${1:-HEAD}; NAME=${2:-prev}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=$(mktemp -d /tmp/ba3c_wt.XXXXXX)
git -C "$ROOT" worktree add -q --detach "$WT" "$REV"
make -s -C "$WT/distributed-ba3c_amd" -j8 >/dev/null
cp "$WT/distributed-ba3c_amd/ba3c_amd/libba3c.so" "$ROOT/distributed-ba3c_amd/ba3c_amd/libba3c_$NAME.so"
git -C "$ROOT" worktree remove --force "$WT"
echo "$ROOT/distributed-ba3c_amd/ba3c_amd/libba3c_$NAME.so"
