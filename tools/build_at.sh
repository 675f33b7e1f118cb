#!/bin/bash
# Builds libgslm.so of a git revision into gaussian-splatting-lm_amd/<outdir> for A/B runs:
#   bash tools/build_at.sh <rev> <outdir>
# The output directory is always rebuilt from scratch: `git archive` gives the sources their commit times,
# so make would otherwise keep stale objects that are newer than those times.
set -eo pipefail
REV=$1; OUT=$2
ROOT=$(pwd)
SRC=$(mktemp -d /tmp/gslm_rev.XXXXXX)
git archive "$REV" gaussian-splatting-lm_amd/csrc include | tar -x -C "$SRC"
rm -rf "$ROOT/gaussian-splatting-lm_amd/$OUT"
make -s -C "$SRC/gaussian-splatting-lm_amd/csrc" -j8 OUTDIR="$ROOT/gaussian-splatting-lm_amd/$OUT"
rm -rf "$SRC"
ls -la "$ROOT/gaussian-splatting-lm_amd/$OUT/libgslm.so"
