#!/bin/bash
# Builds libgslm.so from the working tree with an edit applied to a scratch copy of the sources, for A/B runs of
# experiment variants that are not product code (timing-only builds):
#   bash tools/build_variant.sh <outdir> <edit.py> [EXTRA flags]
# edit.py runs in the scratch copy's csrc directory (it rewrites the .hip / .hpp files there); the library lands in
# gaussian-splatting-lm_amd/<outdir>/libgslm.so.  The working tree is not touched.
set -eo pipefail
OUT=$1; EDIT=$2; shift 2
ROOT=$(pwd)
SRC=$(mktemp -d /tmp/gslm_var.XXXXXX)
mkdir -p "$SRC/gaussian-splatting-lm_amd"
cp -r gaussian-splatting-lm_amd/csrc "$SRC/gaussian-splatting-lm_amd/"
cp -r include "$SRC/"
(cd "$SRC/gaussian-splatting-lm_amd/csrc" && python3 "$ROOT/$EDIT")
rm -rf "$ROOT/gaussian-splatting-lm_amd/$OUT"
make -s -C "$SRC/gaussian-splatting-lm_amd/csrc" -j8 OUTDIR="$ROOT/gaussian-splatting-lm_amd/$OUT" EXTRA="$*"
rm -rf "$SRC"
ls -la "$ROOT/gaussian-splatting-lm_amd/$OUT/libgslm.so"
