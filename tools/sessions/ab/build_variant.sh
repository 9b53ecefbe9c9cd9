#!/bin/bash
# Build a tuning variant of liblac.so with extra -D flags:  tools/sessions/ab/build_variant.sh <name> "<flags>"
# -> tools/sessions/ab/liblac_<name>.so (git-ignored; travels to the GPU box with the tree)
set -eu
cd "$(dirname "$0")/../../.."
python3 -m lac_amd.build --out tools/sessions/ab/liblac_$1.so $2
