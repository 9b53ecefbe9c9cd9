#!/bin/bash
# Build a tuning variant of liblac.so with extra -D flags:  tools/sessions/ab/build_variant.sh <name> "<flags>"
# -> tools/sessions/ab/liblac_<name>.so (git-ignored; travels to the GPU box with the tree)
set -eu
cd "$(dirname "$0")/../.."
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I include -I lac_amd/csrc $2 \
    lac_amd/csrc/lac_kernels.hip -o tools/sessions/ab/liblac_$1.so
