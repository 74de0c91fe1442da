#!/bin/bash
# Build a variant of libaccord_deps.so with extra compile flags into variants/<name>.so (git-ignored;
# separate object directory): scripts/build_variant.sh <name> "-DLEAN_EXP=1 ..."
set -e
name=$1
shift
cd "$(dirname "$0")/../cassandra-accord_amd/csrc"
mkdir -p ../../variants
make -s -j8 OUT=../../variants/$name.so OBJDIR=../../variants/build_$name \
  FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-parameter -Wno-unused-result $*"
