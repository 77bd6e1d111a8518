#!/bin/bash
# Ablation builds (wrong physics, diagnostics only): copies csrc to build/exp/, applies
# exp_switches.patch there and builds build/exp/libbsg_<name>.so with one switch on --
# never into bluesky_gym/_lib, so the product loader cannot pick it up.
#   bash tools/ablation/build_exp.sh SKIP_OWN      (ownship frozen)
#   bash tools/ablation/build_exp.sh CD_NOTEST     (CD phase 1 tests nothing)
#   bash tools/ablation/build_exp.sh CD_NOP1       (every pair a CD candidate)
#   bash tools/ablation/build_exp.sh CD_NOP2       (CD phase 2 skipped)
#   bash tools/ablation/build_exp.sh GS64          (one env per wave)
# Load with bluesky_gym._native.load_library("build/exp/libbsg_<name>.so") before any env.
set -euo pipefail
NAME=$1
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
W=$ROOT/build/exp/src
rm -rf "$W" && mkdir -p "$W/bluesky-gym-hallucination_amd" "$W/include"
cp -r "$ROOT/bluesky-gym-hallucination_amd/csrc" "$W/bluesky-gym-hallucination_amd/"
cp "$ROOT/include/bsg.h" "$W/include/"
(cd "$W" && patch -p1 < "$ROOT/tools/ablation/exp_switches.patch")
name=$(echo "$NAME" | tr 'A-Z' 'a-z')
make -C "$W/bluesky-gym-hallucination_amd/csrc" -j8 OUT="$ROOT/build/exp/libbsg_$name.so" OBJ="$ROOT/build/exp/obj_$name" \
     CXXFLAGS_EXTRA="-DBSG_EXP_$NAME=1"
