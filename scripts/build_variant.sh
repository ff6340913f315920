#!/bin/bash
# Build libmdx.so from another revision's csrc (or "." = the working tree, optionally with -D
# defines appended to the kernels' flags) into motion_detection_amd/lib_var/<name>/libmdx.so, for
# same-box A/B timing through MDX_LIB_PATH (CPU side, before a gpurun call).
# Usage: bash scripts/build_variant.sh <git-rev|.> <name> [-DFOO=1 ...]
set -e
rev=$1; name=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
if [ "$rev" = "." ]; then
    mkdir -p "$tmp/motion_detection_amd"
    cp -r "$root/motion_detection_amd/csrc" "$tmp/motion_detection_amd/"
    cp -r "$root/include" "$tmp/"
else
    git -C "$root" archive "$rev" motion_detection_amd/csrc include | tar -x -C "$tmp"
fi
if [ $# -gt 0 ]; then sed -i "s|^KFLAGS  := \(.*\)|KFLAGS  := \1 $*|" "$tmp/motion_detection_amd/csrc/Makefile"; fi
out="$root/motion_detection_amd/lib_var/$name"
mkdir -p "$out"
make -s -C "$tmp/motion_detection_amd/csrc" OUT="$out" OBJ="$tmp/build" 2>&1 | grep -E "error" || true
rm -rf "$tmp"
test -f "$out/libmdx.so" && echo "$out/libmdx.so"
