#!/bin/bash
# Build timing-only variants of mdx_warp.hip as motion_detection_amd/lib/libmdx_<name>.so
# (each drops one stage of k_warp_diff; results invalid).  "name:-DFLAGS" arguments.
set -e
cd "$(dirname "$0")/../motion_detection_amd/csrc"
H=/opt/rocm/bin/hipcc
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I../../include"
mkdir -p ../build/var
for v in "$@"; do
    name=${v%%:*}; defs=${v#*:}
    $H $F $defs -c mdx_warp.hip -o ../build/var/warp_$name.o
    $H --offload-arch=gfx950 -shared -fPIC -pthread ../build/mdx_kernels.o ../build/mdx_lk.o ../build/mdx_subspace.o ../build/var/warp_$name.o \
        ../build/mdx_api.o ../build/synth.o ../build/buildinfo.o -o ../lib/libmdx_$name.so
    echo "built libmdx_$name.so ($defs)"
done
