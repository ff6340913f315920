#!/bin/bash
# Build timing-only LK variants (each drops one load stream of k_lk_level) as separate
# libraries: motion_detection_amd/lib/libmdx_<name>.so.  Run here (CPU); time on the GPU box
# with: for v in ...; do MDX_LIB_PATH=.../libmdx_$v.so python bench.py ...; done
set -e
cd "$(dirname "$0")/../motion_detection_amd/csrc"
H=/opt/rocm/bin/hipcc
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I../../include"
mkdir -p ../build/var
for v in "$@"; do
    name=${v%%:*}; defs=${v#*:}
    $H $F $defs -c mdx_lk.hip -o ../build/var/lk_$name.o
    $H --offload-arch=gfx950 -shared -fPIC -pthread ../build/mdx_kernels.o ../build/var/lk_$name.o ../build/mdx_warp.o ../build/mdx_subspace.o ../build/mdx_api.o \
        ../build/synth.o -o ../lib/libmdx_$name.so
    echo "built libmdx_$name.so ($defs)"
done
