#!/bin/bash
# Build libkrr_amd.so variants (extra -D flags) for scripts/ab_variants.py.
# usage: bash scripts/build_variants.sh name1:"-DFOO=1 -DBAR=2" name2:"..."
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/krr_amd/lib/variants"
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off \
    -I"$R/include" -I"$R/krr_amd/csrc" $flags "$R/krr_amd/csrc/krr_kernels.hip" \
    -o "$R/krr_amd/lib/variants/lib_$name.so" &
done
wait
ls -la "$R/krr_amd/lib/variants"
