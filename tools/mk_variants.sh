#!/usr/bin/env bash
# tools/mk_variants.sh NAME:FLAGS ... -- build probes/NAME.so from the working
# tree with extra compiler FLAGS (e.g. base: new:-DLGS_X), in parallel.
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p probes
srcs="lgs_api.cpp lgs_encode.hip lgs_decode.hip lgs_table.hip lgs_bloom.hip lgs_table_index.cpp lgs_probe.hip"
args=(); for s in $srcs; do args+=("lcdb_amd/csrc/$s"); done
pids=()
for spec in "$@"; do
  name="${spec%%:*}"; flags="${spec#*:}"
  # shellcheck disable=SC2086
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -pthread \
    -mllvm -phi-node-folding-threshold=8 -mllvm -two-entry-phi-node-folding-threshold=16 \
    -Wl,--version-script=lcdb_amd/csrc/exports.map $flags "${args[@]}" -o "probes/$name.so" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
ls -la probes/*.so
