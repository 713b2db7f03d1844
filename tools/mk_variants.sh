#!/usr/bin/env bash
# tools/mk_variants.sh NAME:FLAGS ... -- build probes/NAME.so from the working
# tree with extra compiler FLAGS (e.g. base: new:-DLGS_X), in parallel.
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p probes
srcs="lgs_api.cpp lgs_encode_service.hip lgs_decode.hip lgs_table.hip lgs_bloom.hip lgs_table_index.cpp lgs_probe.hip"
args=(); for s in $srcs; do args+=("lcdb_amd/csrc/$s"); done
common=(-O3 --offload-arch=gfx950 -std=c++17 -fPIC
        -mllvm -phi-node-folding-threshold=8 -mllvm -two-entry-phi-node-folding-threshold=16)
pids=()
for spec in "$@"; do
  name="${spec%%:*}"; flags="${spec#*:}"
  (
    # shellcheck disable=SC2086
    /opt/rocm/bin/hipcc "${common[@]}" -mllvm -amdgpu-sched-strategy=max-ilp -DLGS_ENCODE_BATCH_ONLY \
      $flags -c lcdb_amd/csrc/lgs_encode.hip -o "probes/$name.enc.o" &&
    /opt/rocm/bin/hipcc "${common[@]}" -shared -pthread \
      -Wl,--version-script=lcdb_amd/csrc/exports.map $flags "${args[@]}" -x none "probes/$name.enc.o" \
      -o "probes/$name.so" && rm -f "probes/$name.enc.o"
  ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
ls -la probes/*.so
