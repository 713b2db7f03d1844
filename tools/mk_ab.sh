#!/usr/bin/env bash
# tools/mk_ab.sh [REV] -- build the A/B pair for tools/ab_run.sh:
#   probes/base.so  the codec library from git REV (default HEAD)
#   probes/new.so   the codec library from the working tree
# (plus the product library itself, lcdb_amd/liblcdb_gpu_snappy.so).
set -euo pipefail
cd "$(dirname "$0")/.."
rev="${1:-HEAD}"
tmp="$(mktemp -d)"
trap 'rm -rf "$tmp"' EXIT
git archive "$rev" lcdb_amd/csrc include | tar -x -C "$tmp"
mkdir -p probes
srcs="lgs_api.cpp lgs_encode.hip lgs_decode.hip lgs_table.hip lgs_bloom.hip lgs_table_index.cpp lgs_probe.hip"
build() {   # $1: source root, $2: output
  local args=()
  for s in $srcs; do args+=("$1/lcdb_amd/csrc/$s"); done
  local map=()
  [ -f "$1/lcdb_amd/csrc/exports.map" ] && map=("-Wl,--version-script=$1/lcdb_amd/csrc/exports.map")
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -pthread \
    -I"$1/include" "${map[@]}" "${args[@]}" -o "$2" "${@:3}"
}
build "$tmp" probes/base.so &
build "$PWD" probes/new.so &
wait %1; wait %2
python -c "from lcdb_amd import build; build.build_hip()"
ls -la probes/base.so probes/new.so
