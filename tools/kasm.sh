#!/bin/bash
# Device-only assembly of gbp_engine.hip (or $1) for gfx950, plus the
# instruction mix of the kernel matching $2 (default: the headline launch,
# k_validate_persistent<float, false, 3, 2, true>).
cd "$(dirname "$0")/../global_body_planner_amd/csrc"
SRC=${1:-gbp_engine.hip}
PAT=${2:-k_validate_persistentIfLb0ELi3ELi2ELb1E}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math \
  -I../../include -I. --cuda-device-only -S -o /tmp/kasm.s "$SRC" || exit 1
python3 ../../tools/asm_mix.py /tmp/kasm.s "$PAT" ${3:-25}
