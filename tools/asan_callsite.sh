#!/bin/bash
# Host-only AddressSanitizer build of the ROS-node call-site check: the planner
# host code (csrc/host/gbp_planner.cpp) compiled into the executable with
# -fsanitize=address; the HIP engine (libgbp.so) is linked uninstrumented.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIB=global_body_planner_amd/lib
g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address -ffp-contract=off -Iinclude \
    tests/integration/node_callsite.cpp global_body_planner_amd/csrc/host/gbp_planner.cpp \
    -L$LIB -lgbp -Wl,-rpath,$PWD/$LIB -o gpurun_out/node_callsite_asan || exit 1
export ASAN_OPTIONS=verify_asan_link_order=0:detect_leaks=0
for mode in plain star; do
  timeout -k 10 180 ./gpurun_out/node_callsite_asan $mode > gpurun_out/asan_$mode.log 2>&1
  rc=$?
  echo "$mode rc=$rc"; tail -40 gpurun_out/asan_$mode.log
  [ $rc -eq 0 ] || exit $rc
done
