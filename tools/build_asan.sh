#!/bin/bash
# Host-only ASan/UBSan build of the C++ test port + library sources
# (the GPU code is not instrumented: -fsanitize flags go after -Xarch_host).
set -e
cd "$(dirname "$0")/.."
mkdir -p tests/cpp/build
hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -Xarch_host -fsanitize=address \
  -Xarch_host -fsanitize=undefined -fno-omit-frame-pointer -Iinclude -Ixrs_amd/csrc \
  tests/cpp/xrs_test.cpp xrs_amd/csrc/codec.cpp xrs_amd/csrc/gf256.cpp xrs_amd/csrc/kernels.hip \
  -o tests/cpp/build/xrs_test_asan
