#!/bin/bash
# Host-only ASan/UBSan build of the C++ test port + library sources
# (tests/cpp/Makefile target build/xrs_test_asan; build() makes it too).
set -e
cd "$(dirname "$0")/.."
make -s -C tests/cpp build/xrs_test_asan
