// version.cpp -- xrs_version(): names the sources the library was built from.
//
// The Makefile passes XRS_SRC_HASH = the first 16 hex digits of the sha256 of
// the library's sources (xrs_amd/csrc: Makefile and every *.cpp *.h *.hip
// *.map, in byte order of their names, then include/xrs_hip.h), and rebuilds
// this file whenever one of them changes.  xrs_amd.source_hash() computes the
// same digest from a source tree, so a test, smoke() and the bench line can
// show that the measured binary is the tree's.
#include "xrs_hip.h"

#ifndef XRS_SRC_HASH
#define XRS_SRC_HASH "unknown"
#endif

extern "C" const char* xrs_version(void) { return "xrs-hip 0.2 gfx950 src " XRS_SRC_HASH; }
