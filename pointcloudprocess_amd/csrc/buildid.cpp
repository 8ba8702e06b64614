// pcp_build_id(): the SHA-1 of the sources this libpcp.so was built from (computed by the
// Makefile over every csrc source and header, include/pcp.h and the Makefile, in sorted name
// order), so a test can prove the library a run loaded matches the tree it runs from.
#include "../../include/pcp.h"

#ifndef PCP_SRC_SHA
#error "PCP_SRC_SHA is set by the Makefile"
#endif

extern "C" const char* pcp_build_id(void) { return PCP_SRC_SHA; }
