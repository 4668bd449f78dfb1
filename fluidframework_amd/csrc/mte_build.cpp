// mte_build_info (include/mte.h): which sources and compiler this libmte.so
// was built from.  MTE_SRC_SHA comes from the Makefile: the first 16 hex
// digits of the sha256 of mte_*.h, mte_*.hip (name order) and include/mte.h.
#include "../../include/mte.h"

#ifndef MTE_SRC_SHA
#define MTE_SRC_SHA "unknown"
#endif

extern "C" const char* mte_build_info(void) { return "src=" MTE_SRC_SHA " arch=gfx950 compiler=" __VERSION__; }
