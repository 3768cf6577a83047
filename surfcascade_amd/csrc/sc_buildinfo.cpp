// sc_buildinfo.cpp -- what this libsurfcascade.so was built from (sc_build_info).
//
// SC_BUILD_ID is a sha256 prefix over every source file of csrc/, the public
// header, the Makefile, the extra compile flags (EXTRA: the -D schedule
// knobs of a variant build), the target (ARCH) and the host sanitizer flags
// (SAN), computed by the Makefile; SC_BUILD_FLAGS is that EXTRA string,
// SC_BUILD_ARCH / SC_BUILD_SAN the other two.  A measurement stamped with a build id (bench.py, the PMC
// table profiles/pmc_windows.json) therefore describes exactly one binary:
// any change to a kernel, to the launch schedule in sc_api.cpp or to a flag
// gives another id.
#include "surfcascade.h"

#ifndef SC_BUILD_ID
#error "SC_BUILD_ID is set by the Makefile"
#endif
#ifndef SC_BUILD_FLAGS
#define SC_BUILD_FLAGS ""
#endif
#ifndef SC_BUILD_ARCH
#error "SC_BUILD_ARCH is set by the Makefile"
#endif
#ifndef SC_BUILD_SAN
#define SC_BUILD_SAN ""
#endif

#ifdef SC_ABLATION_BUILD
#define SC_BI_ABL "true"
#else
#define SC_BI_ABL "false"
#endif
#if defined(SC_TEST_HOOKS) && SC_TEST_HOOKS
#define SC_BI_HOOKS "true"
#else
#define SC_BI_HOOKS "false"
#endif
#if defined(SC_PROF_CHAIN) && SC_PROF_CHAIN
#define SC_BI_PROF "true"
#else
#define SC_BI_PROF "false"
#endif

extern "C" const char *sc_build_info(void) {
    return "{\"build_id\": \"" SC_BUILD_ID "\", \"flags\": \"" SC_BUILD_FLAGS "\", \"arch\": \"" SC_BUILD_ARCH "\", "
           "\"sanitizer\": \"" SC_BUILD_SAN "\", \"ablation\": " SC_BI_ABL ", \"test_hooks\": " SC_BI_HOOKS ", \"profiling\": " SC_BI_PROF "}";
}
