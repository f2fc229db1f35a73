// sas_version.hip -- the source hash this build of libsas_amd.so was compiled from.
// The Makefile passes SAS_SOURCE_HASH = the first 16 hex digits of the sha256 over every
// source and header (csrc/, include/); rebuilt whenever any of them changes.  bench.py
// attaches a committed rocprofv3 --pmc summary to its record only when the summary names
// the same hash, so counters of one build are never reported for another.
#include "../../include/sas.h"

#ifndef SAS_SOURCE_HASH
#define SAS_SOURCE_HASH "unknown"
#endif

extern "C" const char* sas_source_hash(void) { return SAS_SOURCE_HASH; }
