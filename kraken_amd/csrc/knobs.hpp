// knobs.hpp -- internal to libkraken_hip: where the library reads its environment.
//
// KRK_OP_ENV: the operator knobs, the table in INTEGRATION.md ("Operator knobs") and nothing
// else -- sizing (CPU budget, staging and pinned-pool memory, live blobs, descriptors), disk
// I/O mode, placement pins, start-up calibration and trace output.  The production library
// reads these only (tests/test_capi_cpu.py checks its strings against the table).
// KRK_AB_ENV: the A/B switches of measurement sessions (kernel and layout variants, thread
// hand-outs, slot sources, ISA fallbacks, fault injection).  Read by the diag build
// (`make diag`, KRK_DIAG) only; the production library keeps each one's measured default and
// does not even hold the name (every such switch forked the product
// path, and untested combinations grew with each round).
#pragma once
#include <stdlib.h>

#define KRK_OP_ENV(name) getenv(name)
#ifdef KRK_DIAG
#define KRK_AB_ENV(name) getenv(name)
#else
#define KRK_AB_ENV(name) (static_cast<const char*>(nullptr))
#endif
