// probe_res_wrap.cc -- TEST INFRASTRUCTURE ONLY (oracle/probe_cabac.cc): compiles the
// reference's own parser/interpret_residual.cc (included from /root/reference by path, not
// copied) with its file-local tables given external linkage, so that the probe can print
// them.  Every header it uses is included first, so `static` is redefined for that one
// file's own definitions only.
#include <functional>
#include "global.h"
#include "slice.h"
#include "macroblock.h"
#include "neighbour.h"
#define static extern
#include "interpret_residual.cc"
#undef static
