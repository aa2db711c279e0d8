// vw_launch.h -- shared by the launcher units vw_fwd.hip / vw_inv.hip / vw_lvl.hip, each compiled once
// per element type (the Makefile passes -DVW_T=double or -DVW_T=float).
#pragma once
#include "vw_device.h"

#ifndef VW_T
#error "compile with -DVW_T=double or -DVW_T=float"
#endif

namespace vw {

// Unrolled tap counts; other L use the runtime-L kernels.  Dev builds may restrict the list:
// make DEV_TAPS='X(8)' (the runtime-L kernel still covers every other L).
#ifdef VW_DEV_TAPS
#define VW_TAP_LIST(X) VW_DEV_TAPS(X)
#else
#define VW_TAP_LIST(X) X(2) X(4) X(6) X(8) X(10) X(12) X(14) X(16) X(18) X(20) X(24) X(30)
#endif


}  // namespace vw
