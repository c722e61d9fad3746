// tgms_host.h — the explicit host backend of the C ABI (tgms_create_host; tgms_host.cpp).
// Plain C++ (no HIP): compiled by g++ into libtgms.so.
#pragma once

#include <stdint.h>

#include "tgms.h"

namespace tgms {
namespace host {

// One trajectory (include/tgms.h layouts): waypoints [M+1][3], seg_times [M], end_derivs
// NULL or [18], coeffs [M][3][8].  Returns a tgms_status; every failure writes exact zeros.
int solve(int M, const double* waypoints, const double* seg_times, const double* end_derivs, double* coeffs);

// ns samples (tgms_sample_count) of one solved trajectory into out [ns][TGMS_GOAL_STRIDE].
void sample(int M, const double* coeffs, const double* seg_times, const double* waypoints, const double* end_derivs,
            double dt, int yaw_mode, double yaw_const, int64_t ns, double* out);

}  // namespace host
}  // namespace tgms
