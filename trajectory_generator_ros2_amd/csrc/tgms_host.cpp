// tgms_host.cpp — the explicit host backend of the C ABI (tgms_create_host, include/tgms.h)
// for BASELINE config 1: "single goal, 3-segment order-7 min-snap via the CPU
// TrajectoryGenerator (ROS2 node up, no GPU)".  The reference generates its goals on the
// rclcpp executor thread's CPU (src/TrajectoryGenerator.cpp:54-57, :71); a node with no GPU
// gets the same MinSnap primitive from this file when its YAML asks for
// `minsnap_backend: host`.  It is never a fallback: tgms_create still fails with
// TGMS_ERR_NO_DEVICE when no GPU exists, and a host handle accepts only the host-pointer
// solve / sample entry points (B = 1 at config 1; any B works).
//
// The solve is the reduced formulation of DESIGN.md §2 (the product's own math, written
// from the Hermite elimination, not from oracle/): per axis the SPD block-tridiagonal
// system over the free knot derivatives u_k = (v, a, j), k = 1..M-1, with 3x3 blocks
//     H_kk    = KEE o r_{k-1}^(5-d-e) + KSS o r_k^(5-d-e),   H_k,k+1 = KSE o r_k^(5-d-e)
//     rhs_k   = -KEP r_{k-1}^(6-d) (w_k - w_{k-1}) - KSP r_k^(6-d) (w_{k+1} - w_k)
// (r_i = 1/T_i; the same integer matrices as the kernels, tgms_device.h), shared by the
// three axes, solved by a one-sided block LDL^T (block Thomas: S_k = H_kk - C^T S^-1 C),
// then each segment's septic Hermite data converted to monomial coefficients.  The sampler
// evaluates p/v/a/j by Horner in local time with the GPU sampler's conventions (segment
// scan, pinned last sample, yaw).  tests/test_host_backend.py holds both to the oracle and
// the exact goldens at 1e-9.
#include "tgms_host.h"

#include <cfloat>
#include <cmath>

namespace tgms {
namespace host {
namespace {

constexpr double KSS[3][3] = {{25920, 5400, 480}, {5400, 1200, 120}, {480, 120, 16}};
constexpr double KEE[3][3] = {{25920, -5400, 480}, {-5400, 1200, -120}, {480, -120, 16}};
constexpr double KSE[3][3] = {{24480, -4680, 360}, {4680, -840, 60}, {360, -60, 4}};
constexpr double KSP[3] = {-50400, -10080, -840};
constexpr double KEP[3] = {-50400, 10080, -840};

bool finite(double v) { return v * 0.0 == 0.0; }

// r^0 .. r^7
void powers(double r, double (&p)[8]) {
    p[0] = 1.0;
    for (int k = 1; k < 8; ++k) p[k] = p[k - 1] * r;
}

struct Ldl {  // LDL^T of an SPD 3x3 block: reciprocal pivots, unit-lower multipliers
    double i0, i1, i2, l10, l20, l21;
};

bool factor(const double (&D)[3][3], Ldl& f) {
    const double p0 = D[0][0];
    f.i0 = 1.0 / p0;
    f.l10 = D[0][1] * f.i0;
    f.l20 = D[0][2] * f.i0;
    const double p1 = D[1][1] - f.l10 * D[0][1];
    f.i1 = 1.0 / p1;
    const double t12 = D[1][2] - f.l20 * D[0][1];
    f.l21 = t12 * f.i1;
    const double p2 = D[2][2] - f.l20 * D[0][2] - f.l21 * t12;
    f.i2 = 1.0 / p2;
    return p0 > 0.0 && p1 > 0.0 && p2 > 0.0;
}

void solve3(const Ldl& f, const double (&b)[3], double (&x)[3]) {
    const double y1 = b[1] - f.l10 * b[0];
    const double y2 = b[2] - f.l20 * b[0] - f.l21 * y1;
    x[2] = y2 * f.i2;
    x[1] = y1 * f.i1 - f.l21 * x[2];
    x[0] = b[0] * f.i0 - f.l10 * x[1] - f.l20 * x[2];
}

// Septic Hermite data of one axis of a segment (positions w0, w1; derivatives (v, a, j) at
// both ends) -> ascending monomial coefficients in local time, in r = 1/T scaled
// variables: c_k = r^(k-3) P_k for k >= 4, P linear in ((w1 - w0) r^3, v r^2, a r, j).
void hermite(double w0, double w1, const double (&s)[3], const double (&e)[3], double r, double* c) {
    const double r2 = r * r, r3 = r2 * r, r4 = r2 * r2;
    const double D = (w1 - w0) * r3;
    const double V0 = s[0] * r2, A0 = s[1] * r, J0 = s[2], V1 = e[0] * r2, A1 = e[1] * r, J1 = e[2];
    const double P4 = 35.0 * D - 20.0 * V0 - 5.0 * A0 - (2.0 / 3.0) * J0 - 15.0 * V1 + 2.5 * A1 - (1.0 / 6.0) * J1;
    const double P5 = -84.0 * D + 45.0 * V0 + 10.0 * A0 + J0 + 39.0 * V1 - 7.0 * A1 + 0.5 * J1;
    const double P6 = 70.0 * D - 36.0 * V0 - 7.5 * A0 - (2.0 / 3.0) * J0 - 34.0 * V1 + 6.5 * A1 - 0.5 * J1;
    const double P7 = -20.0 * D + 10.0 * V0 + 2.0 * A0 + (1.0 / 6.0) * J0 + 10.0 * V1 - 2.0 * A1 + (1.0 / 6.0) * J1;
    c[0] = w0;
    c[1] = s[0];
    c[2] = 0.5 * s[1];
    c[3] = s[2] * (1.0 / 6.0);
    c[4] = P4 * r;
    c[5] = P5 * r2;
    c[6] = P6 * r3;
    c[7] = P7 * r4;
}

}  // namespace

int solve(int M, const double* W, const double* T, const double* ED, double* C) {
    const int n = M * 24;
    for (int q = 0; q < n; ++q) C[q] = 0.0;
    if (M < 1 || M > TGMS_MAX_SEGMENTS) return TGMS_ERR_INVALID_ARG;
    bool ok = true;
    for (int i = 0; i < M; ++i) ok = ok && T[i] > 0.0 && T[i] <= DBL_MAX;
    for (int q = 0; q < (M + 1) * 3; ++q) ok = ok && finite(W[q]);
    if (ED)
        for (int q = 0; q < 18; ++q) ok = ok && finite(ED[q]);
    if (!ok) return TGMS_ERR_INVALID_ARG;

    double rp[TGMS_MAX_SEGMENTS][8];
    for (int i = 0; i < M; ++i) powers(1.0 / T[i], rp[i]);
    // knot derivatives [knot][derivative][axis]: knot 0 and M from the end derivatives
    double x[TGMS_MAX_SEGMENTS + 1][3][3] = {};
    for (int d = 0; d < 3; ++d)
        for (int a = 0; a < 3; ++a) {
            x[0][d][a] = ED ? ED[d * 3 + a] : 0.0;
            x[M][d][a] = ED ? ED[9 + d * 3 + a] : 0.0;
        }
    const int NK = M - 1;  // interior knots 1..M-1, index k
    Ldl F[TGMS_MAX_SEGMENTS];
    double G[TGMS_MAX_SEGMENTS][3][3];  // G_k = S_k^-1 C_k (C_k couples knots k and k+1)
    bool spd = true;
    for (int k = 1; k <= NK; ++k) {
        const double(&pp)[8] = rp[k - 1];
        const double(&pn)[8] = rp[k];
        double S[3][3];
        for (int d = 0; d < 3; ++d)
            for (int e = 0; e < 3; ++e) S[d][e] = KEE[d][e] * pp[5 - d - e] + KSS[d][e] * pn[5 - d - e];
        if (k >= 2) {  // S_k = H_kk - C_{k-1}^T G_{k-1}
            const double(&pc)[8] = rp[k - 1];
            for (int d = 0; d < 3; ++d)
                for (int e = 0; e < 3; ++e) {
                    double acc = 0.0;
                    for (int f = 0; f < 3; ++f) acc += KSE[f][d] * pc[5 - f - d] * G[k - 1][f][e];
                    S[d][e] -= acc;
                }
        }
        spd = factor(S, F[k]) && spd;
        if (k < NK) {  // G_k = S_k^-1 C_k, C_k[d][e] = KSE[d][e] r_k^(5-d-e)
            for (int e = 0; e < 3; ++e) {
                const double col[3] = {KSE[0][e] * pn[5 - e], KSE[1][e] * pn[4 - e], KSE[2][e] * pn[3 - e]};
                double g[3];
                solve3(F[k], col, g);
                for (int d = 0; d < 3; ++d) G[k][d][e] = g[d];
            }
        }
    }
    if (!spd) return TGMS_ERR_SINGULAR;
    // forward: z_k = y_k - G_{k-1}^T z_{k-1} (C^T S^-1 = G^T: S symmetric), g_k = S_k^-1 z_k,
    // then back: x_k = g_k - G_k x_{k+1}, per axis
    for (int a = 0; a < 3; ++a) {
        double z[TGMS_MAX_SEGMENTS][3];
        for (int k = 1; k <= NK; ++k) {
            const double(&pp)[8] = rp[k - 1];
            const double(&pn)[8] = rp[k];
            const double wp = W[(k - 1) * 3 + a], wk = W[k * 3 + a], wn = W[(k + 1) * 3 + a];
            double y[3];
            for (int d = 0; d < 3; ++d)
                y[d] = -KEP[d] * pp[6 - d] * (wk - wp) - KSP[d] * pn[6 - d] * (wn - wk);
            if (k == 1)  // start derivatives through C_0
                for (int d = 0; d < 3; ++d)
                    for (int e = 0; e < 3; ++e) y[d] -= KSE[e][d] * pp[5 - d - e] * x[0][e][a];
            if (k == NK)  // final derivatives through C_{M-1}
                for (int d = 0; d < 3; ++d)
                    for (int e = 0; e < 3; ++e) y[d] -= KSE[d][e] * pn[5 - d - e] * x[M][e][a];
            if (k >= 2)
                for (int d = 0; d < 3; ++d)
                    for (int f = 0; f < 3; ++f) y[d] -= G[k - 1][f][d] * z[k - 1][f];
            for (int d = 0; d < 3; ++d) z[k][d] = y[d];
        }
        for (int k = NK; k >= 1; --k) {
            double g[3];
            solve3(F[k], z[k], g);
            if (k < NK)
                for (int d = 0; d < 3; ++d)
                    for (int e = 0; e < 3; ++e) g[d] -= G[k][d][e] * x[k + 1][e][a];
            for (int d = 0; d < 3; ++d) x[k][d][a] = g[d];
        }
    }
    double fin = 0.0;
    for (int i = 0; i < M; ++i)
        for (int a = 0; a < 3; ++a) {
            const double s[3] = {x[i][0][a], x[i][1][a], x[i][2][a]};
            const double e[3] = {x[i + 1][0][a], x[i + 1][1][a], x[i + 1][2][a]};
            double* c = C + (i * 3 + a) * 8;
            hermite(W[i * 3 + a], W[(i + 1) * 3 + a], s, e, rp[i][1], c);
            for (int j = 0; j < 8; ++j) fin += c[j] * 0.0;
        }
    if (!finite(fin)) {
        for (int q = 0; q < n; ++q) C[q] = 0.0;
        return TGMS_ERR_NONFINITE;
    }
    return TGMS_OK;
}

void sample(int M, const double* C, const double* T, const double* W, const double* ED, double dt, int yaw_mode,
            double yaw_const, int64_t ns, double* out) {
    double tau[TGMS_MAX_SEGMENTS + 1];
    tau[0] = 0.0;
    double acc = 0.0;
    for (int i = 0; i < M; ++i) tau[i + 1] = (acc += T[i]);  // the same order as tgms_sample_offsets
    int i = 0;
    double t_cur = 0.0, t_next = M > 1 ? tau[1] : 0.0;
    for (int64_t k = 0; k < ns; ++k) {
        double* o = out + k * TGMS_GOAL_STRIDE;
        if (k < ns - 1) {
            const double t = (double)k * dt;
            while (i + 1 < M && t_next <= t) {  // segment scan, as the GPU sampler's
                ++i;
                t_cur = t_next;
                t_next = tau[i + 1 < M ? i + 1 : M];
            }
            const double lt = t - t_cur;
            for (int a = 0; a < 3; ++a) {
                const double* c = C + (i * 3 + a) * 8;
                for (int q = 0; q < 4; ++q) {  // d^q/dt^q by Horner on j!/(j-q)! c_j
                    auto coef = [&](int j) {
                        double f = 1.0;
                        for (int m = 0; m < q; ++m) f *= (double)(j - m);
                        return f * c[j];
                    };
                    double s = coef(7);
                    for (int j = 6; j >= q; --j) s = std::fma(s, lt, coef(j));
                    o[q * 3 + a] = s;
                }
            }
        } else {  // the last sample, pinned to the final waypoint and end derivatives
            for (int a = 0; a < 3; ++a) {
                o[a] = W[M * 3 + a];
                o[3 + a] = ED ? ED[9 + a] : 0.0;
                o[6 + a] = ED ? ED[12 + a] : 0.0;
                o[9 + a] = ED ? ED[15 + a] : 0.0;
            }
        }
        const double vx = o[3], vy = o[4], ax = o[6], ay = o[7];
        const double s2 = vx * vx + vy * vy;
        const bool yv = yaw_mode == TGMS_YAW_VELOCITY && s2 > 1e-6;
        o[12] = yv ? std::atan2(vy, vx) : yaw_const;
        o[13] = yv ? (vx * ay - vy * ax) / s2 : 0.0;
    }
}

}  // namespace host
}  // namespace tgms
