// tgms_plan.cpp — host-only planning of the multi-GPU pipeline (see tgms_plan.h).
#include "tgms_plan.h"

#include <algorithm>

#include "tgms.h"

namespace tgms {

namespace {
size_t align256(size_t x) { return (x + 255) & ~size_t(255); }
}  // namespace

double traj_cost(int method, int32_t M) {
    const double m = (double)M;
    return method == TGMS_METHOD_DENSE_KKT ? (14.0 * m + 2.0) * (14.0 * m + 2.0) * (14.0 * m + 2.0) : 2.0 + m;
}

void plan_shards(int32_t B, const int32_t* so, int parts, int method, int32_t* bounds, int uniform_m) {
    bounds[0] = 0;
    if (B == 0) {
        for (int k = 1; k <= parts; ++k) bounds[k] = 0;
        return;
    }
    if (parts == 1) {
        bounds[1] = B;
        return;
    }
    const double wu = uniform_m > 0 ? traj_cost(method, uniform_m) : 0.0;
    if (uniform_m > 0 && (double)B * wu < 9007199254740992.0) {
        // every trajectory costs the same integer w, so while B w < 2^53 the running sum
        // is exactly (b + 1) w in fp64: the same cuts as the general rule below, by binary
        // search (beyond 2^53 the prefix sum rounds, and only the general rule matches
        // shard.ragged_bounds)
        const double w = wu;
        const double total = (double)B * w;
        int64_t prev = 0;
        for (int k = 1; k < parts; ++k) {
            const double target = (total * (double)k) / (double)parts;
            int64_t lo = 0, hi = B;  // first b with (b + 1) w >= target
            while (lo < hi) {
                const int64_t mid = (lo + hi) / 2;
                if ((double)(mid + 1) * w < target) lo = mid + 1;
                else hi = mid;
            }
            int64_t cut = std::max(lo + 1, prev);
            prev = cut;
            bounds[k] = (int32_t)std::min<int64_t>(cut, B);
        }
        bounds[parts] = B;
        return;
    }
    if (method != TGMS_METHOD_DENSE_KKT && uniform_m <= 0) {
        // the running cost 2 (b + 1) + so[b + 1] - so[0] is an integer below 2^53, so the fp64
        // prefix sum below would hold it exactly: the same cuts by binary search
        const int32_t so0 = so[0];
        auto c_at = [&](int64_t b) { return (double)(2 * (b + 1) + ((int64_t)so[b + 1] - so0)); };
        const double total = c_at(B - 1);
        int64_t prev = 0;
        for (int k = 1; k < parts; ++k) {
            const double target = (total * (double)k) / (double)parts;
            int64_t lo = 0, hi = B;  // lower_bound: first b with c(b) >= target
            while (lo < hi) {
                const int64_t mid = (lo + hi) / 2;
                if (c_at(mid) < target) lo = mid + 1;
                else hi = mid;
            }
            int64_t cut = std::max(lo + 1, prev);
            prev = cut;
            bounds[k] = (int32_t)std::min<int64_t>(cut, B);
        }
        bounds[parts] = B;
        return;
    }
    std::vector<double> c(B);
    double acc = 0.0;
    for (int32_t b = 0; b < B; ++b) {
        acc += uniform_m > 0 ? wu : traj_cost(method, so[b + 1] - so[b]);
        c[b] = acc;
    }
    int64_t prev = 0;
    for (int k = 1; k < parts; ++k) {
        const double target = (c[B - 1] * (double)k) / (double)parts;
        int64_t cut = (int64_t)(std::lower_bound(c.begin(), c.end(), target) - c.begin()) + 1;
        cut = std::max(cut, prev);  // running maximum, then capped at B
        prev = cut;
        bounds[k] = (int32_t)std::min<int64_t>(cut, B);
    }
    bounds[parts] = B;
}

bool cuts_valid(const MultiPlan& P, const int32_t* so) {
    auto ok = [](int64_t n, int64_t span) { return n >= 0 && span >= n && span <= (int64_t)TGMS_MAX_SEGMENTS * n; };
    for (int d = 0; d < P.n; ++d) {
        if (!ok(P.bounds[d + 1] - P.bounds[d], (int64_t)so[P.bounds[d + 1]] - so[P.bounds[d]])) return false;
        for (const PiecePlan& p : P.pieces[d])
            if (!ok(p.n(), p.S())) return false;
    }
    return true;
}

void plan_multi(int n, int32_t B, const int32_t* so, int method, int uniform_m, const MultiFlags& f, MultiPlan* out) {
    MultiPlan& P = *out;
    P.n = n;
    P.bounds.assign(n + 1, 0);
    P.pieces.assign(n, {});
    P.plan_bytes.assign(n, 0);
    P.ws_bytes.assign(n, 0);
    P.xfers.clear();
    P.n_groups = 2 * MULTI_PIECES;
    plan_shards(B, so, n, method, P.bounds.data(), uniform_m);
    for (int d = 0; d < n; ++d) {
        if (d == 0 && !f.self_gather) continue;  // device 0 solves its shard in place
        const int32_t lo = P.bounds[d], hi = P.bounds[d + 1];
        if (hi <= lo) continue;
        int32_t pb[MULTI_PIECES + 1];
        if (uniform_m > 0)
            plan_shards(hi - lo, nullptr, MULTI_PIECES, method, pb, uniform_m);
        else
            plan_shards(hi - lo, so + lo, MULTI_PIECES, method, pb);  // the shard's slice, no copy
        // ragged refinement loop and (round 6) ragged reduced solve: planned on the device
        // (offsets slice scattered with the inputs); ragged band / dense solve: host-planned
        // pieces (plan block uploaded)
        const bool dev_plan = uniform_m <= 0 && (f.refine || method == TGMS_METHOD_REDUCED);
        const bool host_plan = uniform_m <= 0 && !dev_plan;
        std::vector<PiecePlan>& ps = P.pieces[d];
        size_t plan_bytes = 0;
        for (int k = 0; k < MULTI_PIECES; ++k) {
            if (pb[k + 1] <= pb[k]) continue;
            PiecePlan p;
            p.lo = lo + pb[k];
            p.hi = lo + pb[k + 1];
            p.s0 = so ? so[p.lo] : (int64_t)p.lo * uniform_m;
            p.s1 = so ? so[p.hi] : (int64_t)p.hi * uniform_m;
            if (host_plan) {
                p.oSo = plan_bytes;
                plan_bytes = align256(plan_bytes + sizeof(int32_t) * (p.n() + 1));
                p.oPerm = plan_bytes;
                plan_bytes = align256(plan_bytes + sizeof(int32_t) * p.n());
            }
            ps.push_back(p);
        }
        size_t off = plan_bytes;  // the plan block (mirrored in the pinned staging) comes first
        for (PiecePlan& p : ps) {
            if (dev_plan) {
                p.oSo = off; off = align256(off + sizeof(int32_t) * (p.n() + 1));
                p.oPerm = off; off = align256(off + sizeof(int32_t) * p.n());
                p.oHist = off; off = align256(off + dev_hist_bytes(p.n()));
                p.oPlan = off; off = align256(off + DEV_PLAN_BYTES);
            } else if (!host_plan) {
                p.oSo = p.oPerm = p.oHist = p.oPlan = off;  // (empty regions)
            } else {
                p.oHist = p.oPlan = off;
            }
            p.oW = off; off = align256(off + 8 * (size_t)(p.S() + p.n()) * 3);
            p.oT = off; off = align256(off + 8 * (size_t)p.S());
            p.oT2 = off; off = align256(off + (f.refine ? 8 * (size_t)p.S() : 0));
            p.oED = off; off = align256(off + (f.has_ed ? 8 * (size_t)p.n() * 18 : 0));
            p.oC = off; off = align256(off + (f.has_c ? 8 * (size_t)p.S() * 24 : 0));
            p.oSt = off; off = align256(off + 4 * (size_t)p.n());
            p.oCost = off; off = align256(off + (f.refine ? 8 * (size_t)p.n() : 0));
        }
        P.plan_bytes[d] = plan_bytes;
        P.ws_bytes[d] = off;
    }
    // transfers: scatter group k = piece k's inputs of every device (so a device's piece
    // k can start as soon as its own group has landed), then gather group k = piece k's
    // results of every device
    for (int k = 0; k < MULTI_PIECES; ++k)
        for (int d = 0; d < n; ++d) {
            if (k >= (int)P.pieces[d].size()) continue;
            const PiecePlan& p = P.pieces[d][k];
            P.xfers.push_back({d, k, 0, XA_W, (p.s0 + p.lo) * 3, (int64_t)p.oW, (p.S() + p.n()) * 3, 8, k});
            P.xfers.push_back({d, k, 0, XA_T, p.s0, (int64_t)p.oT, p.S(), 8, k});
            if (f.has_ed) P.xfers.push_back({d, k, 0, XA_ED, (int64_t)p.lo * 18, (int64_t)p.oED, (int64_t)p.n() * 18, 8, k});
            if (uniform_m <= 0 && (f.refine || method == TGMS_METHOD_REDUCED))  // the raw offsets slice, device-planned
                P.xfers.push_back({d, k, 0, XA_SO, (int64_t)p.lo, (int64_t)p.oSo, (int64_t)p.n() + 1, 4, k});
        }
    for (int k = 0; k < MULTI_PIECES; ++k)
        for (int d = 0; d < n; ++d) {
            if (k >= (int)P.pieces[d].size()) continue;
            const PiecePlan& p = P.pieces[d][k];
            const int g = MULTI_PIECES + k;
            if (f.has_c) P.xfers.push_back({d, k, 1, XA_C, p.s0 * 24, (int64_t)p.oC, p.S() * 24, 8, g});
            if (f.has_st) P.xfers.push_back({d, k, 1, XA_ST, p.lo, (int64_t)p.oSt, p.n(), 4, g});
            if (f.refine) {
                P.xfers.push_back({d, k, 1, XA_T, p.s0, (int64_t)p.oT, p.S(), 8, g});
                if (f.has_cost) P.xfers.push_back({d, k, 1, XA_COST, p.lo, (int64_t)p.oCost, p.n(), 8, g});
            }
        }
}

}  // namespace tgms
