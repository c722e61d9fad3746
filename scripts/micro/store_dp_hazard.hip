// store_dp_hazard.hip — does a buffer store read store DATA that an FP64 VALU instruction
// wrote a few wait states earlier correctly?  (the band kernel's slab-store
// failure, second hypothesis.)
//
// The round-5 probe (store_hazard.hip) tested the store's OFFSET written by v_add / v_cndmask
// and never failed.  The unguarded band build also has every slab store's DATA written by a
// v_mul_f64 3-12 states before the store (scripts/store_hazard_scan.py, back_data), the
// multiplier comes from a DPP quad broadcast of a v_rcp_f64 result, 32-bit halves of fresh
// FP64 results are re-selected by v_cndmask, and the failing lanes were DPP bank 3 (lanes
// 12-15 of every 16-lane row).  Here every lane walks its own row of `iters` doubles; per
// iteration the shape below writes y (exact in fp64) and stores it with
// buffer_store_dwordx2 — all in ONE asm block, so the distances are what the text says.  A
// store that read y early would write the previous iteration's value.  One JSON line per
// (shape, op, D) with the wrong words per DPP bank ((lane & 15) >> 2).
//   shape 0: op; D v_mov_b32 fillers; store
//   shape 1: the band step's order: v_cmp -> SGPR mask; op; s_nop 0; v_cndmask (the store's
//            offset: lanes q = lane & 3 >= 2 out of range); D fillers; three 16/16/8-B stores
//            to a side area; the store
//   shape 2: shape 0 behind a 4-deep dependent v_fma_f64 chain on another register, so the
//            FP64 pipe is busy when y is written
//   shape 3: the multiplier path: v_rcp_f64 of a power of two (exact), DPP quad broadcast
//            from lane 3 of the quad (two v_mov_b32_dpp), v_mul_f64 by i + 1; D fillers; store
//   shape 4: op; both 32-bit halves re-selected by v_cndmask (lane 3 of each quad: 0.0, the
//            band's "column k stores 0"); D v_mov_b64 fillers; store
//   shape 5: op; D v_mov_b64 fillers; store
//   hipcc --offload-arch=gfx950 -O3 -o store_dp_hazard store_dp_hazard.hip && ./store_dp_hazard
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#define FMA4                               \
    "v_fma_f64 %[w], %[w], %[m], %[x]\n\t" \
    "v_fma_f64 %[w], %[w], %[m], %[x]\n\t" \
    "v_fma_f64 %[w], %[w], %[m], %[x]\n\t" \
    "v_fma_f64 %[w], %[w], %[m], %[x]\n\t"
#define FILL ".rept %c[d]\n\tv_mov_b32 v40, 0\n\t.endr\n\t"
#define FILLB ".rept %c[d]\n\tv_mov_b64 v[40:41], 0\n\t.endr\n\t"
#define ST "buffer_store_dwordx2 %[y], %[off], %[rs], 0 offen\n\t"
#define SIDE                                                   \
    "buffer_store_dwordx4 %[j4], %[s0], %[rside], 0 offen\n\t" \
    "buffer_store_dwordx4 %[j4], %[s1], %[rside], 0 offen\n\t" \
    "buffer_store_dwordx2 %[j2], %[s2], %[rside], 0 offen\n\t"

#define OP_MUL "v_mul_f64 %[y], %[x], %[m]\n\t"
#define OP_FMA "v_fma_f64 %[y], %[x], %[m], %[x]\n\t"
#define OP_ADD "v_add_f64 %[y], %[x], %[m]\n\t"

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

#define CLOB "v40", "v41", "memory"
#define SHAPE0(OPT) asm volatile(OPT FILL ST : [y] "=&v"(y) : [x] "v"(x), [m] "v"(m), [off] "v"(off), \
                                 [rs] "s"(rs), [d] "n"(D) : CLOB)
#define SHAPE5(OPT) asm volatile(OPT FILLB ST : [y] "=&v"(y) : [x] "v"(x), [m] "v"(m), [off] "v"(off), \
                                 [rs] "s"(rs), [d] "n"(D) : CLOB)
#define SHAPE2(OPT) asm volatile(FMA4 OPT FILL ST : [y] "=&v"(y), [w] "+v"(w) : [x] "v"(x), [m] "v"(m), \
                                 [off] "v"(off), [rs] "s"(rs), [d] "n"(D) : CLOB)
#define SHAPE1(OPT)                                                                                          \
    asm volatile("v_cmp_gt_u32_e64 %[mask], 2, %[q]\n\t" OPT "s_nop 0\n\t"                                  \
                 "v_cndmask_b32_e64 %[o], %[oor], %[off], %[mask]\n\t" FILL SIDE                            \
                 "buffer_store_dwordx2 %[y], %[o], %[rs], 0 offen\n\t"                                       \
                 : [y] "=&v"(y), [o] "=&v"(o), [mask] "=&s"(mask)                                            \
                 : [x] "v"(x), [m] "v"(m), [off] "v"(off), [q] "v"(q), [oor] "v"(0x7FFFFF00u), [rs] "s"(rs), \
                   [rside] "s"(rside), [j4] "v"(j4), [j2] "v"(j2), [s0] "v"(soff), [s1] "v"(soff + 16u),     \
                   [s2] "v"(soff + 32u), [d] "n"(D)                                                         \
                 : CLOB)

template <int SHAPE, int OP, int D>
__global__ __launch_bounds__(256) void k_dp(double* out, uint32_t* side, int iters) {
    const uint32_t gl = blockIdx.x * 256 + threadIdx.x;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(out, (short)0, (int)(gridDim.x * 256u * iters * 8u), 0x00020000);
    const __amdgpu_buffer_rsrc_t rside =
        __builtin_amdgcn_make_buffer_rsrc(side, (short)0, (int)(gridDim.x * 256u * 64u), 0x00020000);
    const double x = (double)gl + 0.5;
    const double xp = ldexp(1.0, (int)(gl & 31) - 16);  // shape 3: exact reciprocal
    const uint32_t q = threadIdx.x & 3;
    const uint32_t soff = gl * 64u;
    const u32x4 j4 = {gl, gl, gl, gl};
    const u32x2 j2 = {gl, gl};
    double y, w = 1.0;
    for (int i = 0; i < iters; ++i) {
        const double m = (double)(i + 1);
        const uint32_t off = (gl * (uint32_t)iters + (uint32_t)i) * 8u;
        uint32_t o;
        uint64_t mask;
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (SHAPE == 0) {
            if constexpr (OP == 0) SHAPE0(OP_MUL);
            else if constexpr (OP == 1) SHAPE0(OP_FMA);
            else SHAPE0(OP_ADD);
        } else if constexpr (SHAPE == 5) {
            if constexpr (OP == 0) SHAPE5(OP_MUL);
            else if constexpr (OP == 1) SHAPE5(OP_FMA);
            else SHAPE5(OP_ADD);
        } else if constexpr (SHAPE == 2) {
            if constexpr (OP == 0) SHAPE2(OP_MUL);
            else if constexpr (OP == 1) SHAPE2(OP_FMA);
            else SHAPE2(OP_ADD);
        } else if constexpr (SHAPE == 1) {
            if constexpr (OP == 0) SHAPE1(OP_MUL);
            else if constexpr (OP == 1) SHAPE1(OP_FMA);
            else SHAPE1(OP_ADD);
        } else if constexpr (SHAPE == 3) {
            // VALU write -> DPP read: 2 wait states (s_nop 1), as the compiler pads it
            asm volatile(
                "v_rcp_f64 v[42:43], %[xp]\n\t"
                "s_nop 1\n\t"
                "v_mov_b32_dpp v44, v42 quad_perm:[3,3,3,3] row_mask:0xf bank_mask:0xf\n\t"
                "v_mov_b32_dpp v45, v43 quad_perm:[3,3,3,3] row_mask:0xf bank_mask:0xf\n\t"
                "v_mul_f64 %[y], v[44:45], %[m]\n\t" FILL ST
                : [y] "=&v"(y)
                : [xp] "v"(xp), [m] "v"(m), [off] "v"(off), [rs] "s"(rs), [d] "n"(D)
                : "v40", "v41", "v42", "v43", "v44", "v45", "memory");
        } else {  // SHAPE 4
            asm volatile(
                "v_cmp_eq_u32_e64 %[mask], 3, %[q]\n\t"
                "v_mul_f64 v[42:43], %[x], %[m]\n\t"
                "s_nop 0\n\t"
                "v_cndmask_b32_e64 v43, v43, 0, %[mask]\n\t"
                "v_cndmask_b32_e64 v42, v42, 0, %[mask]\n\t" FILLB
                "buffer_store_dwordx2 v[42:43], %[off], %[rs], 0 offen\n\t"
                : [mask] "=&s"(mask)
                : [x] "v"(x), [m] "v"(m), [q] "v"(q), [off] "v"(off), [rs] "s"(rs), [d] "n"(D)
                : "v40", "v41", "v42", "v43", "memory");
            y = 0.0;
        }
        __builtin_amdgcn_sched_barrier(0);
        (void)o;
        (void)mask;
    }
    (void)q;
    (void)soff;
    (void)j4;
    (void)j2;
    (void)rside;
    (void)y;
    (void)xp;
    if (w == 12345.0) out[0] = w;  // keeps the FP64 chain of shape 2 alive
}

static double expect(int shape, int op, size_t t, double m) {
    const double x = (double)t + 0.5;
    if (shape == 3) return m * ldexp(1.0, 16 - (int)((t | 3) & 31));
    if (shape == 4) return (t & 3) == 3 ? 0.0 : x * m;
    if (shape == 1 && (t & 3) >= 2) return 0.0;  // the out-of-range lanes store nothing
    return op == 0 ? x * m : (op == 1 ? x * m + x : x + m);
}

template <int SHAPE, int OP, int D>
void run(double* d_out, uint32_t* d_side, int blocks, int iters, std::vector<double>& h, int reps) {
    const size_t n = (size_t)blocks * 256 * iters;
    long bad = 0, bad_words = 0, bank[4] = {0, 0, 0, 0}, stale = 0;
    for (int r = 0; r < reps; ++r) {
        (void)hipMemset(d_out, 0, n * 8);
        hipLaunchKernelGGL((k_dp<SHAPE, OP, D>), dim3(blocks), dim3(256), 0, 0, d_out, d_side, iters);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(h.data(), d_out, n * 8, hipMemcpyDeviceToHost);
        for (size_t t = 0; t < (size_t)blocks * 256; ++t) {
            bool tb = false;
            for (int i = 0; i < iters; ++i) {
                const double want = expect(SHAPE, OP, t, (double)(i + 1));
                const double got = h[t * iters + i];
                if (got != want) {
                    ++bad_words;
                    ++bank[(t & 15) >> 2];
                    tb = true;
                    if (i > 0 && got == expect(SHAPE, OP, t, (double)i)) ++stale;
                }
            }
            bad += tb;
        }
    }
    const char* opn = SHAPE == 3 ? "v_rcp_f64+dpp+v_mul_f64"
                                 : (OP == 0 ? "v_mul_f64" : (OP == 1 ? "v_fma_f64" : "v_add_f64"));
    printf("{\"shape\": %d, \"op\": \"%s\", \"D\": %d, \"lanes\": %d, \"iters\": %d, \"reps\": %d, "
           "\"lanes_with_a_wrong_word\": %ld, \"wrong_words\": %ld, \"wrong_by_bank\": [%ld, %ld, %ld, %ld], "
           "\"previous_iteration_value\": %ld}\n",
           SHAPE, opn, D, blocks * 256, iters, reps, bad, bad_words, bank[0], bank[1], bank[2], bank[3], stale);
    fflush(stdout);
}

template <int SHAPE, int OP, int... Ds>
void sweep(double* o, uint32_t* s, int b, int it, std::vector<double>& h, int reps) {
    (run<SHAPE, OP, Ds>(o, s, b, it, h, reps), ...);
}

int main() {
    const int blocks = 2048, iters = 64, reps = 3;  // 524,288 lanes x 64 doubles = 256 MB
    double* d_out = nullptr;
    uint32_t* d_side = nullptr;
    (void)hipMalloc(&d_out, (size_t)blocks * 256 * iters * 8);
    (void)hipMalloc(&d_side, (size_t)blocks * 256 * 64);
    std::vector<double> h((size_t)blocks * 256 * iters);
    sweep<0, 0, 0, 1, 2, 3, 4, 8, 16>(d_out, d_side, blocks, iters, h, reps);
    sweep<0, 1, 0, 1, 2, 3, 4, 8>(d_out, d_side, blocks, iters, h, reps);
    sweep<0, 2, 0, 1, 2, 4>(d_out, d_side, blocks, iters, h, reps);
    sweep<5, 0, 0, 1, 2, 3, 5, 8>(d_out, d_side, blocks, iters, h, reps);
    sweep<2, 0, 0, 1, 2, 3, 4, 8>(d_out, d_side, blocks, iters, h, reps);
    sweep<1, 0, 0, 1, 2, 3, 4, 8, 16>(d_out, d_side, blocks, iters, h, reps);
    sweep<1, 1, 0, 1, 2, 4>(d_out, d_side, blocks, iters, h, reps);
    sweep<3, 0, 0, 1, 2, 3, 4, 8>(d_out, d_side, blocks, iters, h, reps);
    sweep<4, 0, 0, 1, 2, 3, 5, 8>(d_out, d_side, blocks, iters, h, reps);
    (void)hipFree(d_out);
    (void)hipFree(d_side);
    return 0;
}
