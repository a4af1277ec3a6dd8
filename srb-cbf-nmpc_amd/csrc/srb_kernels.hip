// Batched CBF-NMPC solver kernel for MI355X (gfx950).
//
// Replaces the per-control-cycle solve of MPC_dist::run_NMPC
// (/root/reference/src/MPC_dist.cpp:81-454): the LIP/CoP/contact-weight QP of :135-321
// solved with the iSWIFT Mehrotra predictor-corrector
// (/root/reference/optimization/iSWIFT/src/Prime.c:127-230), then the NLP stage with the
// obstacle ("CBF") and velocity rows of include/dec_vars_constr_cost.h:245-395 (SNOPT in
// the reference) solved by a primal-dual interior-point method warm-started from the QP
// solution (MPC_dist.cpp:403).
//
// Execution model: one 64-lane wavefront (= one workgroup) per agent runs the whole path
// -- nearest-obstacle selection, problem setup, both interior-point loops, output -- with
// no host round trip.  The solve is latency-bound (a few thousand dependent instructions
// per IPM iteration on one wave), so the design minimises instructions and LDS round
// trips per iteration:
//
//   * equalities (LIP dynamics, u_k = F_k lambda_k, sum lambda_k = 1) are eliminated by a
//     null-space basis: x = xbar + Z xi, xi = (lambda dofs of every grid, s),
//     nz = N(C-1)+1 (11 at N=10 trot);
//   * every inequality row lives in REGISTERS of a fixed owner lane for the whole solve:
//       - variable slot v (lane v % 64, trip v / 64): x_v, the residual rx_v and the two
//         bound pairs on x_v (A: box / lambda in [0,1]; B: velocity, NLP only);
//       - CoM-CoP slot e: the pair +-(p_i - u_{i+1}) <= mu h / sqrt 2 (row M_e = a_e'Z in LDS);
//       - obstacle slot o = k*K + j: -|p_k - o_kj|^2 - s <= -eps (row M_o = J_o Z in LDS,
//         re-linearised every iteration);
//     so residuals, step lengths and updates are straight-line VALU code with no branches
//     on row type;
//   * the reduced Newton matrix  Z'HZ = sum_t w_t r_t r_t'  over the term rows r_t (Z rows
//     of the variables with their diagonal weights, M_e, M_o) is assembled on the matrix
//     cores (v_mfma_f64_16x16x4f64, LDS operands), inverted by Gauss-Jordan with one matrix
//     row per lane and v_readlane broadcasts (no LDS inside the elimination), and every
//     Newton solve is two register matvecs plus one refinement;
//   * right-hand sides Z'(rx + J'w) are VALU dot products over the same term rows followed
//     by a permlane butterfly; J dx of every slot is its LDS term row dotted with dxi;
//   * rx is carried by the exact recurrence of the iSWIFT update (q += ad A'dy):
//       rx' = (1-ad) rx + (ad-ap) P dx + ad (hess + delta) dx - (J(x') - J(x))' z'
//     so neither J'z nor the equality multipliers are ever formed.
//
// Inputs/outputs are agent-major fp64 arrays in HBM, read once / written once.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "srb_kernel_params.h"

#define WAVE 64
#define SYNC() __syncthreads()

typedef double d4 __attribute__((ext_vector_type(4)));

// --------------------------------------------------------------------------- wave helpers
// Cross-lane traffic stays in the VALU: DPP row permutations for the 16-lane rows and
// gfx950's v_permlane16/32_swap across rows.  Every lane ends with the bit-identical
// result (each stage combines a pair with a commutative op), so branches on it are uniform.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// the two halves of a permlane swap of v with itself: {v, partner} in some order
template <int W>
__device__ __forceinline__ void swap_d(double v, double &a, double &b)
{
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)u, hi = (unsigned)(u >> 32);
    auto l = (W == 16) ? __builtin_amdgcn_permlane16_swap(lo, lo, false, false) : __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    auto h = (W == 16) ? __builtin_amdgcn_permlane16_swap(hi, hi, false, false) : __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    a = __longlong_as_double((long long)(((unsigned long long)h[0] << 32) | l[0]));
    b = __longlong_as_double((long long)(((unsigned long long)h[1] << 32) | l[1]));
}
#define SRB_WAVE_REDUCE(NAME, OP)                                                  \
    __device__ __forceinline__ double NAME(double v)                               \
    {                                                                              \
        v = OP(v, dpp_d<0xB1>(v));   /* quad_perm [1,0,3,2] */                     \
        v = OP(v, dpp_d<0x4E>(v));   /* quad_perm [2,3,0,1] */                     \
        v = OP(v, dpp_d<0x141>(v));  /* row_half_mirror     */                     \
        v = OP(v, dpp_d<0x140>(v));  /* row_mirror          */                     \
        double a, b;                                                               \
        swap_d<16>(v, a, b); v = OP(a, b);                                         \
        swap_d<32>(v, a, b); return OP(a, b);                                      \
    }
__device__ __forceinline__ double op_add(double a, double b) { return a + b; }
SRB_WAVE_REDUCE(wsum, op_add)
SRB_WAVE_REDUCE(wmin, fmin)
SRB_WAVE_REDUCE(wmax, fmax)
// sum over the lanes that share (lane mod W), W = 16 or 32: permlane butterflies only
__device__ __forceinline__ double chunk_sum16(double v)
{
    double a, b;
    swap_d<32>(v, a, b); v = a + b;
    swap_d<16>(v, a, b); return a + b;
}
__device__ __forceinline__ double chunk_sum32(double v)
{
    double a, b;
    swap_d<32>(v, a, b); return a + b;
}
// value of lane `lane` (wave-uniform index) -> wave-uniform value
__device__ __forceinline__ double readlane_d(double v, int lane)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, lane);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// 1/x from the hardware estimate (v_rcp_f64) refined by two Newton steps: within an ulp
// or two of the IEEE quotient, a handful of FMAs instead of the division sequence.
__device__ __forceinline__ double rcp_d(double x)
{
    double r = __builtin_amdgcn_rcp(x);
    r = fma(r, fma(-x, r, 1.0), r);
    r = fma(r, fma(-x, r, 1.0), r);
    return r;
}
__device__ __forceinline__ int rnd4(int x) { return (x + 3) & ~3; }

// --------------------------------------------------------------------------- diagnostic stamps
// Built only with -DSRB_STAMPS (make stamps -> srbnmpc/libsrbnmpc_stamps.so): lane 0 of
// every agent accumulates s_memtime cycles per phase into registers; agent 0 adds them to
// a device buffer nothing else reads.
#ifdef SRB_STAMPS
#define SRB_NSTAMP 64
__device__ unsigned long long srb_stamp_buf[SRB_NSTAMP];
#define STAMP_DECL unsigned long long st_acc[SRB_NSTAMP / 4] = {0}; unsigned long long st_t0 = 0
#define STAMP_BEGIN() do { __builtin_amdgcn_sched_barrier(0); st_t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); } while (0)
#define STAMP_END(slot) do { __builtin_amdgcn_sched_barrier(0); const unsigned long long _t = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0); st_acc[(slot)] += _t - st_t0; st_t0 = _t; } while (0)
#define STAMP_FLUSH(agent) do { if ((agent) == 0 && threadIdx.x == 0) for (int _i = 0; _i < SRB_NSTAMP / 4; _i++) atomicAdd(&srb_stamp_buf[_i], st_acc[_i]); } while (0)
#else
#define STAMP_DECL do {} while (0)
#define STAMP_BEGIN() do {} while (0)
#define STAMP_END(slot) do {} while (0)
#define STAMP_FLUSH(agent) do {} while (0)
#endif

// --------------------------------------------------------------------------- row state
// One bound pair on a scalar function f = a'x (row+:  f <= hp, row-: -f <= hm), or a single
// row (index 0 only).  s, z: slack and dual; the rest is per-iteration scratch.
struct Pair {
    double s[2], z[2], iz[2], is[2], dz[2], ds[2], dsT[2], r3[2];
};

// rz_r = h_r - s_r - sg_r f
__device__ __forceinline__ double rz_of(const Pair &p, int r, double f, double h)
{
    return (r == 0) ? (h - p.s[0] - f) : (h - p.s[1] + f);
}

// --------------------------------------------------------------------------- term rows
// Term row t (Z row of a variable, M_e, M_o) at rows + t * LDR; LDR = NZM + 1 (odd: lane-
// parallel row reads stay conflict-free).  Rows are zero beyond nz and beyond the count.

// out = sum_t w_t r_t r_t' (+ init): v_mfma_f64_16x16x4f64 with A[a][k] = r_{t0+k}[a],
// B[k][b] = w_{t0+k} r_{t0+k}[b]; lane l supplies term t0 + (l >> 4), column l & 15.
// D layout: row (l >> 4) + 4 q, column l & 15.  NZM = 32: tiles (0,0), (0,1), (1,1).
template <int NZM>
__device__ __forceinline__ void gram(const double *rows, const double *w, int cnt, double *out, int lane)
{
    constexpr int LDR = NZM + 1, LDH = NZM + 1;
    constexpr int NT = (NZM == 16) ? 1 : 3;
    const int li = lane & 15, kq = lane >> 4;
    d4 acc0[NT], acc1[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) { acc0[t] = d4{0.0, 0.0, 0.0, 0.0}; acc1[t] = acc0[t]; }
    int t0 = 0;
    for (; t0 + 8 <= cnt; t0 += 8) {
        const double *r0 = rows + (t0 + kq) * LDR, *r1 = r0 + 4 * LDR;
        const double w0 = w[t0 + kq], w1 = w[t0 + 4 + kq];
        if constexpr (NZM == 16) {
            const double a0 = r0[li], a1 = r1[li];
            acc0[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, w0 * a0, acc0[0], 0, 0, 0);
            acc1[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, w1 * a1, acc1[0], 0, 0, 0);
        } else {
            const double a0 = r0[li], b0 = r0[16 + li], a1 = r1[li], b1 = r1[16 + li];
            acc0[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, w0 * a0, acc0[0], 0, 0, 0);
            acc0[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, w0 * b0, acc0[1], 0, 0, 0);
            acc0[2] = __builtin_amdgcn_mfma_f64_16x16x4f64(b0, w0 * b0, acc0[2], 0, 0, 0);
            acc1[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, w1 * a1, acc1[0], 0, 0, 0);
            acc1[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, w1 * b1, acc1[1], 0, 0, 0);
            acc1[2] = __builtin_amdgcn_mfma_f64_16x16x4f64(b1, w1 * b1, acc1[2], 0, 0, 0);
        }
    }
    if (t0 < cnt) {                      // cnt is a multiple of 4
        const double *r0 = rows + (t0 + kq) * LDR;
        const double w0 = w[t0 + kq];
        if constexpr (NZM == 16) {
            const double a0 = r0[li];
            acc0[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, w0 * a0, acc0[0], 0, 0, 0);
        } else {
            const double a0 = r0[li], b0 = r0[16 + li];
            acc0[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, w0 * a0, acc0[0], 0, 0, 0);
            acc0[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, w0 * b0, acc0[1], 0, 0, 0);
            acc0[2] = __builtin_amdgcn_mfma_f64_16x16x4f64(b0, w0 * b0, acc0[2], 0, 0, 0);
        }
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int r = kq + 4 * q;
        out[r * LDH + li] = acc0[0][q] + acc1[0][q];
        if constexpr (NZM == 32) {
            const double v01 = acc0[1][q] + acc1[1][q];
            out[r * LDH + 16 + li] = v01;
            out[(16 + li) * LDH + r] = v01;
            out[(16 + r) * LDH + 16 + li] = acc0[2][q] + acc1[2][q];
        }
    }
}

// out[a] = sum_t c_t r_t[a] for a < nz (VALU): lane (a, chunk) sums the terms of its chunk,
// the chunks combine by permlane swaps.  cnt is a multiple of 4.
template <int NZM>
__device__ __forceinline__ void rmul(const double *rows, const double *cf, int cnt, double *out, int nz, int lane)
{
    constexpr int LDR = NZM + 1;
    constexpr int NCH = 64 / NZM;            // term chunks (4 or 2)
    const int a = lane % NZM, q = lane / NZM;
    double s0 = 0.0, s1 = 0.0;
    int t = q;
    for (; t + NCH < cnt; t += 2 * NCH) {
        s0 = fma(cf[t], rows[t * LDR + a], s0);
        s1 = fma(cf[t + NCH], rows[(t + NCH) * LDR + a], s1);
    }
    if (t < cnt) s0 = fma(cf[t], rows[t * LDR + a], s0);
    double s = s0 + s1;
    s = (NZM == 16) ? chunk_sum16(s) : chunk_sum32(s);
    if (q == 0 && a < nz) out[a] = s;
}

// dot of LDS term row (lane-parallel rows) with a wave-uniform vector held in registers
template <int NZL>
__device__ __forceinline__ double row_dot(const double *row, const double (&v)[NZL])
{
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int j = 0; j + 1 < NZL; j += 2) { s0 = fma(row[j], v[j], s0); s1 = fma(row[j + 1], v[j + 1], s1); }
    if (NZL & 1) s0 = fma(row[NZL - 1], v[NZL - 1], s0);
    return s0 + s1;
}

// --------------------------------------------------------------------------- Gauss-Jordan
// In-place inverse of the nz x nz SPD matrix held one row per lane (lane i: A[0..NZL)),
// rows/columns >= nz padded with the identity.  Step k: the pivot row is broadcast by
// v_readlane; every lane updates its row.  The pivots are those of LDL' in natural order,
// so pivot <= 0 <=> not positive definite; regularise != 0 applies iSWIFT's dynamic pivot
// regularisation (ldl.c:320-321: |D_kk| <= 1e-14 -> 1e-7).  Returns 0 on success (uniform).
template <int NZL>
__device__ __forceinline__ int gj_invert(double (&A)[NZL], int nz, int lane, int regularise)
{
    int fail = 0;
#pragma unroll
    for (int k = 0; k < NZL; k++) {
        if (k >= nz) break;
        double piv = readlane_d(A[k], k);
        if (regularise && piv <= 1e-14 && piv == piv) piv = 1e-7;
        fail |= !(piv > 0.0);
        const double inv = rcp_d(piv);
        double rk[NZL];
#pragma unroll
        for (int j = 0; j < NZL; j++) rk[j] = readlane_d(A[j], k);
        const double fi = A[k] * inv;
        const bool me = lane == k;
#pragma unroll
        for (int j = 0; j < NZL; j++) A[j] = me ? rk[j] * inv : fma(-fi, rk[j], A[j]);
        A[k] = me ? inv : -fi;
    }
    return fail;
}

// lane i (< NZL) loads row i of H (+ delta * Z'Z) with identity padding
template <int NZL>
__device__ __forceinline__ void gj_load(double (&A)[NZL], const double *H, const double *ZtZ, double delta, int nz, int lane)
{
    constexpr int LDH = ((NZL + 15) / 16) * 16 + 1;
    const int i = (lane < NZL) ? lane : 0;
#pragma unroll
    for (int j = 0; j < NZL; j++) {
        double v = H[i * LDH + j];
        if (delta != 0.0) v = fma(delta, ZtZ[i * LDH + j], v);
        A[j] = (lane < nz && j < nz) ? v : ((lane == j) ? 1.0 : 0.0);
    }
}

// Newton solve in the reduced space: out = Hs^-1 g with one step of iterative refinement
// (y = M g; y += M (g - Hs y)): the explicit inverse alone is not backward stable, and near
// the end of an interior-point solve Hs carries barrier weights of 1e8..1e12.
// g, y, r, out: LDS vectors (zero beyond nz).  Returns out in registers (uniform).
template <int NZL>
__device__ __forceinline__ void la_solve(const double (&M)[NZL], const double *Hs, const double *g, double *y,
                                         double *r, double *out, double (&res)[NZL], int nz, int lane)
{
    constexpr int LDH = ((NZL + 15) / 16) * 16 + 1;
    const int i = (lane < NZL) ? lane : 0;
    double gv[NZL];
#pragma unroll
    for (int j = 0; j < NZL; j++) gv[j] = g[j];
    double y0 = 0.0;
#pragma unroll
    for (int j = 0; j < NZL; j++) y0 = fma(M[j], gv[j], y0);
    if (lane < nz) y[lane] = y0;
    SYNC();
    double rr = (lane < nz) ? g[lane] : 0.0;
#pragma unroll
    for (int j = 0; j < NZL; j++) rr = fma(-Hs[i * LDH + j], y[j], rr);
    if (lane < nz) r[lane] = rr;
    SYNC();
    double y1 = y0;
#pragma unroll
    for (int j = 0; j < NZL; j++) y1 = fma(M[j], r[j], y1);
    if (lane < nz) out[lane] = y1;
    SYNC();
#pragma unroll
    for (int j = 0; j < NZL; j++) res[j] = out[j];
}

// --------------------------------------------------------------------------- null space
// Basis of the per-grid contact-weight directions {d : 1'd = 0} (lambda = e_{C-1} + N xi).
// Columns e_i - e_{C-1}, except for C = 4, where one column is replaced by the exact null
// vector n of [F; 1'] (u = F lambda unchanged): its U and X parts are identically zero, so
// the vanishing curvature along it near convergence (both lambda bounds inactive) is held
// exactly in Z'HZ instead of emerging from cancellation between O(1e3) terms.
// Returns 1 when column t is that null column (lam holds it), 0 otherwise.
__device__ __forceinline__ int lambda_basis(const double *F, int C, int t, double lam[4])
{
    for (int i = 0; i < 4; i++) lam[i] = 0.0;
    if (C != 4) { lam[t] = 1.0; lam[C - 1] = -1.0; return 0; }
    double nvec[4];
    for (int i = 0; i < 4; i++) {
        int cidx[3], q = 0;
        for (int k = 0; k < 4; k++) if (k != i) cidx[q++] = k;
        const double *r0 = F, *r1 = F + 4;
        double det = r0[cidx[0]] * (r1[cidx[1]] - r1[cidx[2]]) - r0[cidx[1]] * (r1[cidx[0]] - r1[cidx[2]]) +
                     r0[cidx[2]] * (r1[cidx[0]] - r1[cidx[1]]);
        nvec[i] = (i & 1) ? -det : det;
    }
    int istar = 0;
    for (int i = 1; i < 3; i++) if (fabs(nvec[i]) > fabs(nvec[istar])) istar = i;
    double sc = 1.0 / nvec[istar];
    if (t == 2) { for (int i = 0; i < 4; i++) lam[i] = nvec[i] * sc; return 1; }
    int i = (t < istar) ? t : t + 1;
    lam[i] = 1.0; lam[3] = -1.0;
    return 0;
}

// --------------------------------------------------------------------------- kNN
// (d, index) lexicographic wave argmin; every lane gets the winner
__device__ __forceinline__ void wargmin(double &d, int &idx)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double od = __shfl_xor(d, o, WAVE);
        const int oi = __shfl_xor(idx, o, WAVE);
        if (od < d || (od == d && oi < idx)) { d = od; idx = oi; }
    }
}

// K nearest rows of a table (row i at tab[stride*i], x at +0, y at +1) to (px, py),
// ascending in (d^2, index) -- the order of the reference's strict-'<' scan
// (MPC_dist.cpp:373-382) -- excluding row `self`; indices to sel[0..K).  The wave scans
// the table once: every lane keeps a sorted top-K of its own rows (visited in increasing
// index, so a strict '<' keeps the lower index on ties), then K rounds of a wave argmin
// over the lane heads pop the global order.  Rows stream from L2 coalesced across lanes.
__device__ __forceinline__ void knn_select(int lane, double px, double py, const double *__restrict__ tab,
                                           int stride, int n_rows, int self, int K, int *sel)
{
    double bd[SRB_KNN_MAX]; int bi[SRB_KNN_MAX];
#pragma unroll
    for (int j = 0; j < SRB_KNN_MAX; j++) { bd[j] = 1e300; bi[j] = 0x7fffffff; }
    double wd = 1e300;
    for (int i = lane; i < n_rows; i += WAVE) {
        const double dx = tab[(size_t)stride * i] - px, dy = tab[(size_t)stride * i + 1] - py;
        const double d = dx * dx + dy * dy;
        if (i == self || !(d < wd)) continue;
        double cd = d; int ci = i;
#pragma unroll
        for (int j = 0; j < SRB_KNN_MAX; j++) {
            const bool lt = (j < K) && (cd < bd[j]);
            const double td = bd[j]; const int ti = bi[j];
            bd[j] = lt ? cd : td; bi[j] = lt ? ci : ti;
            cd = lt ? td : cd; ci = lt ? ti : ci;
        }
#pragma unroll
        for (int j = 0; j < SRB_KNN_MAX; j++)
            if (j == K - 1) wd = bd[j];
    }
#pragma clang loop unroll(disable)
    for (int j = 0; j < K; j++) {
        double d = bd[0]; int idx = bi[0];
        wargmin(d, idx);
        if (bi[0] == idx) {
#pragma unroll
            for (int t = 0; t + 1 < SRB_KNN_MAX; t++) { bd[t] = bd[t + 1]; bi[t] = bi[t + 1]; }
            bd[SRB_KNN_MAX - 1] = 1e300; bi[SRB_KNN_MAX - 1] = 0x7fffffff;
        }
        if (lane == 0) sel[j] = (idx == 0x7fffffff) ? -1 : idx;
    }
}

// --------------------------------------------------------------------------- main kernel
// NZL: register bound on nz (rows of the reduced system, one per lane); TV / TO: trips of
// 64 variable / obstacle slots.  CoM-CoP slots use one trip (N <= 33).
template <int NZL, int TV, int TO>
__device__ __forceinline__ void nmpc_agent(const SrbKParams &prm, int agent,
                const double *__restrict__ x0g, const double *__restrict__ refg, const double *__restrict__ footg,
                const double *__restrict__ obstacles, int n_obs,
                const double *__restrict__ nbr_state, int n_all, int agent_offset,
                double *__restrict__ x_qp_out, double *__restrict__ x_out,
                double *__restrict__ obj_out, int *__restrict__ status_out, int *__restrict__ iters_out,
                double *lds)
{
    constexpr int NZM = ((NZL + 15) / 16) * 16;
    constexpr int LDR = NZM + 1, LDH = NZM + 1;
    const int lane = threadIdx.x;
    const int N = prm.N, C = prm.C, K = prm.K_obs + prm.K_nbr, n = prm.n, nz = prm.nz;
    const int NK = N * K, NE = 2 * (N - 1);
    const int n4 = rnd4(n), E4 = rnd4(NE), NK4 = rnd4(NK);
    const int TT = n4 + E4 + NK4;                       // term rows: variables | CoM-CoP | obstacles
    const double tol = prm.tol, th = tol / sqrt(3.0);
    STAMP_DECL;

    // ---- LDS carve (must match srb_lds_doubles)
    double *p = lds;
    double *R = p; p += TT * LDR;                       // term rows (Z rows first)
    double *W = p; p += TT;                             // gram weights
    double *CF = p; p += TT;                            // rhs coefficients
    double *H0 = p; p += NZM * LDH;                     // assembled Z'HZ (delta = 0)
    double *HS = p; p += NZM * LDH;                     // Z'HZ + delta Z'Z (when delta != 0)
    double *ZZ = p; p += NZM * LDH;                     // Z'Z (NLP)
    double *vg = p; p += NZM; double *vy = p; p += NZM; double *vr = p; p += NZM; double *vd = p; p += NZM;
    double *xs = p; p += n4;                            // current x
    double *xb = p; p += n4;                            // xbar
    double *ref = p; p += 4 * N;
    double *foot = p; p += 2 * C * N;
    double *obs = p; p += 2 * NK + 2;
    double *eps = p; p += K + 1;
    double *zo = p; p += NK4;                           // obstacle duals (per-grid sums)
    int *sel = (int *)p; p += (K + 1);
    double *Rt = R + n4 * LDR;                          // CoM-CoP rows, then obstacle rows
    double *Ro = Rt + E4 * LDR;

    STAMP_BEGIN();
    // ---- load inputs (a1/a2/a3: x0, reference window, footholds); zero the padded tables
    const double *x0 = x0g + 4 * (size_t)agent;
    for (int i = lane; i < 4 * N; i += WAVE) ref[i] = refg[(size_t)agent * 4 * N + i];
    for (int i = lane; i < 2 * C * N; i += WAVE) foot[i] = footg[(size_t)agent * 2 * C * N + i];
    for (int i = lane; i < (int)(xs - R) + 2 * n4; i += WAVE) R[i] = 0.0;     // tables, matrices, vectors, xs, xb
    for (int i = lane; i < NK4; i += WAVE) zo[i] = 0.0;
    SYNC();

    // ---- null-space basis Z and particular point xbar (forward LIP rollout, MPC_dist.cpp:232-261)
    if (lane == 0) {
        double X[4] = {x0[0], x0[1], x0[2], x0[3]};
        for (int k = 0; k < N; k++) {
            const double u0 = foot[(k * 2 + 0) * C + C - 1], u1 = foot[(k * 2 + 1) * C + C - 1];
            double Xn[4];
            for (int d = 0; d < 4; d++)
                Xn[d] = prm.Ad[d * 4] * X[0] + prm.Ad[d * 4 + 1] * X[1] + prm.Ad[d * 4 + 2] * X[2] + prm.Ad[d * 4 + 3] * X[3] +
                        prm.Bd[d * 2] * u0 + prm.Bd[d * 2 + 1] * u1;
            for (int d = 0; d < 4; d++) { X[d] = Xn[d]; xb[4 * k + d] = Xn[d]; }
            xb[4 * N + 2 * k] = u0; xb[4 * N + 2 * k + 1] = u1;
            for (int j = 0; j < C; j++) xb[6 * N + C * k + j] = (j == C - 1) ? 1.0 : 0.0;
        }
        xb[n - 1] = 0.0;
    }
    for (int col = lane; col < nz - 1; col += WAVE) {
        const int j = col / (C - 1), t = col % (C - 1);
        double lam[4];
        const int is_null = lambda_basis(foot + j * 2 * C, C, t, lam);
        double g0 = 0.0, g1 = 0.0;
        if (!is_null)
            for (int i = 0; i < C; i++) { g0 += foot[(j * 2 + 0) * C + i] * lam[i]; g1 += foot[(j * 2 + 1) * C + i] * lam[i]; }
        for (int i = 0; i < C; i++) R[(6 * N + C * j + i) * LDR + col] = lam[i];
        R[(4 * N + 2 * j) * LDR + col] = g0;
        R[(4 * N + 2 * j + 1) * LDR + col] = g1;
        double v[4];
        for (int d = 0; d < 4; d++) v[d] = prm.Bd[d * 2] * g0 + prm.Bd[d * 2 + 1] * g1;
        for (int k = j; k < N; k++) {
            for (int d = 0; d < 4; d++) R[(4 * k + d) * LDR + col] = v[d];
            double tt[4];
            for (int d = 0; d < 4; d++) tt[d] = prm.Ad[d * 4] * v[0] + prm.Ad[d * 4 + 1] * v[1] + prm.Ad[d * 4 + 2] * v[2] + prm.Ad[d * 4 + 3] * v[3];
            for (int d = 0; d < 4; d++) v[d] = tt[d];
        }
    }
    if (lane == 0) R[(n - 1) * LDR + nz - 1] = 1.0;
    SYNC();
    // CoM-CoP term rows M_e = Z_p - Z_u (p = CoM position of grid i, u = CoP of grid i+1)
    const int e_i = lane >> 1, e_d = lane & 1;
    const int e_p = 4 * e_i + 2 * e_d, e_u = 4 * N + 2 * (e_i + 1) + e_d;
    const bool e_on = lane < NE;
    if (e_on)
        for (int a = 0; a < NZM; a++) Rt[lane * LDR + a] = R[e_p * LDR + a] - R[e_u * LDR + a];

    // ---- slot constants
    // variable slots: v = lane + 64 t
    double xv[TV], rx[TV], Pv[TV], cv[TV], hAp[TV], hAm[TV];
    bool vok[TV], aon[TV], vel[TV], pos[TV];
    Pair A[TV], B[TV];
#pragma unroll
    for (int t = 0; t < TV; t++) {
        const int v = lane + 64 * t;
        vok[t] = v < n;
        const bool isX = v < 4 * N, isU = !isX && v < 6 * N, isL = !isX && !isU && v < n - 1;
        Pv[t] = isX ? ((v >= 4 * (N - 1)) ? prm.Pw : prm.Qw) : isU ? prm.Rw : isL ? 0.0 : (v == n - 1 ? prm.Sw : 0.0);
        cv[t] = isX ? -Pv[t] * ref[v] : 0.0;
        xv[t] = vok[t] ? xb[v] : 0.0;
        rx[t] = 0.0;
        aon[t] = vok[t] && v < n - 1;
        hAp[t] = isL ? 1.0 : prm.box;
        hAm[t] = isL ? 0.0 : prm.box;
        vel[t] = isX && (v & 1);
        pos[t] = isX && !(v & 1);
#pragma unroll
        for (int r = 0; r < 2; r++) { A[t].s[r] = A[t].z[r] = B[t].s[r] = B[t].z[r] = 1.0; }
    }
    Pair E;                                                  // CoM-CoP slot (one trip)
    E.s[0] = E.s[1] = E.z[0] = E.z[1] = 1.0;
    const double fr = prm.fr;
    // obstacle slots: o = lane + 64 t  (grid k = o / K, obstacle j = o % K)
    Pair O[TO];
    bool ook[TO];
    int ok_[TO];
    double ox[TO], oy[TO], oh[TO];
#pragma unroll
    for (int t = 0; t < TO; t++) {
        O[t].s[0] = O[t].z[0] = 1.0;
        ook[t] = false; ok_[t] = 0; ox[t] = oy[t] = 0.0; oh[t] = 0.0;
    }
    double Mi[NZL];                                          // inverse of the reduced Newton matrix (row = lane)
    double dxi[NZL];                                         // Newton direction in xi (uniform)
#pragma unroll
    for (int j = 0; j < NZL; j++) { Mi[j] = (lane == j) ? 1.0 : 0.0; dxi[j] = 0.0; }
    SYNC();
    STAMP_END(0);

    int qp_flag = 3, qp_it = 0, nlp_flag = 0, nlp_it = 0;
    const int nstage = prm.use_nlp ? 2 : 1;
    const int nchunk_v = (n + 63) / 64, nchunk_o = (NK + 63) / 64;
    // One loop over the two stages so that the interior-point iteration exists once in the
    // code object (keeps the hot loop small for the instruction cache).
#pragma clang loop unroll(disable)
    for (int stage = 0; stage < nstage; stage++) {
        const bool nl = stage == 1;
        int mrows = 0;                                        // active rows (m)
        int cnt = n4 + E4 + (nl ? NK4 : 0);                   // term rows in this stage
        STAMP_BEGIN();
        if (!nl) {
            // ---------------- QP stage setup: kkt_initialize (Auxilary.c:680-755) ----------------
            // [P A' G'; A 0 0; G 0 -I] [x; y; z] = [-c; b; h]  ->  reduced:  (Z'(P + G'G)Z) xi = -Z'(P xbar + c) + Z'G'(h - G xbar)
            mrows = 2 * NE + 2 * (6 * N) + 2 * C * N;         // 4(N-1) + 12N + 2CN
#pragma unroll
            for (int t = 0; t < TV; t++)
                if (t < nchunk_v) {
                    const int v = lane + 64 * t;
                    const double wA = aon[t] ? 2.0 : 0.0;
                    // w = r3 = h - G xbar on both rows of pair A
                    const double wp = hAp[t] - xv[t], wm = hAm[t] + xv[t];
                    if (v < n4) {
                        W[v] = vok[t] ? Pv[t] + wA : 0.0;
                        CF[v] = vok[t] ? (-cv[t] - Pv[t] * xv[t]) + (aon[t] ? (wp - wm) : 0.0) : 0.0;
                    }
                }
            {
                const double ge = e_on ? xb[e_p] - xb[e_u] : 0.0;
                if (lane < E4) { W[n4 + lane] = e_on ? 2.0 : 0.0; CF[n4 + lane] = e_on ? ((fr - ge) - (fr + ge)) : 0.0; }
            }
            SYNC();
            gram<NZM>(R, W, cnt, H0, lane);
            rmul<NZM>(R, CF, cnt, vg, nz, lane);
            SYNC();
            gj_load<NZL>(Mi, H0, ZZ, 0.0, nz, lane);
            if (gj_invert<NZL>(Mi, nz, lane, 1) != 0) {
                qp_flag = 1;
                // x stays xbar (as the reference, the last iterate is returned)
#pragma unroll
                for (int t = 0; t < TV; t++) if (t < nchunk_v && vok[t]) xs[lane + 64 * t] = xv[t];
                SYNC();
                continue;
            }
            la_solve<NZL>(Mi, H0, vg, vy, vr, vd, dxi, nz, lane);
            // x = xbar + Z xi ; zi = h - G x ; s, z shifted (Auxilary.c:716-746)
            double mn = 1e300, mx = -1e300;
#pragma unroll
            for (int t = 0; t < TV; t++)
                if (t < nchunk_v) {
                    const int v = lane + 64 * t;
                    const double dx = row_dot<NZL>(R + (v < n4 ? v : 0) * LDR, dxi);
                    if (vok[t]) xv[t] += dx;
                    if (aon[t]) {
                        const double zp = hAp[t] - xv[t], zm = hAm[t] + xv[t];
                        A[t].s[0] = zp; A[t].s[1] = zm;               // zi, shifted below
                        mn = fmin(mn, fmin(zp, zm)); mx = fmax(mx, fmax(zp, zm));
                    }
                }
            double ge = 0.0;
            if (e_on) {
                ge = xb[e_p] - xb[e_u] + row_dot<NZL>(Rt + lane * LDR, dxi);
                const double zp = fr - ge, zm = fr + ge;
                E.s[0] = zp; E.s[1] = zm;
                mn = fmin(mn, fmin(zp, zm)); mx = fmax(mx, fmax(zp, zm));
            }
            mn = wmin(mn); mx = wmax(mx);
            const double sa = -mn, za = mx;
            const double ssh = (sa < 0) ? 0.0 : 1.0 + sa, zsh = (za < 0) ? 0.0 : 1.0 + za;
#pragma unroll
            for (int t = 0; t < TV; t++)
                if (t < nchunk_v) {
#pragma unroll
                    for (int r = 0; r < 2; r++) {
                        const double zi = A[t].s[r];
                        A[t].s[r] = aon[t] ? zi + ssh : 1.0;
                        A[t].z[r] = aon[t] ? -zi + zsh : 1.0;
                    }
                    if (vok[t]) xs[lane + 64 * t] = xv[t];
                    rx[t] = 0.0;      // = G'(dz_init - z) = -(1+za) G'1 = 0: every G row comes in a +- pair
                }
#pragma unroll
            for (int r = 0; r < 2; r++) {
                const double zi = E.s[r];
                E.s[r] = e_on ? zi + ssh : 1.0;
                E.z[r] = e_on ? -zi + zsh : 1.0;
            }
            SYNC();
            STAMP_END(1);
        } else {
            // ---------------- NLP stage setup (replaces SnoptSolver::Solve, MPC_dist.cpp:402-427) ----------------
            if (x_qp_out)
#pragma unroll
                for (int t = 0; t < TV; t++) if (t < nchunk_v && vok[t]) x_qp_out[(size_t)agent * n + lane + 64 * t] = xv[t];
            mrows = 2 * NE + 2 * (6 * N) + 2 * C * N + NK + 4 * N;
            // obstacles per grid: the K_obs nearest static obstacles (MPC_dist.cpp:371-396,
            // generalised to K) and the K_nbr nearest other agents (get_lastState() rows),
            // predicted at constant velocity o_k = p + v Ts (k+1); query point = own CoM.
#pragma clang loop unroll(disable)
            for (int tsel = 0; tsel < 2; tsel++) {
                const int Kt = tsel ? prm.K_nbr : prm.K_obs;
                if (Kt > 0)
                    knn_select(lane, x0[0], x0[2], tsel ? nbr_state : obstacles, tsel ? 4 : 2, tsel ? n_all : n_obs,
                               tsel ? agent_offset + agent : -1, Kt, sel + (tsel ? prm.K_obs : 0));
            }
            SYNC();
            for (int j = 0; j < K; j++) {
                const bool st = j < prm.K_obs;
                const int bi = sel[j];
                if (lane < N && bi >= 0) {
                    const int k = lane;
                    const double tt = st ? 0.0 : prm.Ts * (k + 1);
                    const double *srcp = st ? obstacles + 2 * (size_t)bi : nbr_state + 4 * (size_t)bi;
                    obs[2 * (k * K + j)] = srcp[0] + (st ? 0.0 : srcp[2] * tt);
                    obs[2 * (k * K + j) + 1] = srcp[1] + (st ? 0.0 : srcp[3] * tt);
                }
                if (lane == 0) eps[j] = st ? prm.eps_obs : prm.eps_nbr;
            }
            SYNC();
            // slacks: shifted h - g(x) over every NLP row; duals 1
            double mn = 1e300;
#pragma unroll
            for (int t = 0; t < TV; t++)
                if (t < nchunk_v) {
                    if (aon[t]) mn = fmin(mn, fmin(hAp[t] - xv[t], hAm[t] + xv[t]));
                    if (vel[t]) mn = fmin(mn, fmin(prm.vsat - xv[t], prm.vsat + xv[t]));
                }
            const double ge0 = e_on ? xs[e_p] - xs[e_u] : 0.0;
            if (e_on) mn = fmin(mn, fmin(fr - ge0, fr + ge0));
            const double s_var = xs[n - 1];
#pragma unroll
            for (int t = 0; t < TO; t++) {
                const int o = lane + 64 * t;
                ook[t] = o < NK;
                const int k = ook[t] ? o / K : 0, j = ook[t] ? o - (o / K) * K : 0;
                ok_[t] = k;
                ox[t] = ook[t] ? obs[2 * o] : 0.0; oy[t] = ook[t] ? obs[2 * o + 1] : 0.0;
                oh[t] = ook[t] ? -eps[j] : 0.0;
                if (ook[t]) {
                    const double dx = xs[4 * k] - ox[t], dy = xs[4 * k + 2] - oy[t];
                    const double g = -(dx * dx + dy * dy) - s_var;
                    mn = fmin(mn, oh[t] - g);
                }
            }
            mn = wmin(mn);
            const double sa = -mn, ssh = (sa < 0) ? 0.0 : 1.0 + sa;
#pragma unroll
            for (int t = 0; t < TV; t++)
                if (t < nchunk_v) {
                    A[t].s[0] = aon[t] ? hAp[t] - xv[t] + ssh : 1.0;
                    A[t].s[1] = aon[t] ? hAm[t] + xv[t] + ssh : 1.0;
                    B[t].s[0] = vel[t] ? prm.vsat - xv[t] + ssh : 1.0;
                    B[t].s[1] = vel[t] ? prm.vsat + xv[t] + ssh : 1.0;
#pragma unroll
                    for (int r = 0; r < 2; r++) { A[t].z[r] = 1.0; B[t].z[r] = 1.0; }
                }
            E.s[0] = e_on ? fr - ge0 + ssh : 1.0;
            E.s[1] = e_on ? fr + ge0 + ssh : 1.0;
            E.z[0] = E.z[1] = 1.0;
#pragma unroll
            for (int t = 0; t < TO; t++) {
                const int o = lane + 64 * t, k = ok_[t];
                const double dx = xs[4 * k] - ox[t], dy = xs[4 * k + 2] - oy[t];
                const double g = -(dx * dx + dy * dy) - s_var;
                O[t].s[0] = ook[t] ? oh[t] - g + ssh : 1.0;
                O[t].z[0] = 1.0;
                // M_o = J_o Z at the current x
                const double jx = -2.0 * dx, jy = -2.0 * dy;
                if (o < NK4)
#pragma unroll
                    for (int a = 0; a < NZM; a++)
                        Ro[o * LDR + a] = ook[t] ? fma(jx, R[(4 * k) * LDR + a], jy * R[(4 * k + 2) * LDR + a]) - (a == nz - 1 ? 1.0 : 0.0) : 0.0;
            }
            // Z'Z (delta shifts) and the projection rx0 = -Z (Z'Z)^-1 Z'(P x + c + J'z), z = 1:
            // J'1 vanishes on every +- pair, leaving the obstacle rows.
#pragma unroll
            for (int t = 0; t < TV; t++)
                if (t < nchunk_v) {
                    const int v = lane + 64 * t;
                    if (v < n4) { W[v] = vok[t] ? 1.0 : 0.0; CF[v] = vok[t] ? fma(Pv[t], xv[t], cv[t]) : 0.0; }
                }
            if (lane < E4) { W[n4 + lane] = 0.0; CF[n4 + lane] = 0.0; }
#pragma unroll
            for (int t = 0; t < TO; t++) {
                const int o = lane + 64 * t;
                if (o < NK4) { W[n4 + E4 + o] = 0.0; CF[n4 + E4 + o] = ook[t] ? 1.0 : 0.0; }
            }
            SYNC();
            gram<NZM>(R, W, n4, ZZ, lane);
            rmul<NZM>(R, CF, cnt, vg, nz, lane);
            SYNC();
            gj_load<NZL>(Mi, ZZ, ZZ, 0.0, nz, lane);
            gj_invert<NZL>(Mi, nz, lane, 0);
            la_solve<NZL>(Mi, ZZ, vg, vy, vr, vd, dxi, nz, lane);
#pragma unroll
            for (int t = 0; t < TV; t++)
                if (t < nchunk_v) {
                    const int v = lane + 64 * t;
                    rx[t] = vok[t] ? -row_dot<NZL>(R + (v < n4 ? v : 0) * LDR, dxi) : 0.0;
                }
            SYNC();
            STAMP_END(2);
        }

        // =============================== interior-point iterations ===============================
        const int maxit = nl ? prm.nlp_maxit : prm.qp_maxit;
        double sigma = 100.0;            // options->sigma = SIGMA
        const double sigma_d = 0.0;
        int flag = 2, it = 0;
        const double inv_m = 1.0 / (double)mrows;
        for (int iter = 0; iter < maxit; iter++) {
            STAMP_BEGIN();
            // ---- residuals (computeresiduals, Auxilary.c:524-553), norms, reciprocals
            const double s_var = xs[n - 1];
            const double ge = e_on ? xs[e_p] - xs[e_u] : 0.0;
            double go[TO];
            double nrx = 0.0, nrz = 0.0, sz = 0.0, gm = 1.0;
#pragma unroll
            for (int t = 0; t < TV; t++)
                if (t < nchunk_v) {
                    nrx = fma(rx[t], rx[t], nrx);
                    if (nl && vok[t]) gm = fmax(gm, fabs(fma(Pv[t], xv[t], cv[t])));
#pragma unroll
                    for (int r = 0; r < 2; r++) {
                        const double rzA = rz_of(A[t], r, xv[t], r ? hAm[t] : hAp[t]);
                        const double rzB = rz_of(B[t], r, xv[t], prm.vsat);
                        const bool bon = nl && vel[t];
                        nrz += (aon[t] ? rzA * rzA : 0.0) + (bon ? rzB * rzB : 0.0);
                        sz += (aon[t] ? A[t].s[r] * A[t].z[r] : 0.0) + (bon ? B[t].s[r] * B[t].z[r] : 0.0);
                        A[t].iz[r] = rcp_d(A[t].z[r]); A[t].is[r] = rcp_d(A[t].s[r]);
                        B[t].iz[r] = rcp_d(B[t].z[r]); B[t].is[r] = rcp_d(B[t].s[r]);
                    }
                }
#pragma unroll
            for (int r = 0; r < 2; r++) {
                const double rzE = rz_of(E, r, ge, fr);
                nrz += e_on ? rzE * rzE : 0.0;
                sz += e_on ? E.s[r] * E.z[r] : 0.0;
                E.iz[r] = rcp_d(E.z[r]); E.is[r] = rcp_d(E.s[r]);
            }
#pragma unroll
            for (int t = 0; t < TO; t++) {
                go[t] = 0.0;
                if (nl && t < nchunk_o) {
                    const int k = ok_[t];
                    const double dx = xs[4 * k] - ox[t], dy = xs[4 * k + 2] - oy[t];
                    go[t] = -(dx * dx + dy * dy) - s_var;
                    const double rzO = rz_of(O[t], 0, go[t], oh[t]);
                    nrz += ook[t] ? rzO * rzO : 0.0;
                    sz += ook[t] ? O[t].s[0] * O[t].z[0] : 0.0;
                    O[t].iz[0] = rcp_d(O[t].z[0]); O[t].is[0] = rcp_d(O[t].s[0]);
                    // re-linearise: M_o = J_o(x) Z
                    const double jx = -2.0 * dx, jy = -2.0 * dy;
                    const int o = lane + 64 * t;
                    if (o < NK4)
#pragma unroll
                        for (int a = 0; a < NZM; a++)
                            Ro[o * LDR + a] = ook[t] ? fma(jx, R[(4 * k) * LDR + a], jy * R[(4 * k + 2) * LDR + a]) - (a == nz - 1 ? 1.0 : 0.0) : 0.0;
                    if (o < NK4) zo[o] = ook[t] ? O[t].z[0] : 0.0;
                }
            }
            nrx = sqrt(wsum(nrx)); nrz = sqrt(wsum(nrz)); sz = wsum(sz);
            if (nl) gm = wmax(gm);
            const double mu = sz * inv_m;
            STAMP_END(3);
            if (!isfinite(nrx) || !isfinite(nrz) || !isfinite(sz)) { flag = 3; break; }
            // NLP: dual residual scaled by max(1, ||Q x + f||_inf) (QP: iSWIFT's absolute test)
            const double thx = nl ? th * gm : th;
            if (nrx < thx && nrz < th && sz * inv_m < tol) { flag = 0; break; }
            const bool pc = nl || (sigma > sigma_d);
            double delta = 0.0;
            if (pc) {
                // ---- weights W^-1 = z/s (updatekktmatrix, Auxilary.c:197-205), Lagrangian
                //      Hessian -2 sum_j z_kj on (x_k, y_k) (NLP), assembly and factorisation
#pragma unroll
                for (int t = 0; t < TV; t++)
                    if (t < nchunk_v) {
                        const int v = lane + 64 * t;
                        double hs = 0.0;
                        if (nl && pos[t]) {
                            const int k = v >> 2;
                            for (int j = 0; j < K; j++) hs += zo[k * K + j];
                            hs *= -2.0;
                        }
                        const double wa = aon[t] ? A[t].z[0] * A[t].is[0] + A[t].z[1] * A[t].is[1] : 0.0;
                        const double wb = (nl && vel[t]) ? B[t].z[0] * B[t].is[0] + B[t].z[1] * B[t].is[1] : 0.0;
                        if (v < n4) W[v] = vok[t] ? Pv[t] + hs + wa + wb : 0.0;
                    }
                if (lane < E4) W[n4 + lane] = e_on ? E.z[0] * E.is[0] + E.z[1] * E.is[1] : 0.0;
#pragma unroll
                for (int t = 0; t < TO; t++) {
                    const int o = lane + 64 * t;
                    if (nl && t < nchunk_o && o < NK4) W[n4 + E4 + o] = ook[t] ? O[t].z[0] * O[t].is[0] : 0.0;
                }
                SYNC();
                gram<NZM>(R, W, cnt, H0, lane);
                SYNC();
                STAMP_END(4);
                double dstart = 0.0;
                int ok = 0;
                for (int tries = 0; tries < (nl ? 14 : 1); tries++) {
                    if (tries == 0) {       // scale-aware first shift: 1e-10 * max(1, max diag of Z'HZ)
                        double dm = (lane < nz) ? H0[lane * LDH + lane] : 1.0;
                        dstart = 1e-10 * fmax(1.0, wmax(dm));
                    }
                    gj_load<NZL>(Mi, H0, ZZ, delta, nz, lane);
                    if (delta != 0.0) {
                        if (lane < nz)
#pragma unroll
                            for (int j = 0; j < NZL; j++) HS[lane * LDH + j] = Mi[j];
                        SYNC();
                    }
                    const int cf = gj_invert<NZL>(Mi, nz, lane, !nl);
                    if (cf == 0) { ok = 1; break; }
                    delta = (delta == 0.0) ? dstart : delta * 10.0;
                }
                STAMP_END(5);
                if (!ok) { flag = 1; break; }
            }
            const double *Hsv = (delta != 0.0) ? HS : H0;

            // ---- predictor (pc) or centring step (Prime.c:193-196), then corrector
            double ap = 1.0, ad = 1.0;
#pragma clang loop unroll(disable)
            for (int pass = (pc ? 0 : 1); pass < 2; pass++) {
                // right-hand side: dsT, r3 = rz - dsT / z, w = om r3, coef = rx + J'w
                const double smu = (pass == 0) ? 0.0 : (pc ? sigma * mu : sigma_d * mu);
#pragma unroll
                for (int t = 0; t < TV; t++)
                    if (t < nchunk_v) {
                        const int v = lane + 64 * t;
                        double cf = rx[t];
#pragma unroll
                        for (int r = 0; r < 2; r++) {
                            const double sg = r ? -1.0 : 1.0;
                            {
                                Pair &q = A[t];
                                double dsT = -q.s[r] * q.z[r];
                                if (pass == 1 && pc) dsT -= q.ds[r] * q.dz[r];
                                dsT += smu;
                                q.dsT[r] = dsT;
                                q.r3[r] = fma(-dsT, q.iz[r], rz_of(q, r, xv[t], r ? hAm[t] : hAp[t]));
                                if (aon[t]) cf = fma(sg, q.z[r] * q.is[r] * q.r3[r], cf);
                            }
                            {
                                Pair &q = B[t];
                                double dsT = -q.s[r] * q.z[r];
                                if (pass == 1 && pc) dsT -= q.ds[r] * q.dz[r];
                                dsT += smu;
                                q.dsT[r] = dsT;
                                q.r3[r] = fma(-dsT, q.iz[r], rz_of(q, r, xv[t], prm.vsat));
                                if (nl && vel[t]) cf = fma(sg, q.z[r] * q.is[r] * q.r3[r], cf);
                            }
                        }
                        if (v < n4) CF[v] = vok[t] ? cf : 0.0;
                    }
                {
                    double cf = 0.0;
#pragma unroll
                    for (int r = 0; r < 2; r++) {
                        double dsT = -E.s[r] * E.z[r];
                        if (pass == 1 && pc) dsT -= E.ds[r] * E.dz[r];
                        dsT += smu;
                        E.dsT[r] = dsT;
                        E.r3[r] = fma(-dsT, E.iz[r], rz_of(E, r, ge, fr));
                        cf = fma(r ? -1.0 : 1.0, E.z[r] * E.is[r] * E.r3[r], cf);
                    }
                    if (lane < E4) CF[n4 + lane] = e_on ? cf : 0.0;
                }
#pragma unroll
                for (int t = 0; t < TO; t++)
                    if (nl && t < nchunk_o) {
                        Pair &q = O[t];
                        double dsT = -q.s[0] * q.z[0];
                        if (pass == 1 && pc) dsT -= q.ds[0] * q.dz[0];
                        dsT += smu;
                        q.dsT[0] = dsT;
                        q.r3[0] = fma(-dsT, q.iz[0], rz_of(q, 0, go[t], oh[t]));
                        const int o = lane + 64 * t;
                        if (o < NK4) CF[n4 + E4 + o] = ook[t] ? q.z[0] * q.is[0] * q.r3[0] : 0.0;
                    }
                SYNC();
                STAMP_END(6 + 4 * pass);
                rmul<NZM>(R, CF, cnt, vg, nz, lane);
                SYNC();
                STAMP_END(7 + 4 * pass);
                la_solve<NZL>(Mi, Hsv, vg, vy, vr, vd, dxi, nz, lane);
                STAMP_END(8 + 4 * pass);
                // J dx per slot; dz = om (J dx - r3); ds = (dsT - s dz) / z; step-length maxima
                double mxs = 0.0, mxz = 0.0;
                double dxv[TV];
#pragma unroll
                for (int t = 0; t < TV; t++) {
                    dxv[t] = 0.0;
                    if (t < nchunk_v) {
                        const int v = lane + 64 * t;
                        dxv[t] = vok[t] ? row_dot<NZL>(R + (v < n4 ? v : 0) * LDR, dxi) : 0.0;
#pragma unroll
                        for (int r = 0; r < 2; r++) {
                            const double sg = r ? -1.0 : 1.0;
                            {
                                Pair &q = A[t];
                                q.dz[r] = aon[t] ? q.z[r] * q.is[r] * fma(sg, dxv[t], -q.r3[r]) : 0.0;
                                q.ds[r] = aon[t] ? fma(-q.s[r], q.dz[r], q.dsT[r]) * q.iz[r] : 0.0;
                                mxs = fmax(mxs, -q.ds[r] * q.is[r]); mxz = fmax(mxz, -q.dz[r] * q.iz[r]);
                            }
                            {
                                Pair &q = B[t];
                                const bool bon = nl && vel[t];
                                q.dz[r] = bon ? q.z[r] * q.is[r] * fma(sg, dxv[t], -q.r3[r]) : 0.0;
                                q.ds[r] = bon ? fma(-q.s[r], q.dz[r], q.dsT[r]) * q.iz[r] : 0.0;
                                mxs = fmax(mxs, -q.ds[r] * q.is[r]); mxz = fmax(mxz, -q.dz[r] * q.iz[r]);
                            }
                        }
                    }
                }
                {
                    const double jd = e_on ? row_dot<NZL>(Rt + (e_on ? lane : 0) * LDR, dxi) : 0.0;
#pragma unroll
                    for (int r = 0; r < 2; r++) {
                        const double sg = r ? -1.0 : 1.0;
                        E.dz[r] = e_on ? E.z[r] * E.is[r] * fma(sg, jd, -E.r3[r]) : 0.0;
                        E.ds[r] = e_on ? fma(-E.s[r], E.dz[r], E.dsT[r]) * E.iz[r] : 0.0;
                        mxs = fmax(mxs, -E.ds[r] * E.is[r]); mxz = fmax(mxz, -E.dz[r] * E.iz[r]);
                    }
                }
#pragma unroll
                for (int t = 0; t < TO; t++)
                    if (nl && t < nchunk_o) {
                        const int o = lane + 64 * t;
                        const double jd = ook[t] ? row_dot<NZL>(Ro + (o < NK4 ? o : 0) * LDR, dxi) : 0.0;
                        Pair &q = O[t];
                        q.dz[0] = ook[t] ? q.z[0] * q.is[0] * (jd - q.r3[0]) : 0.0;
                        q.ds[0] = ook[t] ? fma(-q.s[0], q.dz[0], q.dsT[0]) * q.iz[0] : 0.0;
                        mxs = fmax(mxs, -q.ds[0] * q.is[0]); mxz = fmax(mxz, -q.dz[0] * q.iz[0]);
                    }
                // findsteplength (Auxilary.c:271-294): 1 / max(-dv / v), 1 when no dv < 0
                mxs = wmax(mxs); mxz = wmax(mxz);
                ap = (mxs > 0.0) ? 1.0 / mxs : 1.0;
                ad = (mxz > 0.0) ? 1.0 / mxz : 1.0;
                STAMP_END(9 + 4 * pass);
                if (pass == 0) {
                    // rho = (s + ap ds)'(z + ad dz) / s'z ; sigma = min(1, rho)^3  (formrho, Prime.c:160-170)
                    double num = 0.0;
#pragma unroll
                    for (int t = 0; t < TV; t++)
                        if (t < nchunk_v)
#pragma unroll
                            for (int r = 0; r < 2; r++) {
                                const Pair &a = A[t], &b = B[t];
                                num += aon[t] ? fma(ap, a.ds[r], a.s[r]) * fma(ad, a.dz[r], a.z[r]) : 0.0;
                                num += (nl && vel[t]) ? fma(ap, b.ds[r], b.s[r]) * fma(ad, b.dz[r], b.z[r]) : 0.0;
                            }
#pragma unroll
                    for (int r = 0; r < 2; r++) num += e_on ? fma(ap, E.ds[r], E.s[r]) * fma(ad, E.dz[r], E.z[r]) : 0.0;
#pragma unroll
                    for (int t = 0; t < TO; t++)
                        if (nl && t < nchunk_o) num += ook[t] ? fma(ap, O[t].ds[0], O[t].s[0]) * fma(ad, O[t].dz[0], O[t].z[0]) : 0.0;
                    num = wsum(num);
                    const double rho = num / sz, mr = rho < 1.0 ? rho : 1.0;
                    sigma = mr * mr * mr; if (sigma < sigma_d) sigma = sigma_d;
                    continue;
                }
                // ---- update (Prime.c:208-216): step 0.99 alpha capped at 1
                ap = (0.99 * ap < 1.0) ? 0.99 * ap : 1.0;
                ad = (0.99 * ad < 1.0) ? 0.99 * ad : 1.0;
                // new per-grid obstacle dual sums for the Jacobian-change term of rx
#pragma unroll
                for (int t = 0; t < TO; t++)
                    if (nl && t < nchunk_o) {
                        const int o = lane + 64 * t;
                        O[t].s[0] = fma(ap, O[t].ds[0], O[t].s[0]);
                        O[t].z[0] = fma(ad, O[t].dz[0], O[t].z[0]);
                    }
                // (the hess term uses the old duals still in zo)
#pragma unroll
                for (int t = 0; t < TV; t++)
                    if (t < nchunk_v) {
                        const int v = lane + 64 * t;
                        double hs_old = 0.0;
                        if (nl && pos[t]) {
                            const int k = v >> 2;
                            for (int j = 0; j < K; j++) hs_old += zo[k * K + j];
                        }
                        rx[t] = (1.0 - ad) * rx[t] + ((ad - ap) * Pv[t]) * dxv[t];
                        if (nl) rx[t] = fma(ad * (delta - 2.0 * hs_old), dxv[t], rx[t]);
                        xv[t] = fma(ap, dxv[t], xv[t]);
#pragma unroll
                        for (int r = 0; r < 2; r++) {
                            A[t].s[r] = fma(ap, A[t].ds[r], A[t].s[r]); A[t].z[r] = fma(ad, A[t].dz[r], A[t].z[r]);
                            B[t].s[r] = fma(ap, B[t].ds[r], B[t].s[r]); B[t].z[r] = fma(ad, B[t].dz[r], B[t].z[r]);
                        }
                    }
#pragma unroll
                for (int r = 0; r < 2; r++) {
                    E.s[r] = fma(ap, E.ds[r], E.s[r]); E.z[r] = fma(ad, E.dz[r], E.z[r]);
                }
                SYNC();          // every lane has read the old duals
#pragma unroll
                for (int t = 0; t < TO; t++)
                    if (nl && t < nchunk_o) {
                        const int o = lane + 64 * t;
                        if (o < NK4) zo[o] = ook[t] ? O[t].z[0] : 0.0;
                    }
                SYNC();
#pragma unroll
                for (int t = 0; t < TV; t++)
                    if (t < nchunk_v) {
                        const int v = lane + 64 * t;
                        if (nl && pos[t]) {      // -(J(x') - J(x))' z' on (x_k, y_k): +2 ap dx sum_j z'_kj
                            const int k = v >> 2;
                            double hs_new = 0.0;
                            for (int j = 0; j < K; j++) hs_new += zo[k * K + j];
                            rx[t] = fma(2.0 * ap * hs_new, dxv[t], rx[t]);
                        }
                        if (vok[t]) xs[v] = xv[t];
                    }
                SYNC();
                STAMP_END(14);
            }
            it++;
        }
        if (stage == 0) { qp_flag = flag; qp_it = it; } else { nlp_flag = flag; nlp_it = it; }
    }
    if (x_qp_out && nstage == 1)
#pragma unroll
        for (int t = 0; t < TV; t++) if (t < nchunk_v && vok[t]) x_qp_out[(size_t)agent * n + lane + 64 * t] = xv[t];

    // ---- outputs
    double f = 0.0;
#pragma unroll
    for (int t = 0; t < TV; t++)
        if (t < nchunk_v && vok[t]) {
            x_out[(size_t)agent * n + lane + 64 * t] = xv[t];
            f += fma(0.5 * Pv[t] * xv[t], xv[t], cv[t] * xv[t]);
        }
    f = wsum(f);
    STAMP_END(15);
    STAMP_FLUSH(agent);
    if (lane == 0) {
        obj_out[agent] = f;
        status_out[2 * agent] = qp_flag; status_out[2 * agent + 1] = nlp_flag;
        iters_out[2 * agent] = qp_it; iters_out[2 * agent + 1] = nlp_it;
    }
}

#define SRB_NMPC_KERNEL(NZL, TV, TO)                                                                           \
    extern "C" __global__ void __launch_bounds__(WAVE) srb_nmpc_kernel_##NZL##_##TV##_##TO(                   \
        SrbKParams prm, int n_agents, const double *__restrict__ x0g, const double *__restrict__ refg,          \
        const double *__restrict__ footg, const double *__restrict__ obstacles, int n_obs,                       \
        const double *__restrict__ nbr_state, int n_all, int agent_offset, double *__restrict__ x_qp_out,        \
        double *__restrict__ x_out, double *__restrict__ obj_out, int *__restrict__ status_out,                 \
        int *__restrict__ iters_out)                                                                           \
    {                                                                                                          \
        extern __shared__ __attribute__((aligned(16))) double lds[];                                           \
        const int agent = blockIdx.x;                                                                          \
        if (agent >= n_agents) return;                                                                         \
        nmpc_agent<NZL, TV, TO>(prm, agent, x0g, refg, footg, obstacles, n_obs, nbr_state, n_all, agent_offset, \
                                x_qp_out, x_out, obj_out, status_out, iters_out, lds);                         \
    }

SRB_KERNEL_INSTANCES(SRB_NMPC_KERNEL)
