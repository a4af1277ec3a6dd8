// Batched CBF-NMPC solver kernels for MI355X (gfx950).
//
// Replaces the per-control-cycle solve of MPC_dist::run_NMPC
// (/root/reference/src/MPC_dist.cpp:81-454): the LIP/CoP/contact-weight QP of
// :135-321 solved with the iSWIFT Mehrotra predictor-corrector
// (/root/reference/optimization/iSWIFT/src/Prime.c:127-230), then the NLP stage with
// the obstacle ("CBF") and velocity rows of include/dec_vars_constr_cost.h:245-395
// (SNOPT in the reference) solved by a primal-dual interior-point method warm-started
// from the QP solution (MPC_dist.cpp:403).
//
// Layout / execution model
//   * one 64-lane wavefront (= one workgroup) per agent; the whole solve -- problem
//     assembly, both interior-point loops, output -- runs inside that wave with all
//     per-agent vectors in LDS, so there is no host round trip per iteration;
//   * equality constraints (LIP dynamics, u_k = F_k lambda_k, sum lambda_k = 1) are
//     eliminated by a null-space basis Z built from a forward rollout:
//         x = xbar + Z xi,  xi = (lambda dofs of every grid, s),  nz = N(C-1)+1,
//     so each Newton step is an nz x nz Cholesky (11 x 11 at N=10 trot) instead of
//     the (nv+neq+m)-dimensional sparse LDL' of iSWIFT.  Iterates equal iSWIFT's in
//     exact arithmetic: x, s, z are advanced exactly as Prime.c:208-216 and the
//     equality multipliers are carried as q = A'y (q += alpha_d * A'dy), which is all
//     the residual rx = -Px - A'y - G'z - c of computeresiduals needs;
//   * the solve is latency-bound (one wave per agent, a few thousand flops per
//     iteration), so the dense factor and both triangular solves live in registers,
//     one row of the nz x nz system per lane, with cross-lane values moved by
//     v_readlane (NZM = compile-time bound on nz: 16 or 32); Z'HZ is assembled from
//     its structurally nonzero terms only; per-row reciprocals are formed once per
//     iteration;
//   * inputs/outputs are agent-major fp64 arrays in HBM, read once / written once.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "srb_kernel_params.h"

#define WAVE 64

// --------------------------------------------------------------------------- wave helpers
// Cross-lane traffic stays in the VALU: DPP row permutations for the 16-lane rows and
// gfx950's v_permlane16/32_swap across rows (no LDS round trips, unlike __shfl_xor, which
// lowers to ds_bpermute).  Every lane ends with the bit-identical result (each stage
// combines a pair with a commutative op), so branches on it stay wave-uniform.
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
// value of lane `lane` (wave-uniform index, SGPR) -> wave-uniform value
__device__ __forceinline__ double readlane_d(double v, int lane)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, lane);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// 1/x and 1/sqrt(x) from the hardware estimates (v_rcp_f64 / v_rsq_f64) refined by two
// Newton steps: within an ulp or two of the IEEE results, a handful of FMAs instead of
// the ~12-instruction division / square-root sequences.
__device__ __forceinline__ double rcp_d(double x)
{
    double r = __builtin_amdgcn_rcp(x);
    r = fma(r, fma(-x, r, 1.0), r);
    r = fma(r, fma(-x, r, 1.0), r);
    return r;
}
__device__ __forceinline__ double rsq_d(double x)
{
    double r = __builtin_amdgcn_rsq(x);
    r = fma(0.5 * r, fma(-x * r, r, 1.0), r);
    r = fma(0.5 * r, fma(-x * r, r, 1.0), r);
    return r;
}

// --------------------------------------------------------------------------- diagnostic stamps
// Built only with -DSRB_STAMPS (make stamps -> srbnmpc/libsrbnmpc_stamps.so): lane 0 of
// every agent accumulates s_memtime cycles per phase into LDS (fire-and-forget
// ds_add_u64); agent 0 adds them to a device buffer nothing else reads at the end.
#ifdef SRB_STAMPS
#define SRB_NSTAMP 64
__device__ unsigned long long srb_stamp_buf[SRB_NSTAMP];
#define STAMP_BEGIN(c) do { __builtin_amdgcn_sched_barrier(0); (c).st_t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); } while (0)
#define STAMP_END(c, slot) do { __builtin_amdgcn_sched_barrier(0); const unsigned long long _t = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0); if ((c).tid == 0) atomicAdd(&(c).stamps[slot], _t - (c).st_t0); (c).st_t0 = _t; } while (0)
#else
#define STAMP_BEGIN(c) do {} while (0)
#define STAMP_END(c, slot) do {} while (0)
#endif

// --------------------------------------------------------------------------- per-agent context
struct Ctx {
    const SrbKParams *P;
    int N, C, K, n, nz, mq, m, nl;          // nl: NLP rows/terms active
    int ldz, n16;                            // Z: n16 rows (zero beyond n) x ldz columns (zero beyond nz)
    int rFm, rXp, rXm, rUp, rUm, rLlo, rLhi, rO, rV;
    // LDS arrays
    double *Z, *x, *q, *rx, *dx, *tv, *D, *ref, *foot;
    double *s, *z, *rz, *dz, *dsv, *dsT, *om, *iz, *is, *l2, *jc, *obs, *eps;
    double *Hc, *L, *ZtZ, *ZtZL, *hvec, *xiv, *gbuf;   // L, ZtZL: inverses of Hc, ZtZ
    double *bc;                             // 4 x 64 broadcast scratch (gj_inverse)
    int2 *term;                             // Z'HZ term table: (u*nz, w*nz) per term (see build_Hc)
    int tid;
#ifdef SRB_STAMPS
    unsigned long long *stamps;
    mutable unsigned long long st_t0;
#endif
};

__device__ __forceinline__ int col_stage(const Ctx &c, int a) { return (a == c.nz - 1) ? c.N : a / (c.C - 1); }

// h of row r
__device__ __forceinline__ double row_h(const Ctx &c, int r)
{
    if (r < c.rXp) return c.P->fr;
    if (r < c.rLlo) return c.P->box;
    if (r < c.rLhi) return 0.0;
    if (r < c.mq) return 1.0;
    if (r < c.rV) return -c.eps[(r - c.rO) % c.K];
    return c.P->vsat;
}

// J_r . v  (for obstacle rows this is the Jacobian row at the point the coefficients were taken)
__device__ __forceinline__ double row_dot(const Ctx &c, int r, const double *v)
{
    const int N = c.N;
    if (r < c.rFm) { int i = r >> 1, d = r & 1; return v[4 * i + 2 * d] - v[4 * N + 2 * (i + 1) + d]; }
    if (r < c.rXp) { int rr = r - c.rFm, i = rr >> 1, d = rr & 1; return -v[4 * i + 2 * d] + v[4 * N + 2 * (i + 1) + d]; }
    if (r < c.rXm) return v[r - c.rXp];
    if (r < c.rUp) return -v[r - c.rXm];
    if (r < c.rUm) return v[4 * N + (r - c.rUp)];
    if (r < c.rLlo) return -v[4 * N + (r - c.rUm)];
    if (r < c.rLhi) return -v[6 * N + (r - c.rLlo)];
    if (r < c.mq) return v[6 * N + (r - c.rLhi)];
    if (r < c.rV) {
        int o = r - c.rO, k = o / c.K;
        return c.jc[2 * o] * v[4 * k] + c.jc[2 * o + 1] * v[4 * k + 2] - v[c.n - 1];
    }
    int rr = r - c.rV; double sg = (rr < 2 * N) ? 1.0 : -1.0;
    int t = rr % (2 * N), comp = (t < N) ? 1 : 3, k = t % N;
    return sg * v[4 * k + comp];
}

// (J' w)_v for every variable but s (s handled by a wave reduction)
__device__ __forceinline__ double jt_gather(const Ctx &c, int v, const double *w)
{
    const int N = c.N;
    double acc;
    if (v < 4 * N) {
        int k = v >> 2, cc = v & 3;
        acc = w[c.rXp + v] - w[c.rXm + v];
        if (!(cc & 1)) {
            int d = cc >> 1;
            if (k <= N - 2) acc += w[2 * k + d] - w[c.rFm + 2 * k + d];
            if (c.nl)
                for (int j = 0; j < c.K; j++) acc += c.jc[2 * (k * c.K + j) + d] * w[c.rO + k * c.K + j];
        } else if (c.nl) {
            int t = ((cc == 1) ? 0 : N) + k;
            acc += w[c.rV + t] - w[c.rV + 2 * N + t];
        }
    } else if (v < 6 * N) {
        int j = v - 4 * N, k = j >> 1, d = j & 1;
        acc = w[c.rUp + j] - w[c.rUm + j];
        if (k >= 1) acc += -w[2 * (k - 1) + d] + w[c.rFm + 2 * (k - 1) + d];
    } else {
        int j = v - 6 * N;
        acc = -w[c.rLlo + j] + w[c.rLhi + j];
    }
    return acc;
}

// out[v] = base[v] + sign*(J' w)[v] for all v (s row by reduction).  Collective.
__device__ __forceinline__ void jt_apply(const Ctx &c, const double *w, double *out, const double *base, double sign)
{
    for (int v = c.tid; v < c.n - 1; v += WAVE) out[v] = (base ? base[v] : 0.0) + sign * jt_gather(c, v, w);
    double ps = 0.0;
    if (c.nl)
        for (int o = c.tid; o < c.N * c.K; o += WAVE) ps -= w[c.rO + o];
    ps = wsum(ps);
    if (c.tid == 0) out[c.n - 1] = (base ? base[c.n - 1] : 0.0) + sign * ps;
    __syncthreads();
}

__device__ __forceinline__ double Pdiag(const Ctx &c, int v)
{
    const int N = c.N;
    if (v < 4 * N) return (v >= 4 * (N - 1)) ? c.P->Pw : c.P->Qw;
    if (v < 6 * N) return c.P->Rw;
    if (v < c.n - 1) return 0.0;
    return c.P->Sw;
}
__device__ __forceinline__ double cvec(const Ctx &c, int v) { return (v < 4 * c.N) ? -Pdiag(c, v) * c.ref[v] : 0.0; }

// Lagrangian-Hessian diagonal beyond P (NLP: -2 sum_j z_kj on x_k, y_k)
__device__ __forceinline__ double hess_diag(const Ctx &c, int v)
{
    if (!c.nl || v >= 4 * c.N || (v & 1)) return 0.0;
    int k = v >> 2;
    double zs = 0.0;
    for (int j = 0; j < c.K; j++) zs += c.z[c.rO + k * c.K + j];
    return -2.0 * zs;
}

// obstacle Jacobian coefficients at the current x: jc = -2 (p_k - o_kj)
__device__ __forceinline__ void obstacle_coefs(const Ctx &c)
{
    for (int o = c.tid; o < c.N * c.K; o += WAVE) {
        int k = o / c.K;
        c.jc[2 * o] = -2.0 * (c.x[4 * k] - c.obs[2 * o]);
        c.jc[2 * o + 1] = -2.0 * (c.x[4 * k + 2] - c.obs[2 * o + 1]);
    }
    __syncthreads();
}

// g_r(x) of row r (nonlinear for obstacle rows)
__device__ __forceinline__ double row_val(const Ctx &c, int r)
{
    if (r >= c.rO && r < c.rV) {
        int o = r - c.rO, k = o / c.K;
        double dx = c.x[4 * k] - c.obs[2 * o], dy = c.x[4 * k + 2] - c.obs[2 * o + 1];
        return -(dx * dx + dy * dy) - c.x[c.n - 1];
    }
    return row_dot(c, r, c.x);
}

// --------------------------------------------------------------------------- Z'HZ assembly
// Values of the Z'HZ terms (term_table order): D[0..n) = diag of H, then both orientations
// of the friction couplings and (NLP) the per-grid obstacle couplings (xy, xs, ys).
// H = P + hess + delta I + J' diag(om) J.
__device__ __forceinline__ void build_D(const Ctx &c, double delta)
{
    const int N = c.N, n = c.n;
    for (int v = c.tid; v < n - 1; v += WAVE) {
        double d = Pdiag(c, v) + delta + hess_diag(c, v);
        if (v < 4 * N) {
            int k = v >> 2, cc = v & 3;
            d += c.om[c.rXp + v] + c.om[c.rXm + v];
            if (!(cc & 1)) {
                int dd = cc >> 1;
                if (k <= N - 2) d += c.om[2 * k + dd] + c.om[c.rFm + 2 * k + dd];
                if (c.nl)
                    for (int j = 0; j < c.K; j++) { double jj = c.jc[2 * (k * c.K + j) + dd]; d += c.om[c.rO + k * c.K + j] * jj * jj; }
            } else if (c.nl) {
                int t = ((cc == 1) ? 0 : N) + k;
                d += c.om[c.rV + t] + c.om[c.rV + 2 * N + t];
            }
        } else if (v < 6 * N) {
            int j = v - 4 * N, k = j >> 1, dd = j & 1;
            d += c.om[c.rUp + j] + c.om[c.rUm + j];
            if (k >= 1) d += c.om[2 * (k - 1) + dd] + c.om[c.rFm + 2 * (k - 1) + dd];
        } else {
            int j = v - 6 * N;
            d += c.om[c.rLlo + j] + c.om[c.rLhi + j];
        }
        c.D[v] = d;
    }
    double ps = 0.0;
    if (c.nl)
        for (int o = c.tid; o < N * c.K; o += WAVE) ps += c.om[c.rO + o];
    ps = wsum(ps);
    if (c.tid == 0) c.D[n - 1] = Pdiag(c, n - 1) + delta + ps;
    // off-diagonal terms: both orientations of each coupling (see term_table)
    double *hc = c.D + c.n16;
    const int nf = 2 * (N - 1);
    for (int e = c.tid; e < nf; e += WAVE) { const double v = -(c.om[e] + c.om[c.rFm + e]); hc[2 * e] = v; hc[2 * e + 1] = v; }
    if (c.nl)
        for (int k = c.tid; k < N; k += WAVE) {
            double xy = 0, xs = 0, ys = 0;
            for (int j = 0; j < c.K; j++) {
                int o = k * c.K + j;
                double w = c.om[c.rO + o], jx = c.jc[2 * o], jy = c.jc[2 * o + 1];
                xy += w * jx * jy; xs -= w * jx; ys -= w * jy;
            }
            double *t = hc + 2 * (nf + 3 * k);
            t[0] = xy; t[1] = xy; t[2] = xs; t[3] = xs; t[4] = ys; t[5] = ys;
        }
    __syncthreads();
}

// Z'HZ as a sum of rank-1 terms  sum_t h_t Z[u_t,:]' Z[w_t,:]  over the nonzeros of H:
//   diagonal terms       (u, w) = (v, v),  h = D[v]            (v < n16; Z rows >= n are 0)
//   coupling terms       each coupling (u, w) of H twice, (u, w) and (w, u), h = H_uw:
//                          friction row e = 2i+d: X_i pos d  <->  U_{i+1} d
//                          (NLP) grid k: x_k <-> y_k, x_k <-> s, y_k <-> s
// The coupling table holds the Z row offsets (u*ldz, w*ldz), padded to a multiple of 16
// with (0, 0); h lives in D[n16 + e] (build_D; padding stays 0).  Built once.
__device__ __forceinline__ void term_table(const Ctx &c)
{
    const int N = c.N, n = c.n, ldz = c.ldz, nf = 2 * (N - 1);
    const int ncpl2 = SRB_NCPL2(N), cpl16 = SRB_R16(ncpl2);
    for (int t = c.tid; t < cpl16; t += WAVE) {
        int u = 0, w = 0;
        if (t < ncpl2) {
            const int e = t >> 1;
            if (e < nf) { const int i = e >> 1, d = e & 1; u = 4 * i + 2 * d; w = 4 * N + 2 * (i + 1) + d; }
            else {
                const int o = e - nf, k = o / 3, r = o - 3 * k;
                u = (r == 2) ? 4 * k + 2 : 4 * k;
                w = (r == 0) ? 4 * k + 2 : n - 1;
            }
            if (t & 1) { const int tmp = u; u = w; w = tmp; }
        }
        c.term[t] = make_int2(u * ldz, w * ldz);
    }
    __syncthreads();
}

typedef double srb_d4 __attribute__((ext_vector_type(4)));

// out = Z' H Z (nz x nz, row-major in LDS) on the matrix cores: v_mfma_f64_16x16x4_f64
// with A[a][t] = h_t Z[u_t][a], B[t][b] = Z[w_t][b], four terms per instruction
// (lane l supplies term t0 + (l >> 4), column l & 15).  Z and the term lists are
// zero-padded (rows to n16, columns to ldz, couplings to a multiple of 16), so the loops
// are branch-free with unconditional LDS loads; two accumulator chains per tile keep
// consecutive MFMAs independent.  16x16 output tiles, upper triangle of tiles computed
// and mirrored.  unit != 0: H = I (gives Z'Z).
template <int NZM>
__device__ __forceinline__ void build_Hc(const Ctx &c, double *out, int unit)
{
    constexpr int T = NZM / 16;
    const int nz = c.nz, ldz = c.ldz, n16 = c.n16, li = c.tid & 15, kq = c.tid >> 4;
    const int cpl16 = unit ? 0 : SRB_R16(2 * (2 * (c.N - 1) + (c.nl ? 3 * c.N : 0)));
    const int Tn = ldz >> 4;
    const double *Z = c.Z, *D = c.D, *Dc = c.D + n16;
#pragma unroll
    for (int ta = 0; ta < T; ta++) {
        if (ta >= Tn) break;
        srb_d4 acc0[T], acc1[T];
#pragma unroll
        for (int tb = 0; tb < T; tb++) { acc0[tb] = srb_d4{0.0, 0.0, 0.0, 0.0}; acc1[tb] = acc0[tb]; }
        const int ca = 16 * ta + li;
        for (int t0 = 0; t0 < n16; t0 += 16) {                // diagonal terms, 16 per trip
            double a[4]; int r[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int v = t0 + 4 * u + kq;
                r[u] = v * ldz;
                a[u] = (unit ? 1.0 : D[v]) * Z[r[u] + ca];
            }
#pragma unroll
            for (int tb = 0; tb < T; tb++)
                if (tb >= ta && tb < Tn) {
                    const int cb = 16 * tb + li;
                    acc0[tb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[0], Z[r[0] + cb], acc0[tb], 0, 0, 0);
                    acc1[tb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[1], Z[r[1] + cb], acc1[tb], 0, 0, 0);
                    acc0[tb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[2], Z[r[2] + cb], acc0[tb], 0, 0, 0);
                    acc1[tb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[3], Z[r[3] + cb], acc1[tb], 0, 0, 0);
                }
        }
        for (int e0 = 0; e0 < cpl16; e0 += 16) {              // coupling terms, 16 per trip
            double a[4]; int2 uw[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                uw[u] = c.term[e0 + 4 * u + kq];
                a[u] = Dc[e0 + 4 * u + kq] * Z[uw[u].x + ca];
            }
#pragma unroll
            for (int tb = 0; tb < T; tb++)
                if (tb >= ta && tb < Tn) {
                    const int cb = 16 * tb + li;
                    acc0[tb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[0], Z[uw[0].y + cb], acc0[tb], 0, 0, 0);
                    acc1[tb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[1], Z[uw[1].y + cb], acc1[tb], 0, 0, 0);
                    acc0[tb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[2], Z[uw[2].y + cb], acc0[tb], 0, 0, 0);
                    acc1[tb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[3], Z[uw[3].y + cb], acc1[tb], 0, 0, 0);
                }
        }
        // D layout of v_mfma_f64_16x16x4: col = lane & 15, row = (lane >> 4) + 4 * reg
#pragma unroll
        for (int tb = 0; tb < T; tb++)
            if (tb >= ta && tb < Tn) {
                const int col = 16 * tb + li;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int row = 16 * ta + kq + 4 * r;
                    const double v = acc0[tb][r] + acc1[tb][r];
                    if (row < nz && col < nz) { out[row * nz + col] = v; out[col * nz + row] = v; }
                }
            }
    }
    __syncthreads();
}

// --------------------------------------------------------------------------- Gauss-Jordan inverse
// The reduced Newton matrix (nz x nz SPD) is inverted in place by Gauss-Jordan without
// pivoting; each Newton solve is then one matvec.  Layout: G = 64/NZM lanes per row,
// lane = G*i + g holds A[i][CW*g .. CW*g+CW-1] (CW = NZM/G: 4 entries at NZM = 16), so a
// step costs each lane CW FMAs.  Step k: the pivot comes from its lane by v_readlane;
// lanes of row k publish the scaled row, lanes of column k the multipliers, through a
// double-buffered LDS broadcast; every lane updates its entries.  The pivots are those
// of L D L' in natural order, so pivot <= 0 <=> not positive definite, and regularise
// != 0 applies iSWIFT's dynamic pivot regularisation to them (ldl.c:320-321:
// |D_kk| <= 1e-14 -> 1e-7) for the QP stage.  Padding rows/columns (>= nz) are the
// identity, so the steps of the last 4-step chunk beyond nz are no-ops.  Steps run in
// straight-line chunks of 4 (one uniform branch per chunk).  Minv (row-major, stride
// nz) may alias H.  Returns 0 on success (wave-uniform).
template <int NZM>
__device__ __forceinline__ int gj_inverse(const Ctx &c, const double *H, double *Minv, int nz, int regularise)
{
    constexpr int G = WAVE / NZM, CW = NZM / G;
    const int i = c.tid / G, g = c.tid % G;
    double A[CW];
#pragma unroll
    for (int q = 0; q < CW; q++) {
        const int j = CW * g + q;
        A[q] = (i < nz && j < nz) ? H[i * nz + j] : (i == j ? 1.0 : 0.0);
    }
    __syncthreads();
    int fail = 0;
#pragma unroll
    for (int k0 = 0; k0 < NZM; k0 += 4) {
        if (k0 >= nz) continue;
#pragma unroll
        for (int k = k0; k < k0 + 4; k++) {
            const int gk = k / CW, qk = k % CW;
            double piv = readlane_d(A[qk], G * k + gk);
            if (regularise && piv <= 1e-14 && piv == piv) piv = 1e-7;
            fail |= !(piv > 0.0);
            const double inv = rcp_d(piv);
            double *rb = c.bc + 2 * WAVE * (k & 1), *cb = rb + WAVE;
            if (i == k) {
#pragma unroll
                for (int q = 0; q < CW; q++) rb[CW * g + q] = (q == qk && g == gk) ? inv : A[q] * inv;
            }
            if (g == gk) cb[i] = A[qk];
            __builtin_amdgcn_wave_barrier();
            const double f = cb[i];
            if (g == gk) A[qk] = 0.0;                       // column k becomes -f * inv
#pragma unroll
            for (int q = 0; q < CW; q++) {
                const double r = rb[CW * g + q];
                A[q] = (i == k) ? r : fma(-f, r, A[q]);
            }
        }
    }
    if (i < nz) {
#pragma unroll
        for (int q = 0; q < CW; q++)
            if (CW * g + q < nz) Minv[i * nz + CW * g + q] = A[q];
    }
    __syncthreads();
    return fail;
}

// y = M x for an nz x nz row-major LDS matrix and an LDS vector: lane (i, g) sums its CW
// columns, the G lanes of row i (adjacent) combine by DPP; every lane of row i holds y_i.
template <int NZM>
__device__ __forceinline__ double gj_matvec(const Ctx &c, const double *M, const double *x)
{
    constexpr int G = WAVE / NZM, CW = NZM / G;
    const int nz = c.nz, i = c.tid / G, g = c.tid % G;
    double acc = 0.0;
#pragma unroll
    for (int q = 0; q < CW; q++) {
        const int j = CW * g + q;
        if (i < nz && j < nz) acc = fma(M[i * nz + j], x[j], acc);
    }
    if (G >= 2) acc += dpp_d<0xB1>(acc);
    if (G >= 4) acc += dpp_d<0x4E>(acc);
    return acc;
}

// out = H^-1 gin with one step of iterative refinement (x = M g; x += M (g - H x)):
// the explicit inverse alone is not backward stable, and near the end of an interior-
// point solve H carries barrier weights of 1e8..1e12.  gin, out, c.bc scratch in LDS.
template <int NZM>
__device__ __forceinline__ void gj_solve(const Ctx &c, const double *H, const double *Minv, const double *gin, double *out)
{
    constexpr int G = WAVE / NZM;
    const int nz = c.nz, i = c.tid / G, g = c.tid % G;
    double *xs = c.bc, *rs = c.bc + WAVE;
    const double x0 = gj_matvec<NZM>(c, Minv, gin);
    if (g == 0 && i < nz) xs[i] = x0;
    __syncthreads();
    const double r = (i < nz ? gin[i] : 0.0) - gj_matvec<NZM>(c, H, xs);
    if (g == 0 && i < nz) rs[i] = r;
    __syncthreads();
    const double x1 = x0 + gj_matvec<NZM>(c, Minv, rs);
    if (g == 0 && i < nz) out[i] = x1;
    __syncthreads();
}

// out[0..nz) = Z' v (LDS).  Lanes (a, d) = (4a + d) sum the X rows of state component d
// over grids >= stage(a); the quad is reduced by DPP; the U/lambda rows of the column's
// own grid are added by the d == 0 / d == 1 lanes.
template <int NZM>
__device__ __forceinline__ void zt_mul(const Ctx &c, const double *v, double *out)
{
    const int N = c.N, nz = c.nz, C = c.C, d = c.tid & 3;
#pragma unroll
    for (int round = 0; round < (NZM + 15) / 16; round++) {
        const int a = round * 16 + (c.tid >> 2);
        double acc = 0.0;
        if (a < nz) {
            const int ja = col_stage(c, a);
            if (ja < N) {
                double a0 = 0.0, a1 = 0.0;
                int k = ja;
                for (; k + 1 < N; k += 2) {
                    a0 += c.Z[(4 * k + d) * c.ldz + a] * v[4 * k + d];
                    a1 += c.Z[(4 * (k + 1) + d) * c.ldz + a] * v[4 * (k + 1) + d];
                }
                if (k < N) a0 += c.Z[(4 * k + d) * c.ldz + a] * v[4 * k + d];
                acc = a0 + a1;
                if (d == 0) {
                    for (int r = 4 * N + 2 * ja; r < 4 * N + 2 * ja + 2; r++) acc += c.Z[r * c.ldz + a] * v[r];
                } else if (d == 1) {
                    for (int r = 6 * N + C * ja; r < 6 * N + C * ja + C; r++) acc += c.Z[r * c.ldz + a] * v[r];
                }
            } else if (d == 0) {
                acc = v[c.n - 1];
            }
        }
        acc += dpp_d<0xB1>(acc);
        acc += dpp_d<0x4E>(acc);
        if (d == 0 && a < nz) out[a] = acc;
    }
    __syncthreads();
}

// out = Z xi  (xi in LDS); columns of grid j reach X rows of grids >= j and
// the U/lambda rows of grid j only.
template <int NZM>
__device__ __forceinline__ void z_mul(const Ctx &c, const double *xs, double *out)
{
    const int N = c.N, nz = c.nz, C = c.C, n = c.n;
    for (int v = c.tid; v < n; v += WAVE) {
        double a0 = 0.0, a1 = 0.0;
        if (v < 4 * N) {
            const int lim = ((v >> 2) + 1) * (C - 1);     // columns of grids <= k
            int a = 0;
            for (; a + 1 < lim; a += 2) {
                a0 += c.Z[v * c.ldz + a] * xs[a];
                a1 += c.Z[v * c.ldz + a + 1] * xs[a + 1];
            }
            if (a < lim) a0 += c.Z[v * c.ldz + a] * xs[a];
        } else if (v < n - 1) {
            const int j = (v < 6 * N) ? (v - 4 * N) >> 1 : (v - 6 * N) / C;
            for (int a = j * (C - 1); a < (j + 1) * (C - 1); a++) a0 += c.Z[v * c.ldz + a] * xs[a];
        } else {
            a0 = xs[nz - 1];
        }
        out[v] = a0 + a1;
    }
    __syncthreads();
}

// Newton solve with the current factor L and weights om:
//   [H A' J'; A 0 0; J 0 -W][dx;dy;dz] = [r1; 0; r3], W^-1 = om
// r1 (n) given, r3 in r3dz on entry (overwritten with dz).  dx -> c.dx.  Uses c.tv, c.dsv.
template <int NZM>
__device__ __forceinline__ void newton_solve(const Ctx &c, const double *r1, double *r3dz, int sslot)
{
    double *w = c.dsv;                      // scratch m-vector (callers recompute dsv after)
    for (int r = c.tid; r < c.m; r += WAVE) w[r] = c.om[r] * r3dz[r];
    __syncthreads();
    jt_apply(c, w, c.tv, r1, 1.0);
    STAMP_END(c, sslot + 0);
    zt_mul<NZM>(c, c.tv, c.gbuf);
    STAMP_END(c, sslot + 1);
    gj_solve<NZM>(c, c.Hc, c.L, c.gbuf, c.xiv);
    STAMP_END(c, sslot + 2);
    z_mul<NZM>(c, c.xiv, c.dx);
    STAMP_END(c, sslot + 3);
    for (int r = c.tid; r < c.m; r += WAVE) r3dz[r] = c.om[r] * (row_dot(c, r, c.dx) - r3dz[r]);
    __syncthreads();
    STAMP_END(c, sslot + 4);
}

// findsteplength (Auxilary.c:271-294): min over dv_r < 0 of -v_r/dv_r, 1 when no dv_r < 0.
// Evaluated as 1 / max_r(-dv_r * (1/v_r)) with the per-iteration reciprocals of s and z,
// so one division per call instead of one per row (equal up to rounding).  Uniform.
__device__ __forceinline__ double steplen(const Ctx &c, const double *inv_v, const double *dv)
{
    double mx = 0.0;
    for (int r = c.tid; r < c.m; r += WAVE) mx = fmax(mx, -dv[r] * inv_v[r]);
    mx = wmax(mx);
    return (mx > 0.0) ? 1.0 / mx : 1.0;
}

// One interior-point solve (QP stage: nl = 0, iSWIFT; NLP stage: nl = 1).
// Returns exit code; *iters gets the number of steps taken.
template <int NZM>
__device__ __forceinline__ int ipm(Ctx &c, int maxit, int *iters)
{
    const double tol = c.P->tol, th = tol / sqrt(3.0);
    double sigma = 100.0;               // options->sigma = SIGMA
    const double sigma_d = 0.0;
    int flag = 2, it = 0;
    double delta = 0.0;
    const int sb = c.nl ? 32 : 0;       // stamp slots: QP 0..17, NLP 32..49 (tools/stamps.py)
    for (int iter = 0; iter < maxit; iter++) {
        // Opaque lane id per iteration: per-lane addresses are recomputed inside the loop
        // instead of being hoisted out of it and held in registers for its whole length.
        asm volatile("" : "+v"(c.tid));
        STAMP_BEGIN(c);
        if (c.nl) obstacle_coefs(c);
        // rz = h - s - g(x); tv = -(P x + c) - q
        for (int r = c.tid; r < c.m; r += WAVE) c.rz[r] = c.hvec[r] - c.s[r] - row_val(c, r);
        for (int v = c.tid; v < c.n; v += WAVE) c.tv[v] = -(Pdiag(c, v) * c.x[v] + cvec(c, v)) - c.q[v];
        __syncthreads();
        jt_apply(c, c.z, c.rx, c.tv, -1.0);     // rx = -(P x + c) - q - J'z
        double nrx = 0, nrz = 0, sz = 0, mu = 0, gm = 1.0;
        for (int v = c.tid; v < c.n; v += WAVE) {
            nrx += c.rx[v] * c.rx[v];
            if (c.nl) gm = fmax(gm, fabs(Pdiag(c, v) * c.x[v] + cvec(c, v)));
        }
        for (int r = c.tid; r < c.m; r += WAVE) {
            const double sr = c.s[r], zr = c.z[r];
            nrz += c.rz[r] * c.rz[r]; sz += sr * zr;
            const double l2 = sr * zr;                        // formlambda then lambda.*lambda
            c.l2[r] = l2; mu += l2;
            c.iz[r] = rcp_d(zr); c.is[r] = rcp_d(sr);
        }
        nrx = sqrt(wsum(nrx)); nrz = sqrt(wsum(nrz)); sz = wsum(sz); mu = wsum(mu) / c.m;
        if (c.nl) gm = wmax(gm);
        STAMP_END(c, sb + 0);
        if (!isfinite(nrx) || !isfinite(nrz) || !isfinite(sz)) { flag = 3; break; }
        // NLP: dual residual scaled by max(1, ||Q x + f||_inf) (QP: iSWIFT's absolute test)
        const double thx = c.nl ? th * gm : th;
        if (nrx < thx && nrz < th && sz / c.m < tol) { flag = 0; break; }
        const int pc = c.nl || (sigma > sigma_d);
        if (pc) {
            // weights W^-1 = z/s (updatekktmatrix, Auxilary.c:197-205) and factor
            for (int r = c.tid; r < c.m; r += WAVE) c.om[r] = c.z[r] * c.is[r];
            __syncthreads();
            STAMP_END(c, sb + 1);
            delta = 0.0;
            double dstart = 0.0;
            int ok = 0;
            for (int tries = 0; tries < (c.nl ? 14 : 1); tries++) {
                build_D(c, delta);
                STAMP_END(c, sb + 2);
                build_Hc<NZM>(c, c.Hc, 0);
                STAMP_END(c, sb + 3);
                if (tries == 0) {       // scale-aware first shift: 1e-10 * max(1, max diag of Z'HZ)
                    double dm = 1.0;
                    for (int a = c.tid; a < c.nz; a += WAVE) dm = fmax(dm, c.Hc[a * c.nz + a]);
                    dstart = 1e-10 * wmax(dm);
                }
                int cf = gj_inverse<NZM>(c, c.Hc, c.L, c.nz, !c.nl);
                STAMP_END(c, sb + 4);
                if (cf == 0) { ok = 1; break; }
                delta = (delta == 0.0) ? dstart : delta * 10.0;
            }
            if (!ok) { flag = 1; break; }
            // predictor: ds = -lambda.*lambda
            for (int r = c.tid; r < c.m; r += WAVE) {
                c.dsT[r] = -c.l2[r];
                c.dz[r] = c.rz[r] - c.dsT[r] * c.iz[r];
            }
            __syncthreads();
            STAMP_END(c, sb + 5);
            newton_solve<NZM>(c, c.rx, c.dz, sb + 6);
            for (int r = c.tid; r < c.m; r += WAVE) c.dsv[r] = (c.dsT[r] - c.s[r] * c.dz[r]) * c.iz[r];
            __syncthreads();
            double ap = steplen(c, c.is, c.dsv), ad = steplen(c, c.iz, c.dz);
            double num = 0;
            for (int r = c.tid; r < c.m; r += WAVE) num += (c.s[r] + ap * c.dsv[r]) * (c.z[r] + ad * c.dz[r]);
            num = wsum(num);
            double rho = num / sz, mr = rho < 1.0 ? rho : 1.0;
            sigma = mr * mr * mr; if (sigma < sigma_d) sigma = sigma_d;
            for (int r = c.tid; r < c.m; r += WAVE) c.dsT[r] = -c.l2[r] - (c.dsv[r] * c.dz[r]) + sigma * mu;
        } else {
            // Prime.c:193-196: centring step with the previous factor
            sigma = sigma_d;
            for (int r = c.tid; r < c.m; r += WAVE) c.dsT[r] = -c.l2[r] + sigma * mu;
        }
        __syncthreads();
        for (int r = c.tid; r < c.m; r += WAVE) c.dz[r] = c.rz[r] - c.dsT[r] * c.iz[r];
        __syncthreads();
        STAMP_END(c, sb + 11);
        newton_solve<NZM>(c, c.rx, c.dz, sb + 12);
        for (int r = c.tid; r < c.m; r += WAVE) c.dsv[r] = (c.dsT[r] - c.s[r] * c.dz[r]) * c.iz[r];
        // dq = A'dy = rx - (P + hess + delta) dx - J' dz
        for (int v = c.tid; v < c.n; v += WAVE)
            c.tv[v] = c.rx[v] - (Pdiag(c, v) + hess_diag(c, v) + (c.nl ? delta : 0.0)) * c.dx[v];
        __syncthreads();
        double ap = steplen(c, c.is, c.dsv), ad = steplen(c, c.iz, c.dz);
        ap = (0.99 * ap < 1.0) ? 0.99 * ap : 1.0;
        ad = (0.99 * ad < 1.0) ? 0.99 * ad : 1.0;
        // tv - J'dz needs the dz of this step: apply before updating z (hess uses old z)
        jt_apply(c, c.dz, c.tv, c.tv, -1.0);
        for (int v = c.tid; v < c.n; v += WAVE) { c.x[v] += c.dx[v] * ap; c.q[v] += c.tv[v] * ad; }
        for (int r = c.tid; r < c.m; r += WAVE) { c.s[r] += c.dsv[r] * ap; c.z[r] += c.dz[r] * ad; }
        __syncthreads();
        STAMP_END(c, sb + 17);
        it++;
    }
    *iters = it;
    return flag;
}

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
    // n_i = (-1)^i det of [F; 1'] with column i removed
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
    int i = (t < istar) ? t : t + 1;           // the two of {0,1,2} other than istar
    lam[i] = 1.0; lam[3] = -1.0;
    return 0;
}

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
__device__ __forceinline__ void knn_select(const Ctx &c, double px, double py, const double *__restrict__ tab,
                                           int stride, int n_rows, int self, int K, int *sel)
{
    double bd[SRB_KNN_MAX]; int bi[SRB_KNN_MAX];
#pragma unroll
    for (int j = 0; j < SRB_KNN_MAX; j++) { bd[j] = 1e300; bi[j] = 0x7fffffff; }
    double wd = 1e300;                                  // this lane's K-th best (admission threshold)
    for (int i = c.tid; i < n_rows; i += WAVE) {
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
        if (bi[0] == idx) {                             // the owning lane pops its head
#pragma unroll
            for (int t = 0; t + 1 < SRB_KNN_MAX; t++) { bd[t] = bd[t + 1]; bi[t] = bi[t + 1]; }
            bd[SRB_KNN_MAX - 1] = 1e300; bi[SRB_KNN_MAX - 1] = 0x7fffffff;
        }
        if (c.tid == 0) sel[j] = (idx == 0x7fffffff) ? -1 : idx;
    }
}

// --------------------------------------------------------------------------- main kernel
template <int NZM>
__device__ __forceinline__ void nmpc_agent(const SrbKParams &prm, int agent,
                const double *__restrict__ x0g, const double *__restrict__ refg, const double *__restrict__ footg,
                const double *__restrict__ obstacles, int n_obs,
                const double *__restrict__ nbr_state, int n_all, int agent_offset,
                double *__restrict__ x_qp_out, double *__restrict__ x_out,
                double *__restrict__ obj_out, int *__restrict__ status_out, int *__restrict__ iters_out,
                double *lds)
{
    Ctx c;
    c.P = &prm; c.tid = threadIdx.x;
    c.N = prm.N; c.C = prm.C; c.K = prm.K_obs + prm.K_nbr;
    c.n = prm.n; c.nz = prm.nz; c.mq = prm.mq;
    const int N = c.N, C = c.C, n = c.n, nz = c.nz, K = c.K;
    c.rFm = 2 * (N - 1); c.rXp = 4 * (N - 1); c.rXm = c.rXp + 4 * N; c.rUp = c.rXm + 4 * N;
    c.rUm = c.rUp + 2 * N; c.rLlo = c.rUm + 2 * N; c.rLhi = c.rLlo + C * N;
    c.rO = c.mq; c.rV = c.mq + N * K;
    const int mmax = prm.use_nlp ? (c.mq + N * K + 4 * N) : c.mq;
    // carve LDS (offsets must match srb_lds_doubles())
    double *p = lds;
    c.ldz = SRB_LDZ(nz); c.n16 = SRB_R16(n);
    const int cpl16 = SRB_R16(SRB_NCPL2(N));
    c.Z = p; p += c.n16 * c.ldz;
    c.x = p; p += n; c.q = p; p += n; c.rx = p; p += n; c.dx = p; p += n; c.tv = p; p += n;
    c.D = p; p += c.n16 + cpl16; c.term = (int2 *)p; p += cpl16;
    c.ref = p; p += 4 * N; c.foot = p; p += 2 * C * N;
    c.s = p; p += mmax; c.z = p; p += mmax; c.rz = p; p += mmax; c.dz = p; p += mmax;
    c.dsv = p; p += mmax; c.dsT = p; p += mmax; c.om = p; p += mmax; c.hvec = p; p += mmax;
    c.iz = p; p += mmax; c.is = p; p += mmax; c.l2 = p; p += mmax;
    c.jc = p; p += 2 * N * K + 2; c.obs = p; p += 2 * N * K + 2; c.eps = p; p += K + 1;
    // assembled matrices and their inverses (the solves refine against the originals)
    c.Hc = p; p += nz * nz; c.L = p; p += nz * nz; c.ZtZ = p; p += nz * nz; c.ZtZL = p; p += nz * nz;
    c.xiv = p; p += WAVE; c.gbuf = p; p += WAVE;
    c.bc = p; p += 4 * WAVE;
#ifdef SRB_STAMPS
    c.stamps = (unsigned long long *)p; p += SRB_NSTAMP;
    c.stamps[c.tid] = 0;
    __syncthreads();
#endif

    STAMP_BEGIN(c);
    // ---- load inputs (a1/a2/a3: x0, reference window, footholds)
    const double *x0 = x0g + 4 * (size_t)agent;
    for (int i = c.tid; i < 4 * N; i += WAVE) c.ref[i] = refg[(size_t)agent * 4 * N + i];
    for (int i = c.tid; i < 2 * C * N; i += WAVE) c.foot[i] = footg[(size_t)agent * 2 * C * N + i];
    for (int i = c.tid; i < c.n16 * c.ldz; i += WAVE) c.Z[i] = 0.0;
    for (int i = c.tid; i < c.n16 + cpl16; i += WAVE) c.D[i] = 0.0;      // padding terms stay 0
    __syncthreads();

    // ---- null-space basis Z and particular point xbar (forward LIP rollout, MPC_dist.cpp:232-261)
    if (c.tid == 0) {
        double X[4] = {x0[0], x0[1], x0[2], x0[3]};
        for (int k = 0; k < N; k++) {
            double u0 = c.foot[(k * 2 + 0) * C + C - 1], u1 = c.foot[(k * 2 + 1) * C + C - 1];
            double Xn[4];
            for (int d = 0; d < 4; d++)
                Xn[d] = prm.Ad[d * 4] * X[0] + prm.Ad[d * 4 + 1] * X[1] + prm.Ad[d * 4 + 2] * X[2] + prm.Ad[d * 4 + 3] * X[3] +
                        prm.Bd[d * 2] * u0 + prm.Bd[d * 2 + 1] * u1;
            for (int d = 0; d < 4; d++) { X[d] = Xn[d]; c.x[4 * k + d] = Xn[d]; }
            c.x[4 * N + 2 * k] = u0; c.x[4 * N + 2 * k + 1] = u1;
            for (int j = 0; j < C; j++) c.x[6 * N + C * k + j] = (j == C - 1) ? 1.0 : 0.0;
        }
        c.x[n - 1] = 0.0;
    }
    for (int col = c.tid; col < nz - 1; col += WAVE) {
        int j = col / (C - 1), t = col % (C - 1);
        double lam[4];
        int is_null = lambda_basis(c.foot + j * 2 * C, C, t, lam);
        double g0 = 0.0, g1 = 0.0;
        if (!is_null)
            for (int i = 0; i < C; i++) { g0 += c.foot[(j * 2 + 0) * C + i] * lam[i]; g1 += c.foot[(j * 2 + 1) * C + i] * lam[i]; }
        for (int i = 0; i < C; i++) c.Z[(6 * N + C * j + i) * c.ldz + col] = lam[i];
        c.Z[(4 * N + 2 * j) * c.ldz + col] = g0;
        c.Z[(4 * N + 2 * j + 1) * c.ldz + col] = g1;
        double v[4];
        for (int d = 0; d < 4; d++) v[d] = prm.Bd[d * 2] * g0 + prm.Bd[d * 2 + 1] * g1;
        for (int k = j; k < N; k++) {
            for (int d = 0; d < 4; d++) c.Z[(4 * k + d) * c.ldz + col] = v[d];
            double tt[4];
            for (int d = 0; d < 4; d++) tt[d] = prm.Ad[d * 4] * v[0] + prm.Ad[d * 4 + 1] * v[1] + prm.Ad[d * 4 + 2] * v[2] + prm.Ad[d * 4 + 3] * v[3];
            for (int d = 0; d < 4; d++) v[d] = tt[d];
        }
    }
    if (c.tid == 0) c.Z[(n - 1) * c.ldz + nz - 1] = 1.0;
    __syncthreads();
    term_table(c);

    STAMP_END(c, 28);
    // One loop over the two stages so that the interior-point iteration exists once in
    // the code object (the solve is latency-bound; keeping the hot loop small keeps it in
    // the instruction cache).  stage 0: QP (iSWIFT, Prime.c:35-230); stage 1: NLP
    // (replaces SnoptSolver::Solve, MPC_dist.cpp:402-427), warm-started from stage 0.
    int qp_flag = 3, qp_it = 0, nlp_flag = 0, nlp_it = 0;
    const int nstage = prm.use_nlp ? 2 : 1;
#pragma clang loop unroll(disable)
    for (int stage = 0; stage < nstage; stage++) {
        asm volatile("" : "+v"(c.tid));     // see ipm()
        if (stage == 0) {
            c.m = c.mq; c.nl = 0;
            for (int r = c.tid; r < c.m; r += WAVE) c.hvec[r] = row_h(c, r);
            for (int r = c.tid; r < c.m; r += WAVE) c.om[r] = 1.0;     // kkt_initialize: -I block
            __syncthreads();
            build_D(c, 0.0);
            build_Hc<NZM>(c, c.Hc, 0);
            if (gj_inverse<NZM>(c, c.Hc, c.L, nz, 1) != 0) { qp_flag = 1; continue; }
            // r1 = -c - P xbar ; r3 = h - G xbar   ->  dx ; x = xbar + dx
            for (int v = c.tid; v < n; v += WAVE) c.rx[v] = -cvec(c, v) - Pdiag(c, v) * c.x[v];
            for (int r = c.tid; r < c.m; r += WAVE) c.dz[r] = c.hvec[r] - row_dot(c, r, c.x);
            __syncthreads();
            newton_solve<NZM>(c, c.rx, c.dz, 20);   // dz <- G x - h (z of the init system)
            for (int v = c.tid; v < n; v += WAVE) c.x[v] += c.dx[v];
            __syncthreads();
            // q = A'y = -c - P x - G'(G x - h)
            for (int v = c.tid; v < n; v += WAVE) c.tv[v] = -cvec(c, v) - Pdiag(c, v) * c.x[v];
            __syncthreads();
            jt_apply(c, c.dz, c.q, c.tv, -1.0);
            // s, z from z_inter = h - G x (Auxilary.c:716-746)
            double mn = 1e300, mx = -1e300;
            for (int r = c.tid; r < c.m; r += WAVE) {
                double zi = c.hvec[r] - row_dot(c, r, c.x);
                c.rz[r] = zi;
                mn = fmin(mn, zi); mx = fmax(mx, zi);
            }
            mn = wmin(mn); mx = wmax(mx);
            double ap = -mn, ad = mx;
            for (int r = c.tid; r < c.m; r += WAVE) {
                double zi = c.rz[r];
                c.s[r] = (ap < 0) ? zi : zi + (1 + ap);
                c.z[r] = (ad < 0) ? -zi : -zi + (1 + ad);
            }
            __syncthreads();
            STAMP_END(c, 29);
        } else {
            if (x_qp_out)
                for (int v = c.tid; v < n; v += WAVE) x_qp_out[(size_t)agent * n + v] = c.x[v];
            c.nl = 1; c.m = mmax;
            // obstacles per grid: the K_obs nearest static obstacles (MPC_dist.cpp:371-396,
            // generalised to K) and the K_nbr nearest other agents (get_lastState() rows),
            // predicted at constant velocity o_k = p + v Ts (k+1); query point = own CoM.
            int *sel = (int *)c.jc;                     // scratch until obstacle_coefs
#pragma clang loop unroll(disable)
            for (int tsel = 0; tsel < 2; tsel++) {
                const int Kt = tsel ? prm.K_nbr : prm.K_obs;
                if (Kt > 0)
                    knn_select(c, x0[0], x0[2], tsel ? nbr_state : obstacles, tsel ? 4 : 2, tsel ? n_all : n_obs,
                               tsel ? agent_offset + agent : -1, Kt, sel + (tsel ? prm.K_obs : 0));
            }
            __syncthreads();
            for (int j = 0; j < K; j++) {
                const bool st = j < prm.K_obs;
                const int bi = sel[j];
                if (c.tid < N && bi >= 0) {
                    const int k = c.tid;
                    const double t = st ? 0.0 : prm.Ts * (k + 1);
                    const double *srcp = st ? obstacles + 2 * (size_t)bi : nbr_state + 4 * (size_t)bi;
                    c.obs[2 * (k * K + j)] = srcp[0] + (st ? 0.0 : srcp[2] * t);
                    c.obs[2 * (k * K + j) + 1] = srcp[1] + (st ? 0.0 : srcp[3] * t);
                }
                if (c.tid == 0) c.eps[j] = st ? prm.eps_obs : prm.eps_nbr;
            }
            __syncthreads();
            for (int r = c.tid; r < c.m; r += WAVE) c.hvec[r] = row_h(c, r);
            __syncthreads();
            obstacle_coefs(c);
            // slacks: shifted h - g(x); duals 1
            double mn = 1e300;
            for (int r = c.tid; r < c.m; r += WAVE) {
                c.rz[r] = c.hvec[r] - row_val(c, r);
                mn = fmin(mn, c.rz[r]);
            }
            mn = wmin(mn);
            double ap = -mn;
            for (int r = c.tid; r < c.m; r += WAVE) { c.s[r] = (ap < 0) ? c.rz[r] : c.rz[r] + (1 + ap); c.z[r] = 1.0; }
            // Z'Z and its factor: projection for q0
            build_Hc<NZM>(c, c.ZtZ, 1);
            gj_inverse<NZM>(c, c.ZtZ, c.ZtZL, nz, 0);
            // v = P x + c + J'z ; rx0 = -Z (Z'Z)^-1 Z' v ; q = -v - rx0
            for (int v = c.tid; v < n; v += WAVE) c.tv[v] = Pdiag(c, v) * c.x[v] + cvec(c, v);
            __syncthreads();
            jt_apply(c, c.z, c.rx, c.tv, 1.0);
            zt_mul<NZM>(c, c.rx, c.gbuf);
            gj_solve<NZM>(c, c.ZtZ, c.ZtZL, c.gbuf, c.xiv);
            z_mul<NZM>(c, c.xiv, c.dx);
            for (int v = c.tid; v < n; v += WAVE) c.q[v] = -c.rx[v] + c.dx[v];
            __syncthreads();
            STAMP_END(c, 30);
        }
        int it = 0;
        const int f = ipm<NZM>(c, stage == 0 ? prm.qp_maxit : prm.nlp_maxit, &it);
        if (stage == 0) { qp_flag = f; qp_it = it; } else { nlp_flag = f; nlp_it = it; }
        STAMP_BEGIN(c);
    }
    if (x_qp_out && nstage == 1)
        for (int v = c.tid; v < n; v += WAVE) x_qp_out[(size_t)agent * n + v] = c.x[v];

    // ---- outputs
    for (int v = c.tid; v < n; v += WAVE) x_out[(size_t)agent * n + v] = c.x[v];
    double f = 0;
    for (int v = c.tid; v < n; v += WAVE) f += 0.5 * Pdiag(c, v) * c.x[v] * c.x[v] + cvec(c, v) * c.x[v];
    f = wsum(f);
    STAMP_END(c, 31);
#ifdef SRB_STAMPS
    if (agent == 0) atomicAdd(&srb_stamp_buf[c.tid], c.stamps[c.tid]);
#endif
    if (c.tid == 0) {
        obj_out[agent] = f;
        status_out[2 * agent] = qp_flag; status_out[2 * agent + 1] = nlp_flag;
        iters_out[2 * agent] = qp_it; iters_out[2 * agent + 1] = nlp_it;
    }
}

#define SRB_NMPC_KERNEL(NAME, NZM)                                                                            \
    extern "C" __global__ void __launch_bounds__(WAVE) NAME(                                                   \
        SrbKParams prm, int n_agents, const double *__restrict__ x0g, const double *__restrict__ refg,          \
        const double *__restrict__ footg, const double *__restrict__ obstacles, int n_obs,                       \
        const double *__restrict__ nbr_state, int n_all, int agent_offset, double *__restrict__ x_qp_out,        \
        double *__restrict__ x_out, double *__restrict__ obj_out, int *__restrict__ status_out,                 \
        int *__restrict__ iters_out)                                                                           \
    {                                                                                                          \
        extern __shared__ __attribute__((aligned(16))) double lds[];                                           \
        const int agent = blockIdx.x;                                                                          \
        if (agent >= n_agents) return;                                                                         \
        nmpc_agent<NZM>(prm, agent, x0g, refg, footg, obstacles, n_obs, nbr_state, n_all, agent_offset,       \
                        x_qp_out, x_out,                                                                       \
                        obj_out, status_out, iters_out, lds);                                                  \
    }

SRB_NMPC_KERNEL(srb_nmpc_kernel_nz16, 16)
SRB_NMPC_KERNEL(srb_nmpc_kernel_nz32, 32)
