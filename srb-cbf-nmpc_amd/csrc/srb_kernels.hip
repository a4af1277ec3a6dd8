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
__device__ __forceinline__ double wsum(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
    return v;
}
__device__ __forceinline__ double wmin(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, WAVE));
    return v;
}
__device__ __forceinline__ double wmax(double v) { return -wmin(-v); }
__device__ __forceinline__ int wor(int v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o, WAVE);
    return v;
}
// value of lane `lane` (wave-uniform index, SGPR) -> wave-uniform value
__device__ __forceinline__ double readlane_d(double v, int lane)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, lane);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// --------------------------------------------------------------------------- diagnostic stamps
// Built only with -DSRB_STAMPS (make stamps -> srbnmpc/libsrbnmpc_stamps.so): lane 0 of
// agent 0 accumulates s_memtime cycles per phase into a buffer nothing else reads.
#ifdef SRB_STAMPS
__device__ unsigned long long srb_stamp_buf[32];
#define STAMP_DECL unsigned long long _st_t0 = 0; const bool _st_on = (blockIdx.x == 0 && threadIdx.x == 0);
#define STAMP_BEGIN() do { __builtin_amdgcn_sched_barrier(0); _st_t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); } while (0)
#define STAMP_END(slot) do { __builtin_amdgcn_sched_barrier(0); unsigned long long _t = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0); if (_st_on) srb_stamp_buf[slot] += _t - _st_t0; _st_t0 = _t; } while (0)
#else
#define STAMP_DECL
#define STAMP_BEGIN() do {} while (0)
#define STAMP_END(slot) do {} while (0)
#endif

// --------------------------------------------------------------------------- per-agent context
struct Ctx {
    const SrbKParams *P;
    int N, C, K, n, nz, mq, m, nl;          // nl: NLP rows/terms active
    int rFm, rXp, rXm, rUp, rUm, rLlo, rLhi, rO, rV;
    // LDS arrays
    double *Z, *x, *q, *rx, *dx, *tv, *D, *ref, *foot, *offv;
    double *s, *z, *rz, *dz, *dsv, *dsT, *om, *iz, *is, *l2, *jc, *obs, *eps;
    double *Hc, *L, *dinv, *ZtZ, *ZtZL, *ZtZdinv, *hvec, *xiv;
    int tid;
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
// D (diag of H), friction couplings offv[0..2N-3], obstacle couplings per grid
// (xy, xs, ys) at offv[2N-2 + 3k].  H = P + hess + delta I + J' diag(om) J.
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
    const int nf = 2 * (N - 1);
    for (int e = c.tid; e < nf; e += WAVE) c.offv[e] = -(c.om[e] + c.om[c.rFm + e]);
    if (c.nl)
        for (int k = c.tid; k < N; k += WAVE) {
            double xy = 0, xs = 0, ys = 0;
            for (int j = 0; j < c.K; j++) {
                int o = k * c.K + j;
                double w = c.om[c.rO + o], jx = c.jc[2 * o], jy = c.jc[2 * o + 1];
                xy += w * jx * jy; xs -= w * jx; ys -= w * jy;
            }
            c.offv[nf + 3 * k] = xy; c.offv[nf + 3 * k + 1] = xs; c.offv[nf + 3 * k + 2] = ys;
        }
    __syncthreads();
}

// out[a][b] = (Z' H Z)[a][b] from the structurally nonzero terms only:
//   lambda columns of grid j touch X rows of grids >= j, the U/lambda rows of grid j;
//   a friction coupling (X_i pos, U_{i+1}) links columns of grids <= i and i+1;
//   the s column touches only s and (NLP) the obstacle couplings.
// unit != 0: H = I (gives Z'Z).
__device__ __forceinline__ void build_Hc(const Ctx &c, double *out, int unit)
{
    const int N = c.N, n = c.n, nz = c.nz, C = c.C, nf = 2 * (N - 1);
    const double *Z = c.Z, *D = c.D, *off = c.offv;
    const int npair = nz * (nz + 1) / 2;
    for (int pidx = c.tid; pidx < npair; pidx += WAVE) {
        int b = (int)((sqrt(8.0 * pidx + 1.0) - 1.0) * 0.5);
        while (b * (b + 1) / 2 > pidx) b--;
        while ((b + 1) * (b + 2) / 2 <= pidx) b++;
        const int a = pidx - b * (b + 1) / 2;          // a <= b, so stage(a) <= stage(b)
        const int ja = col_stage(c, a), jb = col_stage(c, b);
        double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0, acc3 = 0.0;
        if (jb < N) {
            // X rows of grids >= jb: 4 independent accumulators (one per state component)
            for (int k = jb; k < N; k++) {
                const int v = 4 * k;
                const double d0 = unit ? 1.0 : D[v], d1 = unit ? 1.0 : D[v + 1];
                const double d2 = unit ? 1.0 : D[v + 2], d3 = unit ? 1.0 : D[v + 3];
                acc0 += d0 * Z[v * nz + a] * Z[v * nz + b];
                acc1 += d1 * Z[(v + 1) * nz + a] * Z[(v + 1) * nz + b];
                acc2 += d2 * Z[(v + 2) * nz + a] * Z[(v + 2) * nz + b];
                acc3 += d3 * Z[(v + 3) * nz + a] * Z[(v + 3) * nz + b];
                if (c.nl && !unit) {
                    const double xa = Z[v * nz + a], ya = Z[(v + 2) * nz + a];
                    const double xb = Z[v * nz + b], yb = Z[(v + 2) * nz + b];
                    acc1 += off[nf + 3 * k] * (xa * yb + ya * xb);
                }
            }
            if (ja == jb) {
                for (int v = 4 * N + 2 * ja; v < 4 * N + 2 * ja + 2; v++)
                    acc2 += (unit ? 1.0 : D[v]) * Z[v * nz + a] * Z[v * nz + b];
                for (int v = 6 * N + C * ja; v < 6 * N + C * ja + C; v++)
                    acc3 += (unit ? 1.0 : D[v]) * Z[v * nz + a] * Z[v * nz + b];
            } else if (!unit) {
                const int i = jb - 1;                 // friction rows between grid i pos and grid jb CoP
                for (int d = 0; d < 2; d++)
                    acc0 += off[2 * i + d] * Z[(4 * i + 2 * d) * nz + a] * Z[(4 * N + 2 * jb + d) * nz + b];
            }
        } else if (ja < N) {
            if (c.nl && !unit)
                for (int k = ja; k < N; k++)
                    acc0 += off[nf + 3 * k + 1] * Z[(4 * k) * nz + a] + off[nf + 3 * k + 2] * Z[(4 * k + 2) * nz + a];
        } else {
            acc0 = unit ? 1.0 : D[n - 1];
        }
        const double acc = (acc0 + acc1) + (acc2 + acc3);
        out[a * nz + b] = acc;
        out[b * nz + a] = acc;
    }
    __syncthreads();
}

// --------------------------------------------------------------------------- register Cholesky
// Lane i holds row i of the trailing matrix in a register window row[0..NZM-1] that
// shifts left by one column per elimination step, so the pivot column is always row[0]
// and every register index is a compile-time constant while the step loop over k stays
// a runtime loop (small code: one copy of an NZM-wide body).  Cross-lane operands move
// by v_readlane with a wave-uniform lane index.  Writes L (lower, LDS) and 1/L_kk.
// regularise != 0 mirrors iSWIFT's dynamic pivot regularisation (ldl.c:320-321:
// |D_kk| <= 1e-14 -> 1e-7) for the QP stage.  Returns 0 on success (wave-uniform).
template <int NZM>
__device__ __forceinline__ int chol_reg(const Ctx &c, const double *H, double *L, double *dinv, int nz, int regularise)
{
    const int i = c.tid;
    double row[NZM];
#pragma unroll
    for (int j = 0; j < NZM; j++) row[j] = (i < nz && j < nz) ? H[i * nz + j] : 0.0;
    int fail = 0;
#pragma clang loop unroll(disable)
    for (int k = 0; k < nz; k++) {
        double piv = readlane_d(row[0], k);
        if (regularise && piv <= 1e-14 && piv == piv) piv = 1e-7;
        if (!(piv > 0.0)) { fail = 1; break; }
        const double d = sqrt(piv), inv = 1.0 / d;
        const double l = (i > k && i < nz) ? row[0] * inv : 0.0;
        if (i > k && i < nz) L[i * nz + k] = l;
        if (i == k) { L[k * nz + k] = d; dinv[k] = inv; }
#pragma unroll
        for (int t = 1; t < NZM; t++) {
            const double lj = readlane_d(l, (k + t) & (WAVE - 1));   // lanes <= k hold l = 0
            row[t - 1] = row[t] - l * lj;
        }
        row[NZM - 1] = 0.0;
    }
    __syncthreads();
    return fail;
}

// (L L') x = b with b one entry per lane (lane i < nz); returns x in the same layout.
// Runtime loops; the L operand of step k+1 is loaded while step k completes.
__device__ __forceinline__ double chol_solve_reg(const Ctx &c, const double *L, const double *dinv, int nz, double b)
{
    const int i = c.tid;
    double lnext = (i > 0 && i < nz) ? L[i * nz] : 0.0;
#pragma clang loop unroll(disable)
    for (int k = 0; k < nz; k++) {
        const double lik = lnext;
        lnext = (k + 1 < nz && i > k + 1 && i < nz) ? L[i * nz + k + 1] : 0.0;
        const double yk = readlane_d(b, k) * dinv[k];
        b = (i == k) ? yk : b - lik * yk;
    }
    lnext = (nz - 1 > i) ? L[(nz - 1) * nz + i] : 0.0;
#pragma clang loop unroll(disable)
    for (int k = nz - 1; k >= 0; k--) {
        const double lki = lnext;
        lnext = (k >= 1 && k - 1 > i) ? L[(k - 1) * nz + i] : 0.0;
        const double xk = readlane_d(b, k) * dinv[k];
        b = (i == k) ? xk : b - lki * xk;
    }
    return b;
}

// xi-vector (one entry per lane) = Z' v.  Lanes (a, d) = (4a + d) sum the X rows of state
// component d over grids >= stage(a); the quad is reduced by xor-shuffles; the U/lambda
// rows of the column's own grid are added by the d == 0 lane.
template <int NZM>
__device__ __forceinline__ double zt_mul(const Ctx &c, const double *v)
{
    const int N = c.N, nz = c.nz, C = c.C, d = c.tid & 3;
    double res = 0.0;
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
                    a0 += c.Z[(4 * k + d) * nz + a] * v[4 * k + d];
                    a1 += c.Z[(4 * (k + 1) + d) * nz + a] * v[4 * (k + 1) + d];
                }
                if (k < N) a0 += c.Z[(4 * k + d) * nz + a] * v[4 * k + d];
                acc = a0 + a1;
                if (d == 0) {
                    for (int r = 4 * N + 2 * ja; r < 4 * N + 2 * ja + 2; r++) acc += c.Z[r * nz + a] * v[r];
                } else if (d == 1) {
                    for (int r = 6 * N + C * ja; r < 6 * N + C * ja + C; r++) acc += c.Z[r * nz + a] * v[r];
                }
            } else if (d == 0) {
                acc = v[c.n - 1];
            }
        }
        acc += __shfl_xor(acc, 1, WAVE);
        acc += __shfl_xor(acc, 2, WAVE);
        // lane a' takes column a' of this round from lane 4 (a' - 16 round)
        const int src = 4 * ((c.tid - round * 16) & 15);
        const double got = __shfl(acc, src, WAVE);
        if (c.tid >= round * 16 && c.tid < round * 16 + 16) res = got;
    }
    return (c.tid < nz) ? res : 0.0;
}

// out = Z xi  (xi one entry per lane); columns of grid j reach X rows of grids >= j and
// the U/lambda rows of grid j only.
template <int NZM>
__device__ __forceinline__ void z_mul(const Ctx &c, double xi, double *out)
{
    const int N = c.N, nz = c.nz, C = c.C, n = c.n;
    if (c.tid < nz) c.xiv[c.tid] = xi;
    __syncthreads();
    const double *xs = c.xiv;                       // LDS broadcast reads
    for (int v = c.tid; v < n; v += WAVE) {
        double a0 = 0.0, a1 = 0.0;
        if (v < 4 * N) {
            const int lim = ((v >> 2) + 1) * (C - 1);     // columns of grids <= k
            int a = 0;
            for (; a + 1 < lim; a += 2) {
                a0 += c.Z[v * nz + a] * xs[a];
                a1 += c.Z[v * nz + a + 1] * xs[a + 1];
            }
            if (a < lim) a0 += c.Z[v * nz + a] * xs[a];
        } else if (v < n - 1) {
            const int j = (v < 6 * N) ? (v - 4 * N) >> 1 : (v - 6 * N) / C;
            for (int a = j * (C - 1); a < (j + 1) * (C - 1); a++) a0 += c.Z[v * nz + a] * xs[a];
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
__device__ __forceinline__ void newton_solve(const Ctx &c, const double *r1, double *r3dz)
{
    double *w = c.dsv;                      // scratch m-vector (callers recompute dsv after)
    for (int r = c.tid; r < c.m; r += WAVE) w[r] = c.om[r] * r3dz[r];
    __syncthreads();
    jt_apply(c, w, c.tv, r1, 1.0);
    const double g = zt_mul<NZM>(c, c.tv);
    const double xi = chol_solve_reg(c, c.L, c.dinv, c.nz, g);
    z_mul<NZM>(c, xi, c.dx);
    for (int r = c.tid; r < c.m; r += WAVE) r3dz[r] = c.om[r] * (row_dot(c, r, c.dx) - r3dz[r]);
    __syncthreads();
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
    STAMP_DECL
    const int sb = c.nl ? 16 : 0;       // stamp slots: QP 0..15, NLP 16..31
    for (int iter = 0; iter < maxit; iter++) {
        STAMP_BEGIN();
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
            const double l = sqrt(sr * zr), l2 = l * l;     // formlambda, lambda.*lambda
            c.l2[r] = l2; mu += l2;
            c.iz[r] = 1.0 / zr; c.is[r] = 1.0 / sr;
        }
        nrx = sqrt(wsum(nrx)); nrz = sqrt(wsum(nrz)); sz = wsum(sz); mu = wsum(mu) / c.m;
        if (c.nl) gm = wmax(gm);
        STAMP_END(sb + 0);
        if (!isfinite(nrx) || !isfinite(nrz) || !isfinite(sz)) { flag = 3; break; }
        // NLP: dual residual scaled by max(1, ||Q x + f||_inf) (QP: iSWIFT's absolute test)
        const double thx = c.nl ? th * gm : th;
        if (nrx < thx && nrz < th && sz / c.m < tol) { flag = 0; break; }
        const int pc = c.nl || (sigma > sigma_d);
        if (pc) {
            // weights W^-1 = 1/(s/z) (updatekktmatrix, Auxilary.c:197-205) and factor
            for (int r = c.tid; r < c.m; r += WAVE) c.om[r] = 1.0 / (c.s[r] / c.z[r]);
            __syncthreads();
            STAMP_END(sb + 1);
            delta = 0.0;
            double dstart = 0.0;
            int ok = 0;
            for (int tries = 0; tries < (c.nl ? 14 : 1); tries++) {
                build_D(c, delta);
                build_Hc(c, c.Hc, 0);
                STAMP_END(sb + 2);
                if (tries == 0) {       // scale-aware first shift: 1e-10 * max(1, max diag of Z'HZ)
                    double dm = 1.0;
                    for (int a = c.tid; a < c.nz; a += WAVE) dm = fmax(dm, c.Hc[a * c.nz + a]);
                    dstart = 1e-10 * wmax(dm);
                }
                int cf = chol_reg<NZM>(c, c.Hc, c.L, c.dinv, c.nz, !c.nl);
                STAMP_END(sb + 3);
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
            STAMP_END(sb + 4);
            newton_solve<NZM>(c, c.rx, c.dz);
            STAMP_END(sb + 5);
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
        STAMP_END(sb + 6);
        newton_solve<NZM>(c, c.rx, c.dz);
        STAMP_END(sb + 7);
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
        STAMP_END(sb + 8);
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

// --------------------------------------------------------------------------- main kernel
template <int NZM>
__device__ __forceinline__ void nmpc_agent(const SrbKParams &prm, int agent,
                const double *__restrict__ x0g, const double *__restrict__ refg, const double *__restrict__ footg,
                const double *__restrict__ obstacles, const int *__restrict__ obs_idx,
                const double *__restrict__ nbr_state, const int *__restrict__ nbr_idx,
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
    c.Z = p; p += n * nz;
    c.x = p; p += n; c.q = p; p += n; c.rx = p; p += n; c.dx = p; p += n; c.tv = p; p += n; c.D = p; p += n;
    c.ref = p; p += 4 * N; c.foot = p; p += 2 * C * N; c.offv = p; p += 2 * (N - 1) + 3 * N;
    c.s = p; p += mmax; c.z = p; p += mmax; c.rz = p; p += mmax; c.dz = p; p += mmax;
    c.dsv = p; p += mmax; c.dsT = p; p += mmax; c.om = p; p += mmax; c.hvec = p; p += mmax;
    c.iz = p; p += mmax; c.is = p; p += mmax; c.l2 = p; p += mmax;
    c.jc = p; p += 2 * N * K + 2; c.obs = p; p += 2 * N * K + 2; c.eps = p; p += K + 1;
    c.Hc = p; p += nz * nz; c.L = p; p += nz * nz; c.ZtZ = p; p += nz * nz; c.ZtZL = p; p += nz * nz;
    c.dinv = p; p += nz; c.ZtZdinv = p; p += nz; c.xiv = p; p += nz;

    STAMP_DECL
    STAMP_BEGIN();
    // ---- load inputs (a1/a2/a3: x0, reference window, footholds)
    const double *x0 = x0g + 4 * (size_t)agent;
    for (int i = c.tid; i < 4 * N; i += WAVE) c.ref[i] = refg[(size_t)agent * 4 * N + i];
    for (int i = c.tid; i < 2 * C * N; i += WAVE) c.foot[i] = footg[(size_t)agent * 2 * C * N + i];
    for (int i = c.tid; i < n * nz; i += WAVE) c.Z[i] = 0.0;
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
        for (int i = 0; i < C; i++) c.Z[(6 * N + C * j + i) * nz + col] = lam[i];
        c.Z[(4 * N + 2 * j) * nz + col] = g0;
        c.Z[(4 * N + 2 * j + 1) * nz + col] = g1;
        double v[4];
        for (int d = 0; d < 4; d++) v[d] = prm.Bd[d * 2] * g0 + prm.Bd[d * 2 + 1] * g1;
        for (int k = j; k < N; k++) {
            for (int d = 0; d < 4; d++) c.Z[(4 * k + d) * nz + col] = v[d];
            double tt[4];
            for (int d = 0; d < 4; d++) tt[d] = prm.Ad[d * 4] * v[0] + prm.Ad[d * 4 + 1] * v[1] + prm.Ad[d * 4 + 2] * v[2] + prm.Ad[d * 4 + 3] * v[3];
            for (int d = 0; d < 4; d++) v[d] = tt[d];
        }
    }
    if (c.tid == 0) c.Z[(n - 1) * nz + nz - 1] = 1.0;
    __syncthreads();

    STAMP_END(10);
    // One loop over the two stages so that the interior-point iteration exists once in
    // the code object (the solve is latency-bound; keeping the hot loop small keeps it in
    // the instruction cache).  stage 0: QP (iSWIFT, Prime.c:35-230); stage 1: NLP
    // (replaces SnoptSolver::Solve, MPC_dist.cpp:402-427), warm-started from stage 0.
    int qp_flag = 3, qp_it = 0, nlp_flag = 0, nlp_it = 0;
    const int nstage = prm.use_nlp ? 2 : 1;
#pragma clang loop unroll(disable)
    for (int stage = 0; stage < nstage; stage++) {
        if (stage == 0) {
            c.m = c.mq; c.nl = 0;
            for (int r = c.tid; r < c.m; r += WAVE) c.hvec[r] = row_h(c, r);
            for (int r = c.tid; r < c.m; r += WAVE) c.om[r] = 1.0;     // kkt_initialize: -I block
            __syncthreads();
            build_D(c, 0.0);
            build_Hc(c, c.Hc, 0);
            if (chol_reg<NZM>(c, c.Hc, c.L, c.dinv, nz, 1) != 0) { qp_flag = 1; continue; }
            // r1 = -c - P xbar ; r3 = h - G xbar   ->  dx ; x = xbar + dx
            for (int v = c.tid; v < n; v += WAVE) c.rx[v] = -cvec(c, v) - Pdiag(c, v) * c.x[v];
            for (int r = c.tid; r < c.m; r += WAVE) c.dz[r] = c.hvec[r] - row_dot(c, r, c.x);
            __syncthreads();
            newton_solve<NZM>(c, c.rx, c.dz);   // dz <- G x - h (z of the init system)
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
            STAMP_END(11);
        } else {
            if (x_qp_out)
                for (int v = c.tid; v < n; v += WAVE) x_qp_out[(size_t)agent * n + v] = c.x[v];
            c.nl = 1; c.m = mmax;
            // obstacles per grid: K_obs nearest static (MPC_dist.cpp:371-396; srb_knn_kernel over
            // the obstacle table) + K_nbr nearest agents predicted at constant velocity
            for (int j = 0; j < K; j++) {
                const bool st = j < prm.K_obs;
                const int bi = st ? obs_idx[(size_t)agent * prm.K_obs + j] : nbr_idx[(size_t)agent * prm.K_nbr + (j - prm.K_obs)];
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
            build_Hc(c, c.ZtZ, 1);
            chol_reg<NZM>(c, c.ZtZ, c.ZtZL, c.ZtZdinv, nz, 0);
            // v = P x + c + J'z ; rx0 = -Z (Z'Z)^-1 Z' v ; q = -v - rx0
            for (int v = c.tid; v < n; v += WAVE) c.tv[v] = Pdiag(c, v) * c.x[v] + cvec(c, v);
            __syncthreads();
            jt_apply(c, c.z, c.rx, c.tv, 1.0);
            const double g = zt_mul<NZM>(c, c.rx);
            const double t = chol_solve_reg(c, c.ZtZL, c.ZtZdinv, nz, g);
            z_mul<NZM>(c, t, c.dx);
            for (int v = c.tid; v < n; v += WAVE) c.q[v] = -c.rx[v] + c.dx[v];
            __syncthreads();
            STAMP_END(12);
        }
        int it = 0;
        const int f = ipm<NZM>(c, stage == 0 ? prm.qp_maxit : prm.nlp_maxit, &it);
        if (stage == 0) { qp_flag = f; qp_it = it; } else { nlp_flag = f; nlp_it = it; }
        STAMP_BEGIN();
    }
    if (x_qp_out && nstage == 1)
        for (int v = c.tid; v < n; v += WAVE) x_qp_out[(size_t)agent * n + v] = c.x[v];

    // ---- outputs
    for (int v = c.tid; v < n; v += WAVE) x_out[(size_t)agent * n + v] = c.x[v];
    double f = 0;
    for (int v = c.tid; v < n; v += WAVE) f += 0.5 * Pdiag(c, v) * c.x[v] * c.x[v] + cvec(c, v) * c.x[v];
    f = wsum(f);
    STAMP_END(13);
    if (c.tid == 0) {
        obj_out[agent] = f;
        status_out[2 * agent] = qp_flag; status_out[2 * agent + 1] = nlp_flag;
        iters_out[2 * agent] = qp_it; iters_out[2 * agent + 1] = nlp_it;
    }
}

#define SRB_NMPC_KERNEL(NAME, NZM)                                                                            \
    extern "C" __global__ void __launch_bounds__(WAVE) NAME(                                                   \
        SrbKParams prm, int n_agents, const double *__restrict__ x0g, const double *__restrict__ refg,          \
        const double *__restrict__ footg, const double *__restrict__ obstacles, const int *__restrict__ obs_idx, \
        const double *__restrict__ nbr_state, const int *__restrict__ nbr_idx, double *__restrict__ x_qp_out,   \
        double *__restrict__ x_out, double *__restrict__ obj_out, int *__restrict__ status_out,                 \
        int *__restrict__ iters_out)                                                                           \
    {                                                                                                          \
        extern __shared__ __attribute__((aligned(16))) double lds[];                                           \
        const int agent = blockIdx.x;                                                                          \
        if (agent >= n_agents) return;                                                                         \
        nmpc_agent<NZM>(prm, agent, x0g, refg, footg, obstacles, obs_idx, nbr_state, nbr_idx, x_qp_out, x_out, \
                        obj_out, status_out, iters_out, lds);                                                  \
    }

SRB_NMPC_KERNEL(srb_nmpc_kernel_nz16, 16)
SRB_NMPC_KERNEL(srb_nmpc_kernel_nz32, 32)
SRB_NMPC_KERNEL(srb_nmpc_kernel_nz64, 64)

// --------------------------------------------------------------------------- k nearest neighbours
// One thread per agent; table rows streamed through LDS tiles.  Order: (d^2, index)
// ascending -- the order the reference's strict-'<' argmin scan produces (MPC_dist.cpp:373-382).
// Used twice: static obstacles (table = Pobs_real columns, stride 2, no self) and other
// agents (table = get_lastState() rows, stride 4, self = agent_offset + a excluded).
// The query point is the agent's own current CoM from x0 (q[0], q[1] -- what the
// reference's scan uses, MPC_dist.cpp:366).
extern "C" __global__ void __launch_bounds__(256)
srb_knn_kernel(int n_agents, int agent_offset, const double *__restrict__ x0g, const double *__restrict__ state,
               int stride, int n_all, int K, int *__restrict__ nbr_idx)
{
    __shared__ double tile[1024 * 2];
    const int a = blockIdx.x * blockDim.x + threadIdx.x;
    const int self = (agent_offset >= 0) ? agent_offset + a : -1;
    double px = 0, py = 0;
    if (a < n_agents) { px = x0g[4 * (size_t)a]; py = x0g[4 * (size_t)a + 2]; }
    // sorted top-K in registers: fixed-size compare-swap insertion chain (no dynamic indexing)
    double bd[SRB_KNN_MAX]; int bi[SRB_KNN_MAX];
#pragma unroll
    for (int j = 0; j < SRB_KNN_MAX; j++) { bd[j] = 1e300; bi[j] = 0x7fffffff; }
    double wd = 1e300; int wi = 0x7fffffff;        // current K-th best (admission threshold)
    for (int base = 0; base < n_all; base += 1024) {
        int cnt = n_all - base < 1024 ? n_all - base : 1024;
        __syncthreads();
        for (int i = threadIdx.x; i < cnt; i += blockDim.x) {
            tile[2 * i] = state[(size_t)stride * (base + i)];
            tile[2 * i + 1] = state[(size_t)stride * (base + i) + 1];
        }
        __syncthreads();
        if (a < n_agents)
            for (int i = 0; i < cnt; i++) {
                int gi = base + i;
                double dx = px - tile[2 * i], dy = py - tile[2 * i + 1];
                double d = (gi == self) ? 1e300 : dx * dx + dy * dy;
                if (gi == self || !(d < wd || (d == wd && gi < wi))) continue;
                double cd = d; int ci = gi;
#pragma unroll
                for (int j = 0; j < SRB_KNN_MAX; j++) {
                    bool lt = (j < K) && (cd < bd[j] || (cd == bd[j] && ci < bi[j]));
                    double td = bd[j]; int ti = bi[j];
                    bd[j] = lt ? cd : td; bi[j] = lt ? ci : ti;
                    cd = lt ? td : cd; ci = lt ? ti : ci;
                }
#pragma unroll
                for (int j = 0; j < SRB_KNN_MAX; j++)
                    if (j == K - 1) { wd = bd[j]; wi = bi[j]; }
            }
    }
    if (a < n_agents)
#pragma unroll
        for (int j = 0; j < SRB_KNN_MAX; j++)
            if (j < K) nbr_idx[(size_t)a * K + j] = (bi[j] == 0x7fffffff) ? -1 : bi[j];
}
