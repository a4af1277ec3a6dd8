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
#include <type_traits>
#include "srb_kernel_params.h"

#define WAVE 64
// Barrier of the NW-wave workgroup.  NW = 1 (one agent per wave, the large-batch instances): the LDS
// accesses of one wavefront execute in issue order, so a wavefront-scope fence (no s_waitcnt) and a wave
// barrier suffice -- __syncthreads would wait for every outstanding LDS store first.  (Every SYNC site
// sits in a function templated on NW.)
// What this relies on: (1) LLVM IR -- a fence, whatever its scope, orders the thread's memory
// operations: no load or store is moved across it (an acq_rel fence is a read-write of all memory for
// alias analysis), so the ISA keeps the source order of the LDS accesses around SYNC; the wave barrier
// is IntrNoMem (a convergence point only) and is not what orders them.  (2) The AMDGPU memory model
// (LLVM AMDGPUUsage, memory model for GFX942 / GFX950): the LDS operations of one wavefront are performed
// in issue order, so a ds_read by any lane observes an earlier ds_write of the same wave without an
// s_waitcnt; the compiler still waits (lgkmcnt) before a loaded value is used.
template <int NW>
__device__ __forceinline__ void srb_sync()
{
    if constexpr (NW == 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
    } else {
        __syncthreads();
    }
}
#define SYNC() srb_sync<NW>()

#include "srb_wave.h"


// --------------------------------------------------------------------------- diagnostic stamps
// Built only with -DSRB_STAMPS (make stamps -> srbnmpc/libsrbnmpc_stamps.so): lane 0 of
// every agent accumulates s_memtime cycles per phase into registers; agent 0 adds them to
// a device buffer nothing else reads.
#ifdef SRB_STAMPS
#define SRB_NSTAMP 64
__device__ unsigned long long srb_stamp_buf[SRB_NSTAMP];
#define STAMP_DECL unsigned long long st_t0 = 0; int st_off = 0
#define STAMP_BEGIN() do { __builtin_amdgcn_sched_barrier(0); st_t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); } while (0)
#define STAMP_END(slot) do { __builtin_amdgcn_sched_barrier(0); const unsigned long long _t = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0); if (threadIdx.x == 0 && stamp_lds) atomicAdd(&stamp_lds[st_off + (slot)], _t - st_t0); st_t0 = _t; } while (0)
#define STAMP_STAGE(s) (st_off = 32 * (s))
#define STAMP_FLUSH(agent) do { SYNC(); if ((agent) == 0 && threadIdx.x < 64) atomicAdd(&srb_stamp_buf[threadIdx.x], stamp_lds[threadIdx.x]); } while (0)
#else
#define STAMP_DECL do {} while (0)
#define STAMP_BEGIN() do {} while (0)
#define STAMP_END(slot) do {} while (0)
#define STAMP_STAGE(s) do {} while (0)
#define STAMP_FLUSH(agent) do {} while (0)
#endif

// --------------------------------------------------------------------------- fp32 storage (diagnostic)
// Built only with -DSRB_DIAG_ROUND32 (make lipvar TAG=r32): every term row and every entry of the
// assembled reduced matrix rounded to fp32 where it is stored -- the arithmetic effect of storing them in fp32 with
// fp64 accumulation and the fp64 refinement (which then refines against the rounded matrix).  The LDS it would save
// buys no occupancy (config 5 is register-bound at two agents per CU), so only the accuracy is measured.
#ifdef SRB_DIAG_ROUND32
#ifndef SRB_DIAG_BUILD
#error "SRB_DIAG_ROUND32 is a diagnostic-build option"
#endif
#define R32(v) ((double)(float)(v))
#else
#define R32(v) (v)
#endif

// --------------------------------------------------------------------------- LDS bounds (diagnostic)
// Built only with -DSRB_DIAG_LDS_CHECK (make fullvar TAG=ldsck VARFLAGS=-DSRB_DIAG_LDS_CHECK):
// the indices a slot derives its LDS accesses from -- its term row, weight entry, iterate entries, obstacle and
// dual entries, exported active-set entry --, the term-row ranges of the Gram, and the carve's end against the
// size the host allocated (srb_lds_doubles) are checked, each failed check setting one bit of a workgroup
// flag; a flagged agent reports QP status 1000 + flag (never a fault: the kernel goes on).  Round 5's fold
// build read obstacle term rows past the end of R with four waves -- bit 1 here.
#ifdef SRB_DIAG_LDS_CHECK
#ifndef SRB_DIAG_BUILD
#error "SRB_DIAG_LDS_CHECK is a diagnostic-build option"
#endif
__device__ __forceinline__ int *lds_oob_flag()
{
    __shared__ int f;
    return &f;
}
#define LCK(ok, bit) do { if (!(ok)) __hip_atomic_fetch_or(lds_oob_flag(), 1 << (bit), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); } while (0)
#define LCK_INIT() do { if (threadIdx.x == 0) *lds_oob_flag() = 0; } while (0)
#define LCK_REPORT(slot) do { SYNC(); if (tid == 0 && *lds_oob_flag()) status_out[(slot)] = 1000 + *lds_oob_flag(); } while (0)
#else
#define LCK(ok, bit) do {} while (0)
#define LCK_INIT() do {} while (0)
#define LCK_REPORT(slot) do {} while (0)
#endif

// --------------------------------------------------------------------------- diagnostic trace
// Built only with -DSRB_NLPDBG (make nlpdbg -> srbnmpc/libsrbnmpc_nlpdbg.so): agent
// srb_nlp_dbg_agent records, per NLP iteration, ||rx||, its threshold, ||rz||, s'z/m, ap, ad,
// delta and sigma (8 doubles) into srb_nlp_dbg; nothing else reads it.
#ifdef SRB_NLPDBG
__device__ double srb_nlp_dbg[SRB_NLP_DBG_LEN];
__device__ int srb_nlp_dbg_agent = -1;
#define NLPDBG(it, k, v) do { if (nl && agent == srb_nlp_dbg_agent && tid == 0 && (it) < 64) srb_nlp_dbg[8 * (it) + (k)] = (v); } while (0)
// polish kernel: pass p of the traced agent into row 56 + p: primal, |c_A|, -min z_A, max |z_A|,
// max inactive violation, last |dx|, accepted, Newton steps
#define POLDBG(p, k, v) do { if (agent == srb_nlp_dbg_agent && tid == 0 && (p) < 8) srb_nlp_dbg[8 * (56 + (p)) + (k)] = (v); } while (0)
// polish kernel, first Newton step of pass 0: the reduced matrix (32 x 32 at 512) and right-hand
// side (at 512 + 1024) of the traced agent, for an eigenvalue check on the host
// and, at the polish kernel's start, the exported zpol row values (2 S at 1568) and x (at 2592)
#define POLDBG_IN(zp, S, xs, n) do { if (agent == srb_nlp_dbg_agent) { \
    for (int e = tid; e < 2 * (S) && e < 1024; e += NTH) srb_nlp_dbg[1568 + e] = (zp)[e]; \
    for (int e = tid; e < (n) && e < 256; e += NTH) srb_nlp_dbg[2592 + e] = (xs)[e]; } } while (0)
// x after each Newton step of pass 0 (3 x 256 at 2848)
#define POLDBG_X(p, it, xs, n) do { SYNC(); if (agent == srb_nlp_dbg_agent && (p) == 0 && (it) < 3) \
    for (int e = tid; e < (n) && e < 256; e += NTH) srb_nlp_dbg[2848 + 256 * (it) + e] = (xs)[e]; } while (0)
#define POLDBG_MAT(H, LDH, v, nz) do { if (agent == srb_nlp_dbg_agent) \
    for (int e = tid; e < (nz) * (nz); e += NTH) { srb_nlp_dbg[512 + 32 * (e / (nz)) + e % (nz)] = (H)[(e / (nz)) * (LDH) + e % (nz)]; \
        if (e < (nz)) srb_nlp_dbg[512 + 1024 + e] = (v)[e]; } } while (0)
#else
#define POLDBG_MAT(H, LDH, v, nz) do {} while (0)
#define POLDBG_IN(zp, S, xs, n) do {} while (0)
#define POLDBG_X(p, it, xs, n) do {} while (0)
#define NLPDBG(it, k, v) do {} while (0)
#define POLDBG(p, k, v) do {} while (0)
#endif

// --------------------------------------------------------------------------- term rows
// Term row t (Z row of a variable, M_e) at R + t * LDR; LDR = NZL + 1 (odd: lane-parallel row reads stay
// conflict-free).  Rows are zero beyond nz and beyond the count.  Row order: X rows (4N) | CoM-CoP rows |
// U, lambda, slack rows.  Reduced columns: 0 the slack, 1 + j (C - 1) + i the i-th contact-weight dof of
// grid j.
struct TermLayout {
    int N, C, n, nz, E4;
    __device__ __forceinline__ int zr(int v) const { return v < 4 * N ? v : v + E4; }
};

// Obstacle rows, folded per grid (round 5).  Row o = k K + j of grid k is M_o = J_o Z = jx Z_x + jy Z_y - e_s
// (Z_x, Z_y: the stored Z rows 4k, 4k + 2 of the grid's CoM position; OJ[2 o] = jx, OJ[2 o + 1] = jy, set
// by the re-linearisation).  With V_k = [Z_x, Z_y, e_s] and v_o = (jx, jy, -1), the K rows of a grid add
//   sum_j W_o M_o M_o' = V_k S_k V_k',  S_k = sum_j W_o v_o v_o'   and   sum_j CF_o M_o = V_k c_k,  c_k = sum_j CF_o v_o
// to the Gram and the right-hand side: 3 terms a grid instead of K rows (obs_fold forms S_k, c_k; the
// Gram's term (k, u) has A = column u of V_k, B = V_k S_k e_u).  FO holds S_k (00 01 02 11 12 22) and c_k per
// grid, 9 doubles, and a zero entry at grid N for the padding terms.
struct ObsFold {
    const double *OJ;
    double *FO;
    int rO, N, K, NOP;                 // obstacle rows' W / CF offset, grids, rows per grid, 3N padded to 16 NW
    uint64_t mask;                     // NZM = 32: grid-term batches that reach column 16 (all three tiles)
    int rU, C, n;                      // the U, lambda, slack rows (ul_add): first row, contacts, variables
};

// The U, lambda and slack rows [rU, rU + n - 4N) touch only their own grid's C - 1 columns (the slack row
// column 0), so their part of the Gram is block diagonal: H[a][b] += sum_r W_r R[r][a] R[r][b] over the
// 2 + C rows of grid j for a, b in grid j's columns (and W_s at [0][0]), g[a] += sum_r CF_r R[r][a] --
// added directly instead of as MFMA batches of single-entry rows (configs[2] Gram 14 -> 11 batches,
// N = 20 14 + 4 -> 8 + 4).  Lanes tid0, tid0 + step, .. of the caller; after its tile stores.
template <int NZL, bool GRAM, bool RHS>
__device__ __forceinline__ void ul_add(const double *R, const double *W, const double *CF, const ObsFold &F, double *H,
                                       double *g, int nz, int tid0, int step)
{
    constexpr int LDR = NZL + 1, LDH = NZL + 1;
    const int c1 = F.C - 1, np = F.N * c1 * c1, rl = F.rU + 2 * F.N, rs = F.rU + F.n - 1 - 4 * F.N;
    if (GRAM) {
        for (int e = tid0; e <= np; e += step) {
            if (e == np) { H[0] = R32(H[0] + W[rs]); continue; }  // slack row: Z = e_0
            const int j = e / (c1 * c1), rem = e - j * c1 * c1, a = 1 + j * c1 + rem / c1, b = 1 + j * c1 + rem % c1;
            double v = 0.0;
            for (int d = 0; d < 2; d++) { const int r = F.rU + 2 * j + d; v = fma(W[r] * R[r * LDR + a], R[r * LDR + b], v); }
            for (int i = 0; i < F.C; i++) { const int r = rl + F.C * j + i; v = fma(W[r] * R[r * LDR + a], R[r * LDR + b], v); }
            H[a * LDH + b] = R32(H[a * LDH + b] + v);
        }
    }
    if (RHS) {
        for (int a = tid0; a < nz; a += step) {
            if (a == 0) { g[0] += CF[rs]; continue; }
            const int j = (a - 1) / c1;
            double v = 0.0;
            for (int d = 0; d < 2; d++) { const int r = F.rU + 2 * j + d; v = fma(CF[r], R[r * LDR + a], v); }
            for (int i = 0; i < F.C; i++) { const int r = rl + F.C * j + i; v = fma(CF[r], R[r * LDR + a], v); }
            g[a] += v;
        }
    }
}

// S_k and c_k (GRAM) or c_k alone into FO: one lane per grid, the K rows in index order
template <bool GRAM>
__device__ __forceinline__ void obs_fold(const double *W, const double *CF, const ObsFold &F, int tid, int NTH)
{
    for (int k = tid; k < F.N; k += NTH) {
        double s00 = 0.0, s01 = 0.0, s02 = 0.0, s11 = 0.0, s12 = 0.0, s22 = 0.0, c0 = 0.0, c1 = 0.0, c2 = 0.0;
        // the grid's rows in chunks of 8, every load of a chunk issued before the first use (predicated, as
        // zo_sum): one LDS round trip a chunk instead of one a row; the sums keep the row order
        for (int j0 = 0; j0 < F.K; j0 += 8) {
            double cfv[8], jxv[8], jyv[8], wv[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const bool in = j0 + u < F.K;
                const int o = k * F.K + (in ? j0 + u : 0);
                cfv[u] = in ? CF[F.rO + o] : 0.0; jxv[u] = in ? F.OJ[2 * o] : 0.0; jyv[u] = in ? F.OJ[2 * o + 1] : 0.0;
                wv[u] = (GRAM && in) ? W[F.rO + o] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 8; u++) {
                if (j0 + u >= F.K) break;
                const double cf = cfv[u], jx = jxv[u], jy = jyv[u];
                c0 = fma(cf, jx, c0); c1 = fma(cf, jy, c1); c2 -= cf;
                if (GRAM) {
                    const double w = wv[u], wx = w * jx, wy = w * jy;
                    s00 = fma(wx, jx, s00); s01 = fma(wx, jy, s01); s02 -= wx; s11 = fma(wy, jy, s11); s12 -= wy; s22 += w;
                }
            }
        }
        double *f = F.FO + 9 * k;
        if (GRAM) { f[0] = s00; f[1] = s01; f[2] = s02; f[3] = s11; f[4] = s12; f[5] = s22; }
        f[6] = c0; f[7] = c1; f[8] = c2;
    }
}

// Highest reduced column term row t (t < rO) touches: X rows of grid k reach grid k, a CoM-CoP row of grid i
// grid i + 1, U / lambda rows their own grid.  With NZM = 32 a batch of 16 terms whose rows all stop below
// column 16 needs the (0,0) tile only (gram_rhs, rhs_only; `bmask` bit b = batch b needs all three; the
// obstacle grid terms likewise in ObsFold::mask).
__device__ __forceinline__ int term_maxcol(int t, int N, int C, int n, int rC, int NE, int rU)
{
    const int c1 = C - 1;
    if (t < rC) return (t / 4 + 1) * c1;
    if (t < rC + NE) return ((t - rC) / 2 + 2) * c1;
    if (t < rU) return 0;
    const int v = 4 * N + (t - rU);
    if (v < 6 * N) return ((v - 4 * N) / 2 + 1) * c1;
    if (v < n - 1) return ((v - 6 * N) / C + 1) * c1;
    return 0;                                                    // slack row (column 0), padding
}

template <int NZM>
__device__ __forceinline__ uint64_t full_batches(int rO, int N, int C, int n, int rC, int NE, int rU, int lane)
{
    if constexpr (NZM == 16) return ~0ull;
    int f = 0;
    if (16 * lane < rO) {
        int mx = 0;
        for (int u = 0; u < 16; u++) mx = max(mx, term_maxcol(16 * lane + u, N, C, n, rC, NE, rU));
        f = mx >= 16;
    }
    return __ballot(f) | ((rO > 16 * 64) ? (1ull << 63) : 0ull);   /* (more than 64 batches: the last bit covers the rest) */
}

template <int NZM>
__device__ __forceinline__ uint64_t full_obs_batches(int N, int C, int NOP, int lane)
{
    if constexpr (NZM == 16) return ~0ull;
    const int kmax = min((16 * lane + 15) / 3, N - 1);
    return __ballot(16 * lane < NOP && (kmax + 1) * (C - 1) >= 16) | ((NOP > 16 * 64) ? (1ull << 63) : 0ull);
}

__device__ __forceinline__ bool batch_full(uint64_t bmask, int t0)
{
    const int b = t0 >> 4;
    return (bmask >> (b < 63 ? b : 63)) & 1ull;
}

// element `col` of stored term row r
template <int NZL>
__device__ __forceinline__ double term_elem(const double *R, int r, int col)
{
    constexpr int LDR = NZL + 1;
    return (col < NZL) ? R[r * LDR + col] : 0.0;
}

// obstacle grid term t = 3 k + u: A element (column u of V_k) for column col, and the row of S_k / entry of
// c_k it pairs with (padding terms: grid N, all zero)
template <int NZL>
__device__ __forceinline__ double obs_term_a(const double *R, const ObsFold &F, int t, int col, double &zx, double &zy)
{
    constexpr int LDR = NZL + 1;
    const int k = t / 3, u = t - 3 * k, xr = 4 * min(k, F.N - 1);
    zx = (col < NZL) ? R[xr * LDR + col] : 0.0;
    zy = (col < NZL) ? R[(xr + 2) * LDR + col] : 0.0;
    const double es = (col == 0) ? 1.0 : 0.0;
    return (u == 0) ? zx : (u == 1) ? zy : es;
}

// GRAM: H = sum_t W_t r_t r_t' over the stored term rows [0, cnt) plus the folded obstacle grid terms
//   [0, NOP) (when nko > 0, the NLP stage): v_mfma_f64_16x16x4f64 with A[a][k] = r_{t0+k}[a],
//   B[k][b] = W_{t0+k} r_{t0+k}[b] (grid terms: B = V_k S_k e_u); lane l supplies term t0 + (l >> 4),
//   column l & 15; D layout row (l >> 4) + 4 q, column l & 15; NZM = 32: tiles (0,0), (0,1), (1,1).  Four
//   term groups per batch: every operand load of the batch issues before the first MFMA waits on one.
// RHS: g[a] = sum_t CF_t r_t[a]: the very element lane l forms for the MFMA is the one its (column, term)
//   pair needs, so the right-hand side costs one FMA per element; the four term chunks combine by permlane
//   swaps.
// cnt and NOP are multiples of 16 NW; W / CF are zero beyond every real row.
// NW > 1: wave w takes the w-th NW-th of both ranges; the per-wave partial tiles / right-hand sides are
// summed through LDS (`part`: NW x NT x 256 + NW x NZM doubles).
template <int NZL, bool RHS, int NW>
__device__ __forceinline__ void gram_rhs(const double *R, const double *W, const double *CF, int cnt, const ObsFold &F,
                                         int nko, double *H, double *g, int nz, int tid, double *part, uint64_t bmask)
{
    constexpr int NZM = ((NZL + 15) / 16) * 16;
    constexpr int LDH = NZL + 1;            // H holds rows / columns < NZL only (the rest of the tiles are 0)
    constexpr int NT = (NZM == 16) ? 1 : 3, NTC = NZM / 16;
    const int lane = tid & 63, wv = tid >> 6;
    const int li = lane & 15, kq = lane >> 4;
    constexpr bool FOLD = !SRB_OBS_STORED(NZL);
    if (FOLD && nko > 0) {
        obs_fold<true>(W, CF, F, tid, 64 * NW);
        srb_sync<NW>();
    }
    d4 acc[NT];
    double ps[NTC];
#pragma unroll
    for (int t = 0; t < NT; t++) acc[t] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int t = 0; t < NTC; t++) ps[t] = 0.0;
    // FULL: all NTC column blocks; otherwise block 0 only (every row of the batch is zero beyond column 15)
    auto body = [&](int t0, auto fullc) {
        constexpr bool FULL = decltype(fullc)::value;
        constexpr int NB = FULL ? NTC : 1;
        double a[4][NTC], w[4], c[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int r = t0 + 4 * u + kq;
#pragma unroll
            for (int tc = 0; tc < NB; tc++) a[u][tc] = term_elem<NZL>(R, r, 16 * tc + li);
            w[u] = W[r];
            c[u] = RHS ? CF[r] : 0.0;
        }
        __builtin_amdgcn_sched_barrier(0);     // keep the batch's loads ahead of its MFMAs
#pragma unroll
        for (int u = 0; u < 4; u++) {
            if (RHS)
#pragma unroll
                for (int tc = 0; tc < NB; tc++) ps[tc] = fma(c[u], a[u][tc], ps[tc]);
            if constexpr (NZM == 16 || !FULL) {
                acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u][0], w[u] * a[u][0], acc[0], 0, 0, 0);
            } else {
                acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u][0], w[u] * a[u][0], acc[0], 0, 0, 0);
                acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u][0], w[u] * a[u][NTC - 1], acc[1], 0, 0, 0);
                acc[2] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u][NTC - 1], w[u] * a[u][NTC - 1], acc[2], 0, 0, 0);
            }
        }
    };
    // folded obstacle grid terms t0 .. t0 + 15
    auto obody = [&](int t0, auto fullc) {
        constexpr bool FULL = decltype(fullc)::value;
        constexpr int NB = FULL ? NTC : 1;
        double a[4][NTC], b[4][NTC], c[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int t = t0 + 4 * u + kq, k = t / 3, uu = t - 3 * k;
            const double *f = F.FO + 9 * min(k, F.N);
            const int i1 = (uu == 0) ? 1 : (uu == 1) ? 3 : 4, i2 = (uu == 0) ? 2 : (uu == 1) ? 4 : 5;
            const double s0 = f[uu], s1 = f[i1], s2 = f[i2];
            c[u] = RHS ? f[6 + uu] : 0.0;
#pragma unroll
            for (int tc = 0; tc < NB; tc++) {
                double zx, zy;
                a[u][tc] = obs_term_a<NZL>(R, F, t, 16 * tc + li, zx, zy);
                b[u][tc] = fma(s0, zx, fma(s1, zy, (16 * tc + li == 0) ? s2 : 0.0));
            }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < 4; u++) {
            if (RHS)
#pragma unroll
                for (int tc = 0; tc < NB; tc++) ps[tc] = fma(c[u], a[u][tc], ps[tc]);
            if constexpr (NZM == 16 || !FULL) {
                acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u][0], b[u][0], acc[0], 0, 0, 0);
            } else {
                acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u][0], b[u][0], acc[0], 0, 0, 0);
                acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u][0], b[u][NTC - 1], acc[1], 0, 0, 0);
                acc[2] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u][NTC - 1], b[u][NTC - 1], acc[2], 0, 0, 0);
            }
        }
    };
    {
        // NZM = 32 with several waves: the batches dealt round-robin over the waves (the full-width ones
        // cluster at high grids, so contiguous halves left one wave with most of them); else contiguous
        constexpr bool ILV = NZM == 32 && NW > 1;
        const int chunk = cnt / NW, tb = ILV ? 16 * wv : wv * chunk, te = ILV ? cnt : tb + chunk, ts = ILV ? 16 * NW : 16;
#pragma clang loop unroll(disable)
        for (int t0 = tb; t0 < te; t0 += ts) {
            if (NZM == 16 || batch_full(bmask, t0)) body(t0, std::integral_constant<bool, true>{});
            else body(t0, std::integral_constant<bool, false>{});
        }
        if (FOLD && nko > 0) {
            const int och = F.NOP / NW, ob = ILV ? 16 * wv : wv * och, oe = ILV ? F.NOP : ob + och;
#pragma clang loop unroll(disable)
            for (int t0 = ob; t0 < oe; t0 += ts) {
                if (NZM == 16 || batch_full(F.mask, t0)) obody(t0, std::integral_constant<bool, true>{});
                else obody(t0, std::integral_constant<bool, false>{});
            }
        } else if (nko > 0) {                       // stored obstacle rows [rO, rO + nko)
            const int och = nko / NW, ob = F.rO + wv * och;
#pragma clang loop unroll(disable)
            for (int t0 = ob; t0 < ob + och; t0 += 16) body(t0, std::integral_constant<bool, true>{});
        }
    }
    double gs[NTC];
    if (RHS)
#pragma unroll
        for (int tc = 0; tc < NTC; tc++) gs[tc] = chunk_sum16(ps[tc]);
    if constexpr (NW <= 2) {
        // wave 0 stores its tiles; with two waves, wave 1 then adds its own in place (a fixed
        // order: bit-reproducible, and no partial-Gram scratch in LDS)
        auto put = [&](int i, int j, double v, bool add) {
            if (i < NZL && j < NZL) H[i * LDH + j] = R32(add ? H[i * LDH + j] + v : v);
        };
#pragma unroll
        for (int ph = 0; ph < NW; ph++) {
            if (ph > 0) __syncthreads();
            if (wv == ph) {
                if (RHS)
#pragma unroll
                    for (int tc = 0; tc < NTC; tc++)
                        if (kq == 0 && 16 * tc + li < nz) g[16 * tc + li] = ph ? g[16 * tc + li] + gs[tc] : gs[tc];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int r = kq + 4 * q;
                    put(r, li, acc[0][q], ph > 0);
                    if constexpr (NZM == 32) {
                        put(r, 16 + li, acc[1][q], ph > 0);
                        put(16 + li, r, acc[1][q], ph > 0);
                        put(16 + r, 16 + li, acc[2][q], ph > 0);
                    }
                }
                if (ph == NW - 1) ul_add<NZL, true, RHS>(R, W, CF, F, H, g, nz, lane, 64);   /* (same wave, after its stores) */
            }
        }
    } else {
        double *pg = part + NW * NT * 256;
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int q = 0; q < 4; q++) part[((wv * NT + t) * 4 + q) * 64 + lane] = acc[t][q];
        if (RHS)
#pragma unroll
            for (int tc = 0; tc < NTC; tc++)
                if (kq == 0) pg[wv * NZM + 16 * tc + li] = gs[tc];
        __syncthreads();
        for (int e = tid; e < NT * 256; e += 64 * NW) {
            const int t = e >> 8, q = (e >> 6) & 3, ln = e & 63;
            double v = 0.0;
#pragma unroll
            for (int w2 = 0; w2 < NW; w2++) v += part[((w2 * NT + t) * 4 + q) * 64 + ln];
            const int r = (ln >> 4) + 4 * q, cl = ln & 15;
            v = R32(v);
            if (t == 0) { if (r < NZL && cl < NZL) H[r * LDH + cl] = v; }
            else if (t == 1) { if (16 + cl < NZL) { H[r * LDH + 16 + cl] = v; H[(16 + cl) * LDH + r] = v; } }
            else if (16 + r < NZL && 16 + cl < NZL) H[(16 + r) * LDH + 16 + cl] = v;
        }
        if (RHS && tid < nz) {
            double v = 0.0;
#pragma unroll
            for (int w2 = 0; w2 < NW; w2++) v += pg[w2 * NZM + tid];
            g[tid] = v;
        }
        __syncthreads();
        ul_add<NZL, true, RHS>(R, W, CF, F, H, g, nz, tid, 64 * NW);
    }
}

// g[a] = sum_t CF_t r_t[a] alone (corrector): same lane mapping and term ranges as gram_rhs (c_k refolded,
// S_k kept), eight term groups per batch so that 16 loads are in flight before the FMAs need them.
template <int NZL, int NW>
__device__ __forceinline__ void rhs_only(const double *R, const double *CF, int cnt, const ObsFold &F, int nko, double *g,
                                         int nz, int tid, double *part, uint64_t bmask)
{
    constexpr int NZM = ((NZL + 15) / 16) * 16;
    constexpr int NTC = NZM / 16;
    const int lane = tid & 63, wv = tid >> 6;
    const int li = lane & 15, kq = lane >> 4;
    constexpr bool FOLD = !SRB_OBS_STORED(NZL);
    if (FOLD && nko > 0) {
        obs_fold<false>(nullptr, CF, F, tid, 64 * NW);
        srb_sync<NW>();
    }
    double ps[2][NTC];
#pragma unroll
    for (int t = 0; t < NTC; t++) { ps[0][t] = 0.0; ps[1][t] = 0.0; }
    auto chunk32 = [&](int t0, auto fullc) {
        constexpr int NB = decltype(fullc)::value ? NTC : 1;
        double a[8][NTC], c[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int r = t0 + 4 * u + kq;
            c[u] = CF[r];
#pragma unroll
            for (int tc = 0; tc < NB; tc++) a[u][tc] = term_elem<NZL>(R, r, 16 * tc + li);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < 8; u++)
#pragma unroll
            for (int tc = 0; tc < NB; tc++) ps[u & 1][tc] = fma(c[u], a[u][tc], ps[u & 1][tc]);
    };
    auto schunk16 = [&](int t0, auto fullc) {          // stored rows t0 .. t0 + 15
        constexpr int NB = decltype(fullc)::value ? NTC : 1;
        double a[4][NTC], c[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int r = t0 + 4 * u + kq;
            c[u] = CF[r];
#pragma unroll
            for (int tc = 0; tc < NB; tc++) a[u][tc] = term_elem<NZL>(R, r, 16 * tc + li);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < 4; u++)
#pragma unroll
            for (int tc = 0; tc < NB; tc++) ps[u & 1][tc] = fma(c[u], a[u][tc], ps[u & 1][tc]);
    };
    auto ochunk16 = [&](int t0, auto fullc) {
        constexpr int NB = decltype(fullc)::value ? NTC : 1;
        double a[4][NTC], c[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int t = t0 + 4 * u + kq, k = t / 3, uu = t - 3 * k;
            c[u] = F.FO[9 * min(k, F.N) + 6 + uu];
#pragma unroll
            for (int tc = 0; tc < NB; tc++) {
                double zx, zy;
                a[u][tc] = obs_term_a<NZL>(R, F, t, 16 * tc + li, zx, zy);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < 4; u++)
#pragma unroll
            for (int tc = 0; tc < NB; tc++) ps[u & 1][tc] = fma(c[u], a[u][tc], ps[u & 1][tc]);
    };
    auto range = [&](int tb, int te, bool st) {     // stored rows [tb, te) (st: the stored obstacle rows)
        int t0 = tb;
#pragma clang loop unroll(disable)
        for (; t0 + 32 <= te; t0 += 32) {
            if (NZM == 16 || st || batch_full(bmask, t0) || batch_full(bmask, t0 + 16))
                chunk32(t0, std::integral_constant<bool, true>{});
            else
                chunk32(t0, std::integral_constant<bool, false>{});
        }
#pragma clang loop unroll(disable)
        for (; t0 < te; t0 += 4) {
            const int r = t0 + kq;
            const double cc = CF[r];
#pragma unroll
            for (int tc = 0; tc < NTC; tc++) ps[0][tc] = fma(cc, term_elem<NZL>(R, r, 16 * tc + li), ps[0][tc]);
        }
    };
    {
        constexpr bool ILV = NZM == 32 && NW > 1;       // batches round-robin over the waves, as gram_rhs
        const int chunk = cnt / NW, tb = wv * chunk;
        if constexpr (ILV) {
#pragma clang loop unroll(disable)
            for (int t0 = 16 * wv; t0 < cnt; t0 += 16 * NW) {
                if (batch_full(bmask, t0)) schunk16(t0, std::integral_constant<bool, true>{});
                else schunk16(t0, std::integral_constant<bool, false>{});
            }
        } else {
            range(tb, tb + chunk, false);
        }
        if (!FOLD && nko > 0) {
            const int och = nko / NW, ob = F.rO + wv * och;
            range(ob, ob + och, true);
        }
        if (FOLD && nko > 0) {
            const int och = F.NOP / NW, ob = ILV ? 16 * wv : wv * och, oe = ILV ? F.NOP : ob + och, os = ILV ? 16 * NW : 16;
#pragma clang loop unroll(disable)
            for (int o0 = ob; o0 < oe; o0 += os) {
                if (NZM == 16 || batch_full(F.mask, o0)) ochunk16(o0, std::integral_constant<bool, true>{});
                else ochunk16(o0, std::integral_constant<bool, false>{});
            }
        }
    }
    double sv[NTC];
#pragma unroll
    for (int tc = 0; tc < NTC; tc++) sv[tc] = chunk_sum16(ps[0][tc] + ps[1][tc]);
    if constexpr (NW <= 2) {
#pragma unroll
        for (int ph = 0; ph < NW; ph++) {       // wave 0 stores, wave 1 adds (as gram_rhs)
            if (ph > 0) __syncthreads();
            if (wv == ph) {
#pragma unroll
                for (int tc = 0; tc < NTC; tc++)
                    if (kq == 0 && 16 * tc + li < nz) g[16 * tc + li] = ph ? g[16 * tc + li] + sv[tc] : sv[tc];
                if (ph == NW - 1) ul_add<NZL, false, true>(R, nullptr, CF, F, nullptr, g, nz, lane, 64);
            }
        }
    } else {
#pragma unroll
        for (int tc = 0; tc < NTC; tc++)
            if (kq == 0) part[wv * NZM + 16 * tc + li] = sv[tc];
        __syncthreads();
        if (tid < nz) {
            double v = 0.0;
#pragma unroll
            for (int w2 = 0; w2 < NW; w2++) v += part[w2 * NZM + tid];
            g[tid] = v;
        }
        __syncthreads();
        ul_add<NZL, false, true>(R, nullptr, CF, F, nullptr, g, nz, tid, 64 * NW);
    }
}

// Re-linearisation of obstacle row o at x: J_o = (jx, jy, -1) on (p_x(k), p_y(k), slack).  Stored-row
// instances (SRB_OBS_STORED(NZL)) materialise its term row in R, M_o = jx Z_x(k) + jy Z_y(k) - e_s
// (i0 = 4k, i1 = 4k + 2: the grid's CoM rows); the others keep (jx, jy) in OJ for the fold (ObsFold)
template <int NZL>
__device__ __forceinline__ void obs_relin(double *R, double *OJ, int rO, int o, int i0, int i1, double jx, double jy)
{
    if constexpr (SRB_OBS_STORED(NZL)) {
        constexpr int LDR = NZL + 1;
        double *dst = R + (rO + o) * LDR;
        const double *zx = R + i0 * LDR, *zy = R + i1 * LDR;
#pragma unroll
        for (int a = 0; a < NZL; a++) dst[a] = R32(fma(jx, zx[a], fma(jy, zy[a], (a == 0) ? -1.0 : 0.0)));
    } else {
        OJ[2 * o] = jx; OJ[2 * o + 1] = jy;
    }
}

// dot of LDS term row (lane-parallel rows) with a wave-uniform vector held in registers
template <int NZL, int NZE = NZL>
__device__ __forceinline__ double row_dot(const double *row, const double (&v)[NZL])
{
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int j = 0; j + 1 < NZE; j += 2) { s0 = fma(row[j], v[j], s0); s1 = fma(row[j + 1], v[j + 1], s1); }
    if (NZE & 1) s0 = fma(row[NZE - 1], v[NZE - 1], s0);
    return s0 + s1;
}

// row of the reduced matrix a lane holds: lane (NZL > 16, readlane Gauss-Jordan) or lane & 15
// (NZL <= 16: every 16-lane row of the wave holds the whole matrix, DPP broadcasts)
template <int NZL>
__device__ __forceinline__ int mrow(int lane) { return (NZL <= 16 && SRB_USE_DPP) ? (lane & 15) : lane; }

// lane i (< NZL) loads row i of H (+ delta * Z'Z) with identity padding
template <int NZL, int NZE = NZL>
__device__ __forceinline__ void gj_load(double (&A)[NZL], const double *H, const double *ZtZ, double delta, int nz, int lane)
{
    constexpr int LDH = NZL + 1;
    lane = mrow<NZL>(lane);
    const int i = (lane < NZL) ? lane : 0;
#pragma unroll
    for (int j = 0; j < NZL; j++) {
        if (j >= NZE) { A[j] = (lane == j) ? 1.0 : 0.0; continue; }
        double v = H[i * LDH + j];
        if (delta != 0.0) v = fma(delta, ZtZ[i * LDH + j], v);
        A[j] = (lane < nz && j < nz) ? v : ((lane == j) ? 1.0 : 0.0);
    }
}

// Inverse of the reduced Newton matrix (replicated layout from gj_load): gj_invert.  The
// column-split elimination (gj_invert_split, -DSRB_GJ_SPLIT=1) is bit-identical and issues
// fewer cross-lane moves, but measured slower on MI355X (configs[2] kernel 0.42 vs 0.40 ms,
// configs[1] 0.244 vs 0.206 ms; profiles/r02_gj_split_ab.txt): column k reaches the other
// rows of the wave through two permlane-swap stages on every step's critical path.
#ifndef SRB_GJ_SPLIT
#define SRB_GJ_SPLIT 0
#endif
#if SRB_GJ_SPLIT
template <int NZL, int NZE = NZL>
__device__ __forceinline__ int gj_reduced(double (&A)[NZL], int nz, int lane, int regularise)
{
    if constexpr (NZL <= 16 && NZL % 4 == 0 && SRB_USE_DPP && !SRB_KKT_FP32)
        return gj_invert_split<NZL>(A, lane, regularise);
    else
        return gj_invert<NZL, NZE>(A, nz, lane, regularise);
}
#else
#define gj_reduced gj_invert
#endif

// Newton solve in the reduced space: out = (Hs + dl Zs)^-1 g with one step of iterative refinement
// (y = M g; y += M (g - Hs y)): the explicit inverse alone is not backward stable, and near
// the end of an interior-point solve Hs carries barrier weights of 1e8..1e12.
// g, y, r, out: LDS vectors (zero beyond nz).  Returns out in registers (uniform).
// KF (the fp32-factor instances, configs[4] "fp32 KKT with fp64 iterative-refine residuals"): `nref` steps of
// refinement instead of SRB_REFINE, run-time (more while M is the fp32 inverse); the product instances (KF = 0)
// keep the compile-time count and are unchanged.
template <int NZL, int NW, int NZE = NZL, int KF = 0>
__device__ __forceinline__ void la_solve(const double (&M)[NZL], const double *Hs, const double *Zs, double dl, const double *g,
                                         double *y, double *r, double *out, double (&res)[NZL], int nz, int lane, int nref = SRB_REFINE)
{
    constexpr int LDH = NZL + 1;
    if constexpr (NZL <= 16 && SRB_USE_DPP) {
        // rows replicated per 16-lane row: the three vector broadcasts are DPP moves, no LDS
        // round trip or barrier
        const int i = lane & 15;
        const double gi = (i < nz) ? g[i] : 0.0;         // g is zero beyond nz
        double y0 = 0.0;
#pragma unroll
        for (int j = 0; j < NZE; j++) y0 = fma(M[j], bc16(gi, j), y0);
        // SRB_REFINE steps of iterative refinement with fp64 residuals (1 in the product build;
        // the fp32-factor diagnostic build uses more)
        double y1 = y0;
        const int nr = KF ? nref : SRB_REFINE;
#pragma unroll
        for (int it = 0; it < (KF ? 8 : SRB_REFINE); it++) {
            if (KF && it >= nr) break;
            double rr = gi;
            if (dl != 0.0) {                 // the NLP's inertia shift, applied on the fly (H stays unshifted)
#pragma unroll
                for (int j = 0; j < NZE; j++) rr = fma(-fma(dl, Zs[i * LDH + j], Hs[i * LDH + j]), bc16(y1, j), rr);
            } else {
#pragma unroll
                for (int j = 0; j < NZE; j++) rr = fma(-Hs[i * LDH + j], bc16(y1, j), rr);
            }
            if (i >= nz) rr = 0.0;
#pragma unroll
            for (int j = 0; j < NZE; j++) y1 = fma(M[j], bc16(rr, j), y1);
        }
#pragma unroll
        for (int j = 0; j < NZL; j++) res[j] = (j < NZE) ? bc16(y1, j) : 0.0;
        return;
    }
    const int i = (lane < NZL) ? lane : 0;
    double gv[NZL];
#pragma unroll
    for (int j = 0; j < NZE; j++) gv[j] = g[j];
    double y0 = 0.0;
#pragma unroll
    for (int j = 0; j < NZE; j++) y0 = fma(M[j], gv[j], y0);
    double y1 = y0;
    const int nr = KF ? nref : SRB_REFINE;
    for (int it = 0; it < nr; it++) {
        if (it > 0) SYNC();                      // every lane has read the previous r
        if (lane < nz) y[lane] = y1;
        SYNC();
        double rr = (lane < nz) ? g[lane] : 0.0;
        if (dl != 0.0) {
#pragma unroll
            for (int j = 0; j < NZE; j++) rr = fma(-fma(dl, Zs[i * LDH + j], Hs[i * LDH + j]), y[j], rr);
        } else {
#pragma unroll
            for (int j = 0; j < NZE; j++) rr = fma(-Hs[i * LDH + j], y[j], rr);
        }
        if (lane < nz) r[lane] = rr;
        SYNC();
#pragma unroll
        for (int j = 0; j < NZE; j++) y1 = fma(M[j], r[j], y1);
    }
    if (lane < nz) out[lane] = y1;
    SYNC();
#pragma unroll
    for (int j = 0; j < NZL; j++) res[j] = (j < NZE) ? out[j] : 0.0;
}

// --------------------------------------------------------------------------- null space
// Basis of the per-grid contact-weight directions {d : 1'd = 0} (lambda = e_{C-1} + N xi).
// Columns e_i - e_{C-1}, except for C = 4, where one column is replaced by the exact null
// vector n of [F; 1'] (u = F lambda unchanged): its U and X parts are identically zero, so
// the vanishing curvature along it near convergence (both lambda bounds inactive) is held
// exactly in Z'HZ instead of emerging from cancellation between O(1e3) terms.
// Returns 1 when column t is that null column (lam holds it), 0 otherwise.
// (every index into lam / nvec is a compile-time constant after unrolling: a runtime index would put
// these arrays in scratch memory, 48 B per lane written back to HBM by every launch)
__device__ __forceinline__ int lambda_basis(const double *F, int C, int t, double (&lam)[4])
{
    if (C != 4) {
#pragma unroll
        for (int i = 0; i < 4; i++) lam[i] = (i == t) ? 1.0 : (i == C - 1) ? -1.0 : 0.0;
        return 0;
    }
    double nvec[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int c0 = (i == 0) ? 1 : 0, c1 = (i <= 1) ? 2 : 1, c2 = (i <= 2) ? 3 : 2;
        const double *r0 = F, *r1 = F + 4;
        double det = r0[c0] * (r1[c1] - r1[c2]) - r0[c1] * (r1[c0] - r1[c2]) + r0[c2] * (r1[c0] - r1[c1]);
        nvec[i] = (i & 1) ? -det : det;
    }
    int istar = 0;
    if (fabs(nvec[1]) > fabs(nvec[istar])) istar = 1;
    if (fabs(nvec[2]) > fabs(istar == 1 ? nvec[1] : nvec[0])) istar = 2;
    const double sc = 1.0 / (istar == 0 ? nvec[0] : istar == 1 ? nvec[1] : nvec[2]);
    if (t == 2) {
#pragma unroll
        for (int i = 0; i < 4; i++) lam[i] = nvec[i] * sc;
        return 1;
    }
    const int ii = (t < istar) ? t : t + 1;
#pragma unroll
    for (int j = 0; j < 4; j++) lam[j] = (j == ii) ? 1.0 : (j == 3) ? -1.0 : 0.0;
    return 0;
}

// --------------------------------------------------------------------------- slots
// Every inequality row of the problem belongs to a SLOT: a bound pair on one scalar
// function f of x (row 0: f <= h0, row 1: -f <= h1; a single row has row 1 off) whose
// Jacobian, reduced by Z, is one term row of R.  Slot s lives in registers of lane s % 64
// (trip s / 64) for the whole solve.  Kinds, in slot order:
//   VAR  s in [0, n):            f = x_v (v = s), box +-1e3 on X/U, [0, 1] on lambda, none on
//                                the slack; also carries rx_v, P_v, c_v; term row v (Z row)
//   COP  [n, n + 2(N-1)):        f = p_i - u_{i+1}, +-mu h / sqrt 2; term row M_e
//   VEL  [.., + 2N) (NLP):       f = xdot_k / ydot_k, +-vsat; adds into term row v
//   OBS  [.., + N K) (NLP):      f = -|p_k - o_kj|^2 - s, single row <= -eps_j; term row M_o
// so residuals, Newton rows, step lengths and updates are one straight-line code path.
enum { K_NONE = 0, K_VAR = 1, K_COP = 2, K_VEL = 3, K_OBS = 4 };

struct Slot {
    double s[2], z[2], iz[2], is[2], dz[2], ds[2], dsT[2], r3[2];
    double h[2];        // row bounds
    double a0, a1, rx;  // VAR: P_v, c_v ; OBS: o_x, o_y
    double jd;          // J dx of the latest Newton solve (VAR: dx_v)
    double m[2];        // 1.0 / 0.0: row active in the current stage (arithmetic masks keep
                        // per-lane flags in VGPRs instead of long-lived SGPR lane masks)
    int i0, i1, r;      // xs indices of f, term row
    int wr;             // row this slot stores W / CF to (a scratch entry for VEL / unused slots)
    int kind;
};

// kind read through an opaque copy: comparisons on it are recomputed at each use instead
// of being hoisted into lane masks that stay live across the whole iteration
__device__ __forceinline__ int kind_of(const Slot &q)
{
    int k = q.kind;
    asm volatile("" : "+v"(k));
    return k;
}

__device__ __forceinline__ double slot_f(const Slot &q, const double *xs, double s_var)
{
    const double x0 = xs[q.i0], x1 = xs[q.i1];
    const int k = kind_of(q);
    const double dx = x0 - q.a0, dy = x1 - q.a1;
    return (k == K_OBS) ? -(dx * dx + dy * dy) - s_var : (k == K_COP) ? x0 - x1 : x0;
}



// sum_j z_kj over the K obstacle rows of grid k (zo, LDS), in index order: unrolled in chunks of
// 16 with predicated loads, so the loads of a chunk are in flight together instead of one
// dependent load per row
__device__ __forceinline__ double zo_sum(const double *zo, int k, int K)
{
    const double *z = zo + k * K;
    double s = 0.0;
    for (int j0 = 0; j0 < K; j0 += 16) {
        double v[16];
#pragma unroll
        for (int u = 0; u < 16; u++) v[u] = (j0 + u < K) ? z[j0 + u] : 0.0;
#pragma unroll
        for (int u = 0; u < 16; u++) s += v[u];
    }
    return s;
}

// Slot sl's constants (kind, function indices, term row, bounds, cost terms); see Slot.
__device__ __forceinline__ void slot_init(Slot &q, int sl, const SrbKParams &prm, const TermLayout &TL, const double *ref,
                                          int sE, int sV, int sO, int S, int rC, int rO, int K, int TT)
{
    const int N = prm.N, n = prm.n;
    q.kind = K_NONE; q.i0 = q.i1 = 0; q.r = 0; q.h[0] = q.h[1] = 0.0; q.a0 = q.a1 = 0.0; q.rx = 0.0; q.jd = 0.0;
    q.m[0] = q.m[1] = 0.0; q.wr = TT;
    if (sl < sE) {                                   // VAR
        const int v = sl;
        const bool isX = v < 4 * N, isU = !isX && v < 6 * N, isL = !isX && !isU && v < n - 1;
        q.kind = K_VAR; q.i0 = q.i1 = v; q.r = TL.zr(v);
        q.a0 = isX ? ((v >= 4 * (N - 1)) ? prm.Pw : prm.Qw) : isU ? prm.Rw : isL ? 0.0 : prm.Sw;
        q.a1 = isX ? -q.a0 * ref[v] : 0.0;
        q.h[0] = isL ? 1.0 : prm.box; q.h[1] = isL ? 0.0 : prm.box;
    } else if (sl < sV) {                            // COP
        const int e = sl - sE, i = e >> 1, d = e & 1;
        q.kind = K_COP; q.i0 = 4 * i + 2 * d; q.i1 = 4 * N + 2 * (i + 1) + d; q.r = rC + e;
        q.h[0] = q.h[1] = prm.fr;
    } else if (sl < sO) {                            // VEL
        const int tt = sl - sV, comp = (tt < N) ? 1 : 3, k = tt % N;
        q.kind = K_VEL; q.i0 = q.i1 = 4 * k + comp; q.r = 4 * k + comp;
        q.h[0] = q.h[1] = prm.vsat;
    } else if (sl < S) {                             // OBS (positions filled at the NLP stage)
        const int o = sl - sO, k = o / K;
        q.kind = K_OBS; q.i0 = 4 * k; q.i1 = 4 * k + 2; q.r = rO + o;
    }
#pragma unroll
    for (int r = 0; r < 2; r++) { q.s[r] = q.z[r] = 1.0; q.iz[r] = q.is[r] = 1.0; q.dz[r] = q.ds[r] = q.dsT[r] = q.r3[r] = 0.0; }
}

// the rows of slot q active in the stage (QP: linear rows; NLP: all), and the weight / rhs entry
// it stores to (VEL adds into its variable's term row instead: the scratch entry TT)
__device__ __forceinline__ void slot_stage(Slot &q, int n, bool nl, int TT)
{
    const bool lin = (q.kind == K_VAR && q.i0 < n - 1) || q.kind == K_COP;
    q.m[0] = (lin || (nl && (q.kind == K_VEL || q.kind == K_OBS))) ? 1.0 : 0.0;
    q.m[1] = (lin || (nl && q.kind == K_VEL)) ? 1.0 : 0.0;
    q.wr = (q.kind == K_VAR || q.kind == K_COP || q.kind == K_OBS) ? q.r : TT;
}

// LDS-bounds diagnostic build: the indices slot q (slot number sl) reads and writes through (LCK above)
#define SRB_SLOT_LCK(q, sl) do { \
    LCK((q).wr <= TT, 2); \
    LCK((q).kind == K_NONE || ((q).i0 >= 0 && (q).i0 < n && (q).i1 >= 0 && (q).i1 < n), 3); \
    LCK(!((q).kind == K_VAR || (q).kind == K_COP || (q).kind == K_VEL || ((q).kind == K_OBS && SRB_OBS_STORED(NZL))) || \
        ((q).r >= 0 && (q).r < RROWS), 1); \
    LCK((q).kind != K_OBS || ((sl) - sO >= 0 && (sl) - sO < NK && (q).r - rO == (sl) - sO), 5); \
} while (0)

// cost weight of variable v (Q_qp diagonal, MPC_dist.cpp:168-178)
__device__ __forceinline__ double var_weight(const SrbKParams &prm, int v)
{
    const int N = prm.N;
    return v < 4 * N ? ((v >= 4 * (N - 1)) ? prm.Pw : prm.Qw) : v < 6 * N ? prm.Rw : v < prm.n - 1 ? 0.0 : prm.Sw;
}

// Polish helper: every slot's row function g(x) into q.jd, each obstacle slot's term row M_o
// re-linearised at x (entry by entry: the polish runs a few times per solve, so the register
// staging of the interior-point loop is not worth its pressure here) and its multiplier into zo.
template <int NZL, int TS, int NW>
__device__ __forceinline__ void polish_rows(Slot (&Q)[TS], int nts, const double *xs, double *OJ, double *zo, int n,
                                            int rO, double *R, int nz)
{
    const double s_var = xs[n - 1];
#pragma unroll
    for (int t = 0; t < TS; t++)
        if (t < nts) {
            Slot &q = Q[t];
            q.jd = slot_f(q, xs, s_var);
            if (kind_of(q) == K_OBS) {
                const int o = q.r - rO;
                obs_relin<NZL>(R, OJ, rO, o, q.i0, q.i1, -2.0 * (xs[q.i0] - q.a0), -2.0 * (xs[q.i1] - q.a1));
                zo[o] = q.ds[0] * q.dz[0];
            }
        }
}

// Largest residual, over this thread's grids k = tid, tid + NTH, .., of the equality rows every returned
// point must satisfy (dec_vars_constr_cost.h:154-206): the LIP dynamics X_k = Ad X_{k-1} + Bd U_k
// (X_{-1} = x0), the CoP rows u_k = F_k lambda_k and sum lambda_k = 1.  The polish steps move along the
// null-space basis, so these hold to round-off; its acceptance checks it (SRB_POLISH_EQTOL).
__device__ __forceinline__ double lip_eq_res(const SrbKParams &prm, const double *x0, const double *xs, const double *foot,
                                             int N, int C, int tid, int NTH)
{
    // (x0 and the LDS iterate are read through their own address spaces -- no generic pointer selecting
    // between them: a flat access in this kernel changed its code generation enough to break the polish
    // of the run-time instance)
    double r = 0.0;
#if defined(SRB_DIAG_FLAT_EQRES)         // diagnostic builds only: round 5's first form (one generic pointer)
#ifndef SRB_DIAG_BUILD
#error "SRB_DIAG_FLAT_EQRES is a diagnostic-build option"
#endif
    for (int k = tid; k < N; k += NTH) {
        const double *xp = k ? xs + 4 * (k - 1) : x0;
        const double p0 = xp[0], p1 = xp[1], p2 = xp[2], p3 = xp[3];
#else
    const double g0x = x0[0], g1x = x0[1], g2x = x0[2], g3x = x0[3];
    for (int k = tid; k < N; k += NTH) {
        const int kp = k ? k - 1 : 0;
        const double p0 = k ? xs[4 * kp] : g0x, p1 = k ? xs[4 * kp + 1] : g1x;
        const double p2 = k ? xs[4 * kp + 2] : g2x, p3 = k ? xs[4 * kp + 3] : g3x;
#endif
        const double u0 = xs[4 * N + 2 * k], u1 = xs[4 * N + 2 * k + 1];
#pragma unroll
        for (int d = 0; d < 4; d++) {
            const double v = prm.Ad[4 * d] * p0 + prm.Ad[4 * d + 1] * p1 + prm.Ad[4 * d + 2] * p2 +
                             prm.Ad[4 * d + 3] * p3 + prm.Bd[2 * d] * u0 + prm.Bd[2 * d + 1] * u1;
            r = fmax(r, fabs(xs[4 * k + d] - v));
        }
        double g0 = 0.0, g1 = 0.0, sl = 0.0;
#pragma unroll
        for (int j = 0; j < 4; j++)
            if (j < C) {
                const double lam = xs[6 * N + C * k + j];
                g0 = fma(foot[(2 * k) * C + j], lam, g0); g1 = fma(foot[(2 * k + 1) * C + j], lam, g1); sl += lam;
            }
        r = fmax(r, fmax(fabs(u0 - g0), fmax(fabs(u1 - g1), fabs(sl - 1.0))));
    }
    return r;
}

// Reduced stationarity of the polished point (round 6): g = Z'(grad f(x) + J_A' z_A), grad f from the problem data
// (var_weight, the reference window in LDS) rather than the slots' cost registers, z_A the polish's multipliers
// (ds: active mask, dz: z_A); returns max |M^-1 g| (M: the last Newton step's reduced matrix, Mi its inverse), the
// correction a further step would make, accepted only up to SRB_POLISH_STOL and only where the multipliers that step
// leaves keep their sign (else 1e300).  The other
// tests (feasibility, multiplier signs, converged step, equality rows) held on the points the round-5 generic-
// pointer build returned as OPTIMAL although they were not stationary; this one does not.  The
// term rows are those of the last Newton step (the obstacle rows linearised at its start: O(|dx|) <= 1e-7 off).
// Uniform over the workgroup (every value reduced).  oracle/nlp_ipm.c `polish`: the same test.
template <int NZL, int TS, int NW, int NZE>
__device__ __forceinline__ double polish_stationary(Slot (&Q)[TS], int nts, const SrbKParams &prm, const double *xs,
                                                  const double *ref, double *CF, double *R, double *OJ, double *zo, int rO,
                                                  int cnt, const ObsFold &OF, int nko, double *vg, double *vy, double *vr,
                                                  double *vd, const double (&Mi)[NZL], const double *H0, int nz, int tid,
                                                  double *part, uint64_t bmask, double *red, int N, int n, int TT, int srow)
{
    double gmax = 0.0;
    SYNC();                                              // every lane's reads of R / OJ / CF / vg of the last step are done
    // the obstacle rows linearised at the polished point itself (the last Newton step, up to 1e-4 when the
    // active rows then hold to 1e-10, ran on rows taken before it: J'z would be off by 2 |dx| |z| there)
    polish_rows<NZL, TS, NW>(Q, nts, xs, OJ, zo, n, rO, R, nz);
    SYNC();
#pragma unroll
    for (int t = 0; t < TS; t++)
        if (t < nts) {
            const Slot &q = Q[t];
            const double zj = q.ds[0] * q.dz[0] - q.ds[1] * q.dz[1];
            const int kd = kind_of(q);
            if (kd == K_VAR) {
                const int v = q.i0;
                const double a0 = var_weight(prm, v), gf = fma(a0, xs[v], (v < 4 * N) ? -a0 * ref[v] : 0.0);
                gmax = fmax(gmax, fabs(gf));
                CF[q.wr] = gf + zj;
            } else if (kd == K_COP || kd == K_OBS) {
                CF[q.wr] = zj;
            }
        }
    if (NW > 1) SYNC();                                  // the VAR rows' plain stores land before the VEL adds
#pragma unroll
    for (int t = 0; t < TS; t++)
        if (t < nts && kind_of(Q[t]) == K_VEL)
            __hip_atomic_fetch_add(&CF[Q[t].r], Q[t].ds[0] * Q[t].dz[0] - Q[t].ds[1] * Q[t].dz[1], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
    SYNC();
    rhs_only<NZL, NW>(R, CF, cnt, OF, nko, vg, nz, tid, part, bmask);
    SYNC();
    // the Newton correction g implies, with the last step's inverse (Mi) and matrix (H0): the distance to the
    // stationary point in the reduced coordinates, whatever the scale of the gradient (oracle: the same test)
    double dxs[NZL];
    la_solve<NZL, NW, NZE>(Mi, H0, H0, 0.0, vg, vy, vr, vd, dxs, nz, tid & 63);
    double dm = 0.0;
#pragma unroll
    for (int j = 0; j < NZL; j++) dm = fmax(dm, fabs(dxs[j]));
    // ... and the multipliers that step would leave on the active rows, z_A + rho (c_A + J_A Z dxi) with dxi = -dxs
    // (the polish's own update), must keep their sign: a point stationary only through an active row that
    // should not be active (the row's multiplier of the wrong sign) is not a KKT point either
    constexpr int LDR = NZL + 1;
    double zmin = 1e300, zmax = 1.0;
#pragma unroll
    for (int t = 0; t < TS; t++)
        if (t < nts && (Q[t].ds[0] != 0.0 || Q[t].ds[1] != 0.0)) {
            const Slot &q = Q[t];
            const double jd = -((!SRB_OBS_STORED(NZL) && kind_of(q) == K_OBS)
                ? fma(OJ[2 * (q.r - rO)], row_dot<NZL, NZE>(R + q.i0 * LDR, dxs),
                      fma(OJ[2 * (q.r - rO) + 1], row_dot<NZL, NZE>(R + q.i1 * LDR, dxs), -row_dot<NZL, NZE>(R + srow * LDR, dxs)))
                : row_dot<NZL, NZE>(R + q.r * LDR, dxs));
#pragma unroll
            for (int r = 0; r < 2; r++)
                if (q.ds[r] != 0.0) {
                    const double zn = fma(prm.polish_rho, q.r3[r] + (r ? -jd : jd), q.dz[r]);
                    zmin = fmin(zmin, zn); zmax = fmax(zmax, fabs(zn));
                }
        }
    double rv[2] = {-zmin, zmax};
    wred_x<2, 3u, NW>(rv, red + 5 * 8 * NW, tid);
    (void)gmax;
    // (rho |c_A| <= rho SRB_POLISH_PTOL = 1 is the resolution of that update: the tolerance)
    return (-rv[0] >= -(prm.polish_rho * SRB_POLISH_PTOL + 1e-9 * rv[1])) ? dm : 1e300;
}

// --------------------------------------------------------------------------- shared agent code
// The solve kernel and the polish kernel run on the same per-agent LDS layout and rebuild the
// same null-space basis, so the code they share is written once, as statement macros expanded in
// both template bodies (they bind the locals of the expanding function):
//   SRB_AGENT_LAYOUT     sizes, term-row layout, slot ranges, the LDS carve (srb_lds_doubles)
//   SRB_AGENT_SETUP      inputs (a1/a2/a3: x0, reference window, footholds), Z, xbar, CoM-CoP rows
//   SRB_AGENT_OBSTACLES  the K selected rows per grid (srb_knn_kernel's sel; MPC_dist.cpp:371-396
//                        generalised, neighbours predicted at constant velocity o_k = p + v Ts (k+1))
//   SRB_AGENT_OUTPUTS    x, objective, alpha_COM
#define SRB_AGENT_LAYOUT \
    constexpr int NZM = ((NZL + 15) / 16) * 16; \
    constexpr int LDR = NZL + 1, LDH = NZL + 1; \
    constexpr int NTH = 64 * NW; \
    constexpr int NZE = (NC > 0 && CC > 0) ? NC * (CC - 1) + 1 : NZL;   /* reduced size when the shape is compiled */ \
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6; \
    /* the compiled shape (NC, CC, KC > 0) or the run-time one; n = (6 + C) N + 1, nz = N (C - 1) + 1 */ \
    const int N = NC > 0 ? NC : prm.N, C = CC > 0 ? CC : prm.C, K = KC > 0 ? KC : prm.K_obs + prm.K_nbr; \
    const int n = (NC > 0 && CC > 0) ? (6 + CC) * NC + 1 : prm.n, nz = (NC > 0 && CC > 0) ? NC * (CC - 1) + 1 : prm.nz; \
    const int NK = N * K, NE = 2 * (N - 1); \
    const int n4 = rnd4(n), NK4 = rnd4(NK), UL4 = rnd4(n - 4 * N); \
    const int E4 = (4 * N + NE + 16 * NW - 1) / (16 * NW) * (16 * NW) - 4 * N;   /* CoM-CoP block: rU a multiple of 16 NW */ \
    /* stored term rows: X (4N) | CoM-CoP (E4) | U, lambda, slack (UL4) | zero rows up to rO, a */ \
    /* multiple of 16 NW; then the NKP (NK padded likewise) generated obstacle terms: TT terms */ \
    const int rC = 4 * N, rU = rC + E4, rO = (rU + UL4 + 16 * NW - 1) / (16 * NW) * (16 * NW); \
    const int NKP = (NK + 16 * NW - 1) / (16 * NW) * (16 * NW), TT = rO + NKP; \
    const TermLayout TL{N, C, n, nz, E4}; \
    const uint64_t bmask = full_batches<NZM>(rO, N, C, n, rC, NE, rU, lane);   /* stored-row batches needing every column block */ \
    const int NOP = (3 * N + 16 * NW - 1) / (16 * NW) * (16 * NW);   /* folded obstacle grid terms (3 a grid), padded */ \
    const int sE = n, sV = n + NE, sO = sV + 2 * N, S = sO + NK; \
    const double tol = prm.tol, th = tol / sqrt(3.0); \
    STAMP_DECL; \
    /* LDS carve (must match srb_lds_doubles) */ \
    double *p = lds; \
    double *R = p; p += (SRB_OBS_STORED(NZL) ? TT : rO) * LDR;   /* stored term rows (Z rows first; + obstacle rows) */ \
    double *W = p; p += TT + 1;                   /* gram weights (+ one scratch entry) */ \
    double *CF = p; p += TT + 1;                  /* rhs coefficients (+ one scratch entry) */ \
    double *OJ = p; p += SRB_OBS_STORED(NZL) ? 0 : 2 * NKP;       /* folded instances: obstacle rows' jx, jy */ \
    double *FO = p; p += SRB_OBS_STORED(NZL) ? 0 : 9 * (N + 1);   /* per-grid obstacle fold S_k, c_k (+ a zero grid) */ \
    const ObsFold OF{OJ, FO, rO, N, K, NOP, full_obs_batches<NZM>(N, C, NOP, lane), rU, C, n}; \
    double *H0 = p; p += NZL * LDH;               /* assembled Z'HZ (unshifted; + delta Z'Z on the fly) */ \
    double *ZZ = p; p += NZL * LDH;               /* Z'Z (NLP) */ \
    double *vg = p; p += NZM; double *vy = p; p += NZM; double *vr = p; p += NZM; double *vd = p; p += NZM; \
    double *xs = p; p += n4; \
    double *xb = p; p += n4;                      /* xbar (setup); then dx = Z dxi of the Newton steps (dxv) */ \
    double *dxv = xb; \
    double *xsv = p; p += n4;                     /* NLP: saved iterate (round-off floor / polish) */ \
    double *xprev = p; p += n4;                   /* the iterate before the last update (non-finite fallback) */ \
    double *ref = p; p += 4 * N; \
    double *foot = p; p += 2 * C * N; \
    double *obs = SRB_OBS_IN_ZZ(NZL, NK) ? ZZ : p; p += SRB_OBS_IN_ZZ(NZL, NK) ? 0 : 2 * NK + 2;   /* obstacle positions (setup) */ \
    double *eps = p; p += K + 1; \
    double *zo = p; p += NK4;                     /* obstacle duals (per-grid sums) */ \
    int *sel = (int *)p; p += (K + 1); \
    double *red = p; p += (NW > 1) ? 8 * SRB_RED_SITES * NW : 0;   /* cross-wave reduction sites */ \
    double *part = p; p += (NW > 2) ? NW * ((NZM == 16) ? 1 : 3) * 256 + NW * NZM : 0;   /* partial Gram / rhs (NW = 4) */ \
    float *zpl = (float *)p; p += SRB_FUSED_POLISH_OK(NZL) ? rnd4(S) : 0;   /* fused polish: the exported active set (2 floats a slot) */ \
    const int RROWS = SRB_OBS_STORED(NZL) ? TT : rO;   /* term rows stored in R */ \
    LCK_INIT(); \
    LCK((int)(p - lds) <= srb_lds_doubles(prm, NZL, NW) - (SRB_FUSED_POLISH_OK(NZL) ? 0 : 0), 0); \
    LCK(rU <= RROWS && (!SRB_OBS_STORED(NZL) || rO + NKP <= TT), 4); \
    (void)RROWS; \
    do {} while (0)

#define SRB_AGENT_SETUP \
    const double *x0 = x0g + 4 * (size_t)agent; \
    for (int i = tid; i < 4 * N; i += NTH) ref[i] = refg[(size_t)agent * 4 * N + i]; \
    for (int i = tid; i < 2 * C * N; i += NTH) foot[i] = footg[(size_t)agent * 2 * C * N + i]; \
    if (prm.use_nlp && tid < K) sel[tid] = sel_g[(size_t)agent * K + tid]; \
    for (int i = tid; i < (int)(xs - R) + 2 * n4; i += NTH) R[i] = 0.0; \
    for (int i = tid; i < NK4; i += NTH) zo[i] = 0.0; \
    SYNC(); \
    STAMP_END(23);                 /* stamps build: inputs loaded, LDS cleared */ \
    if (prm.use_nlp) { SRB_AGENT_OBSTACLES; } \
    STAMP_END(24);                 /* stamps build: obstacle rows */ \
    /* null-space basis Z and particular point xbar (forward LIP rollout, MPC_dist.cpp:232-261) */ \
    if (tid == 0) { \
        double X[4] = {x0[0], x0[1], x0[2], x0[3]}; \
        for (int k = 0; k < N; k++) { \
            const double u0 = foot[(k * 2 + 0) * C + C - 1], u1 = foot[(k * 2 + 1) * C + C - 1]; \
            double Xn[4]; \
            for (int d = 0; d < 4; d++) \
                Xn[d] = prm.Ad[d * 4] * X[0] + prm.Ad[d * 4 + 1] * X[1] + prm.Ad[d * 4 + 2] * X[2] + prm.Ad[d * 4 + 3] * X[3] + \
                        prm.Bd[d * 2] * u0 + prm.Bd[d * 2 + 1] * u1; \
            for (int d = 0; d < 4; d++) { X[d] = Xn[d]; xb[4 * k + d] = Xn[d]; } \
            xb[4 * N + 2 * k] = u0; xb[4 * N + 2 * k + 1] = u1; \
            for (int j = 0; j < C; j++) xb[6 * N + C * k + j] = (j == C - 1) ? 1.0 : 0.0; \
        } \
        xb[n - 1] = 0.0; \
    } \
    for (int cg = tid; cg < nz - 1; cg += NTH) {   /* column 1 + cg: dof t of grid j (column 0: the slack) */ \
        const int j = cg / (C - 1), t = cg % (C - 1), col = cg + 1; \
        double lam[4]; \
        const int is_null = lambda_basis(foot + j * 2 * C, C, t, lam); \
        double g0 = 0.0, g1 = 0.0; \
        if (!is_null) \
            _Pragma("unroll") for (int i = 0; i < 4; i++) \
                if (i < C) { g0 += foot[(j * 2 + 0) * C + i] * lam[i]; g1 += foot[(j * 2 + 1) * C + i] * lam[i]; } \
        _Pragma("unroll") for (int i = 0; i < 4; i++) if (i < C) R[TL.zr(6 * N + C * j + i) * LDR + col] = R32(lam[i]); \
        R[TL.zr(4 * N + 2 * j) * LDR + col] = R32(g0); \
        R[TL.zr(4 * N + 2 * j + 1) * LDR + col] = R32(g1); \
        double v[4]; \
        for (int d = 0; d < 4; d++) v[d] = prm.Bd[d * 2] * g0 + prm.Bd[d * 2 + 1] * g1; \
        for (int k = j; k < N; k++) { \
            for (int d = 0; d < 4; d++) R[(4 * k + d) * LDR + col] = R32(v[d]); \
            double tt[4]; \
            for (int d = 0; d < 4; d++) tt[d] = prm.Ad[d * 4] * v[0] + prm.Ad[d * 4 + 1] * v[1] + prm.Ad[d * 4 + 2] * v[2] + prm.Ad[d * 4 + 3] * v[3]; \
            for (int d = 0; d < 4; d++) v[d] = tt[d]; \
        } \
    } \
    if (tid == 0) R[TL.zr(n - 1) * LDR] = 1.0; \
    SYNC(); \
    STAMP_END(25);                 /* stamps build: null-space basis, xbar */ \
    /* CoM-CoP term rows M_e = Z_p - Z_u (p: CoM of grid i, u: CoP of grid i+1); xs = xbar */ \
    if (tid < NE) { \
        const int i = tid >> 1, d = tid & 1, pp = 4 * i + 2 * d, uu = 4 * N + 2 * (i + 1) + d; \
        for (int a = 0; a < NZL; a++) Rt[tid * LDR + a] = R32(R[pp * LDR + a] - R[TL.zr(uu) * LDR + a]); \
    } \
    for (int v = tid; v < n; v += NTH) xs[v] = xb[v]; \
    do {} while (0)

#define SRB_AGENT_OBSTACLES \
    /* every (grid k, row j) pair on its own lane, all loads of a lane issued before its stores */ \
    { \
        double ox_[TS], oy_[TS]; \
        _Pragma("unroll") for (int t = 0; t < TS; t++) { \
            const int e = tid + NTH * t; \
            ox_[t] = oy_[t] = 0.0; \
            if (e < NK) { \
                const int k = e / K, j = e - k * K; \
                const bool st = j < prm.K_obs; \
                const int bi = sel[j]; \
                const double tt = st ? 0.0 : prm.Ts * (k + 1); \
                const size_t bj = (bi >= 0) ? bi : 0; \
                const double *srcp = st ? obstacles + 2 * bj : nbr_state + 4 * bj; \
                /* no selection (-1): a row 1000 m along +x, as the oracle */ \
                ox_[t] = (bi >= 0) ? srcp[0] + (st ? 0.0 : srcp[2] * tt) : x0[0] + 1000.0; \
                oy_[t] = (bi >= 0) ? srcp[1] + (st ? 0.0 : srcp[3] * tt) : x0[2]; \
            } \
        } \
        _Pragma("unroll") for (int t = 0; t < TS; t++) { \
            const int e = tid + NTH * t; \
            if (e < NK) { obs[2 * e] = ox_[t]; obs[2 * e + 1] = oy_[t]; } \
        } \
        if (tid < K) eps[tid] = (tid < prm.K_obs) ? prm.eps_obs : prm.eps_nbr; \
    } \
    do {} while (0)

#define SRB_AGENT_OUTPUTS \
    /* x and the objective 0.5 x'Q_qp x + f'x (ExCost::GetCost, dec_vars_constr_cost.h:423-438) */ \
    double f = 0.0; \
    for (int v = tid; v < n; v += NTH) { \
        const double xv = xs[v]; \
        x_out[(size_t)agent * n + v] = xv; \
        const double a0 = var_weight(prm, v), a1 = (v < 4 * N) ? -a0 * ref[v] : 0.0; \
        f += fma(0.5 * a0 * xv, xv, a1 * xv); \
    } \
    { \
        double rv[1] = {f}; \
        wred_x<1, 0u, NW>(rv, red + 6 * 8 * NW, tid); \
        f = rv[0]; \
    } \
    /* fitComTrajectory_eventbase (MPC_dist.cpp:784-855) as an epilogue: alpha_COM (4 x 5) interpolates */ \
    /* [buffer, X_0..X_3] at s = 0, 1/4, .., 1 (the reference's 24 x 24 KKT keeps only the s = 0 end */ \
    /* point row, so its solution is this interpolation): alpha[d][j] = sum_i Binv[j][i] p_i[d] */ \
    if (alpha_out && tid < 20) { \
        const int d = tid / 5, j = tid - 5 * (tid / 5); \
        double acc = prm.Binv[5 * j] * alpha_buf[(size_t)agent * 4 + d]; \
        for (int i = 1; i < 5; i++) acc = fma(prm.Binv[5 * j + i], xs[4 * (i - 1) + d], acc); \
        alpha_out[(size_t)agent * 20 + 5 * d + j] = acc; \
    } \
    do {} while (0)

// Diagnostic builds only (-DSRB_DIAG_POLISH_OUT, make lipvar): the fused polish's last acceptance test --
// its stationarity ratio (or, where the other tests failed, its equality residual) into obj, the tests it met
// as bits into the QP iteration count (1 primal, 2 active rows, 4 multipliers, 8 last step, 16 equality rows,
// 32 equality residual not finite, 64 a pass ran, 128 stationary)
#ifdef SRB_DIAG_POLISH_OUT
#ifndef SRB_DIAG_BUILD
#error "SRB_DIAG_POLISH_OUT is a diagnostic-build option"
#endif
#define SRB_POLISH_DIAG() do { dg_eqr = pcand ? sratio : eqr; dg_bits = 64 | (pv <= SRB_POLISH_PTOL) | ((cv <= SRB_POLISH_PTOL) << 1) | \
    ((nzmin <= 1e-9 * zm) << 2) | ((lastdx <= SRB_POLISH_DXTOL) << 3) | ((eqr <= SRB_POLISH_EQTOL) << 4) | ((!isfinite(eqr)) << 5) | \
    ((pcand && sratio <= SRB_POLISH_STOL) << 7); } while (0)
#else
#define SRB_POLISH_DIAG() do {} while (0)
#endif

// The passes of the active-set polish (polish_agent, and the fused polish at the end of nmpc_agent):
// PS[t] holds each slot's active mask (ds), multiplier z_A (dz) and the inactive rows' proximal weight
// (s); xs the interior-point result, also saved in xsv.  Sets `accepted`.
#define SRB_POLISH_PASSES_LOOP(PS)                                                                                                            \
_Pragma("clang loop unroll(disable)")                                                                                                         \
    for (int pass = 0; pass < SRB_POLISH_PASSES; pass++) {                                                                                    \
        bool bad = false;                                                                                                                     \
        double lastdx = 1e300;                                                                                                                \
_Pragma("clang loop unroll(disable)")                                                                                                         \
        for (int pit = 0; pit < SRB_POLISH_IT; pit++) {                                                                                       \
            SYNC(); /* xs of the previous step / pass */                                                                                      \
            polish_rows<NZL, TS, NW>(PS, nts, xs, OJ, zo, n, rO, R, nz); /* q.jd = g(x), M_o (OJ), zo = z_A */                                \
            SYNC(); /* R rows, zo */                                                                                                          \
            if (pit > 0) { /* converged after a small step (oracle, same rule) */                                                             \
                double cm = 0.0;                                                                                                              \
_Pragma("unroll")                                                                                                                             \
                for (int t = 0; t < TS; t++)                                                                                                  \
                    if (t < nts) {                                                                                                            \
                        const Slot &q = PS[t];                                                                                                \
                        cm = fmax(cm, fmax(q.ds[0] * fabs(q.jd - q.h[0]), q.ds[1] * fabs(q.jd + q.h[1])));                                    \
                    }                                                                                                                         \
                double rv[1] = {cm};                                                                                                          \
                wred_x<1, 1u, NW>(rv, red + 6 * 8 * NW, tid);                                                                                 \
                if (lastdx <= SRB_POLISH_DX1 && rv[0] <= SRB_POLISH_CTOL) { lastdx = 0.0; break; }                                            \
            }                                                                                                                                 \
_Pragma("unroll")                                                                                                                             \
            for (int t = 0; t < TS; t++)                                                                                                      \
                if (t < nts) {                                                                                                                \
                    Slot &q = PS[t];                                                                                                          \
                    q.r3[0] = q.jd - q.h[0]; q.r3[1] = -q.jd - q.h[1];                                                                        \
                    const double cfa = q.ds[0] * fma(prm.polish_rho, q.r3[0], q.dz[0]) - q.ds[1] * fma(prm.polish_rho, q.r3[1], q.dz[1]);     \
                    const double wa = (q.ds[0] != 0.0 ? prm.polish_rho : q.s[0]) + (q.ds[1] != 0.0 ? prm.polish_rho : q.s[1]);                \
                    if (kind_of(q) == K_VAR) {                                                                                                \
                        double hs = 0.0;                                                                                                      \
                        if (q.i0 < 4 * N && !(q.i0 & 1)) hs = -2.0 * zo_sum(zo, q.i0 >> 2, K);                                                \
                        W[q.wr] = q.a0 + hs + wa;                                                                                             \
                        CF[q.wr] = -(fma(q.a0, q.jd, q.a1) + cfa);                                                                            \
                    } else {                                                                                                                  \
                        W[q.wr] = wa; /* COP / OBS rows (VEL: the scratch entry) */                                                           \
                        CF[q.wr] = -cfa;                                                                                                      \
                    }                                                                                                                         \
                }                                                                                                                             \
            if (NW > 1) SYNC(); /* the VAR rows' plain stores land before the VEL adds */                                                     \
_Pragma("unroll")                                                                                                                             \
            for (int t = 0; t < TS; t++)                                                                                                      \
                if (t < nts && kind_of(PS[t]) == K_VEL) {                                                                                     \
                    const Slot &q = PS[t];                                                                                                    \
                    const double cfa = q.ds[0] * fma(prm.polish_rho, q.r3[0], q.dz[0]) - q.ds[1] * fma(prm.polish_rho, q.r3[1], q.dz[1]);     \
                    __hip_atomic_fetch_add(&W[q.r], (q.ds[0] != 0.0 ? prm.polish_rho : q.s[0]) + (q.ds[1] != 0.0 ? prm.polish_rho : q.s[1]),  \
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);                                                   \
                    __hip_atomic_fetch_add(&CF[q.r], -cfa, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);                                   \
                }                                                                                                                             \
            SYNC();                                                                                                                           \
            gram_rhs<NZL, true, NW>(R, W, CF, cnt, OF, nko, H0, vg, nz, tid, part, bmask);                                                    \
            SYNC();                                                                                                                           \
            if (pass == 0 && pit == 0) POLDBG_MAT(H0, LDH, vg, nz);                                                                           \
            gj_load<NZL, NZE>(Mi, H0, ZZ, 0.0, nz, lane);                                                                                          \
            if (gj_reduced<NZL, NZE>(Mi, nz, lane, 0) != 0) { bad = true; break; } /* not PD: reject */                                            \
            la_solve<NZL, NW, NZE>(Mi, H0, ZZ, 0.0, vg, vy, vr, vd, dxi, nz, lane);                                                                    \
            double mdx = 0.0;                                                                                                                 \
_Pragma("unroll")                                                                                                                             \
            for (int t = 0; t < TS; t++)                                                                                                      \
                if (t < nts) {                                                                                                                \
                    Slot &q = PS[t];                                                                                                          \
                    const double jd = (!SRB_OBS_STORED(NZL) && kind_of(q) == K_OBS) /* J_o Z dxi, folded instances (OJ) */                \
                        ? fma(OJ[2 * (q.r - rO)], row_dot<NZL, NZE>(R + q.i0 * LDR, dxi),                                                          \
                              fma(OJ[2 * (q.r - rO) + 1], row_dot<NZL, NZE>(R + q.i1 * LDR, dxi), -row_dot<NZL, NZE>(R + TL.zr(n - 1) * LDR, dxi)))     \
                        : row_dot<NZL, NZE>(R + q.r * LDR, dxi);                                                                                   \
                    q.dz[0] = fma(q.ds[0] * prm.polish_rho, q.r3[0] + jd, q.dz[0]);                                                           \
                    q.dz[1] = fma(q.ds[1] * prm.polish_rho, q.r3[1] - jd, q.dz[1]);                                                           \
                    if (kind_of(q) == K_VAR) {                                                                                                \
                        xs[q.i0] = q.jd + jd; /* every read of xs this step is behind a barrier */                                            \
                        mdx = fmax(mdx, fabs(jd));                                                                                            \
                    }                                                                                                                         \
                }                                                                                                                             \
            {                                                                                                                                 \
                double rv[1] = {mdx};                                                                                                         \
                wred_x<1, 1u, NW>(rv, red + 8 * 8 * NW, tid);                                                                                 \
                lastdx = rv[0];                                                                                                               \
            }                                                                                                                                 \
            POLDBG(4 + pass, pit, lastdx);                                                                                                    \
            POLDBG_X(pass, pit, xs, n);                                                                                                       \
            if (lastdx <= SRB_POLISH_DXTOL) break; /* converged: no further step */                                                           \
        }                                                                                                                                     \
        if (bad) break;                                                                                                                       \
        SYNC();                                                                                                                               \
 /* ---- acceptance at the polished point */                                                                                                  \
        double pv = -1e300, cv = 0.0, nzmin = -1e300, zm = 1.0, vi = -1e300, eqr = 0.0;                                                       \
        {                                                                                                                                     \
            const double s_var = xs[n - 1];                                                                                                   \
_Pragma("unroll")                                                                                                                             \
            for (int t = 0; t < TS; t++)                                                                                                      \
                if (t < nts) {                                                                                                                \
                    Slot &q = PS[t];                                                                                                          \
                    const double fq = slot_f(q, xs, s_var);                                                                                   \
_Pragma("unroll")                                                                                                                             \
                    for (int r = 0; r < 2; r++) {                                                                                             \
                        const double v = r ? -fq - q.h[1] : fq - q.h[0];                                                                      \
                        q.r3[r] = v;                                                                                                          \
                        if (q.m[r] != 0.0) pv = fmax(pv, v);                                                                                  \
                        if (q.ds[r] != 0.0) { cv = fmax(cv, fabs(v)); nzmin = fmax(nzmin, -q.dz[r]); zm = fmax(zm, fabs(q.dz[r])); }          \
                        else if (q.m[r] != 0.0) vi = fmax(vi, v);                                                                             \
                    }                                                                                                                         \
                }                                                                                                                             \
            double rv[6] = {pv, cv, nzmin, zm, vi, SRB_POLISH_EQCHECK ? lip_eq_res(prm, x0, xs, foot, N, C, tid, NTH) : 0.0};                \
            wred_x<6, 0x3Fu, NW>(rv, red + 7 * 8 * NW, tid);                                                                                  \
            pv = rv[0]; cv = rv[1]; nzmin = rv[2]; zm = rv[3]; vi = rv[4]; eqr = rv[5];                                                       \
        }                                                                                                                                     \
        POLDBG(pass, 0, pv); POLDBG(pass, 1, cv); POLDBG(pass, 2, nzmin); POLDBG(pass, 3, zm); POLDBG(pass, 4, vi);                           \
        POLDBG(pass, 5, lastdx); POLDBG(pass, 7, eqr);                                                                                        \
        const bool pcand = pv <= SRB_POLISH_PTOL && cv <= SRB_POLISH_PTOL && nzmin <= 1e-9 * zm && lastdx <= SRB_POLISH_DXTOL &&           \
                           eqr <= SRB_POLISH_EQTOL;                                                                                           \
        const double sratio = pcand ? polish_stationary<NZL, TS, NW, NZE>(PS, nts, prm, xs, ref, CF, R, OJ, zo, rO, cnt, OF, nko, vg, vy,    \
                                                              vr, vd, Mi, H0, nz, tid, part, bmask, red, N, n, TT, TL.zr(n - 1)) : 0.0;       \
        SRB_POLISH_DIAG();                                                                                                                    \
        if (pcand && sratio <= SRB_POLISH_STOL) {                                                                                             \
            POLDBG(pass, 6, 1.0);                                                                                                             \
            accepted = true;                                                                                                                  \
            break;                                                                                                                            \
        }                                                                                                                                     \
 /* next pass: the most negative multiplier leaves A, violated rows join; the rows */                                                         \
 /* that stay keep their multipliers (>= 0), the new ones start at 0 */                                                                       \
        double wd = 1e300;                                                                                                                    \
        int wk = 0x7fffffff;                                                                                                                  \
_Pragma("unroll")                                                                                                                             \
        for (int t = 0; t < TS; t++)                                                                                                          \
            if (t < nts)                                                                                                                      \
_Pragma("unroll")                                                                                                                             \
                for (int r = 0; r < 2; r++)                                                                                                   \
                    if (PS[t].ds[r] != 0.0 && PS[t].dz[r] < -1e-9 * zm) lexmin(wd, wk, PS[t].dz[r], 2 * (tid + NTH * t) + r);                 \
        wargmin_x<NW>(wd, wk, red + 9 * 8 * NW, tid);                                                                                         \
        if (wk == 0x7fffffff && !(vi > SRB_POLISH_PTOL)) break; /* nothing to change: rejected */                                             \
_Pragma("unroll")                                                                                                                             \
        for (int t = 0; t < TS; t++) {                                                                                                        \
            Slot &q = PS[t];                                                                                                                  \
_Pragma("unroll")                                                                                                                             \
            for (int r = 0; r < 2; r++) {                                                                                                     \
                if (2 * (tid + NTH * t) + r == wk) q.ds[r] = 0.0;                                                                             \
                else if (t < nts && q.ds[r] == 0.0 && q.m[r] != 0.0 && q.r3[r] > SRB_POLISH_PTOL) q.ds[r] = 1.0;                              \
                q.dz[r] = q.ds[r] * fmax(q.dz[r], 0.0);                                                                                       \
            }                                                                                                                                 \
        }                                                                                                                                     \
        SYNC();                                                                                                                               \
        for (int v = tid; v < n; v += NTH) xs[v] = xsv[v]; /* the next pass starts from the interior-point result */                          \
    }                                                                                                                                         \
    do {} while (0)

// --------------------------------------------------------------------------- main kernel
// NZL: register bound on nz (one reduced-matrix row per lane); TS: slot trips per thread;
// NW: wavefronts per agent (1, or 4 = one per SIMD of a CU for small batches).  With NW > 1
// the row slots and the term-row passes are split across the waves and combined through LDS;
// the reduced-system factorisation and solves run redundantly in every wave (identical data,
// identical results, no communication).
template <int NZL, int TS, int NW, int NC, int CC, int KC, int KF = 0>
__device__ __forceinline__ void nmpc_agent(const SrbKParams &prm, int agent,
                const double *__restrict__ x0g, const double *__restrict__ refg, const double *__restrict__ footg,
                const double *__restrict__ obstacles, int n_obs,
                const double *__restrict__ nbr_state, int n_all, int agent_offset,
                double *__restrict__ x_qp_out, double *__restrict__ x_out,
                double *__restrict__ obj_out, int *__restrict__ status_out, int *__restrict__ iters_out,
                const double *__restrict__ alpha_buf, double *__restrict__ alpha_out,
                const int *__restrict__ sel_g, float *__restrict__ zpol_g, int zstride, double *lds)
{
    SRB_AGENT_LAYOUT;
#ifdef SRB_STAMPS
    unsigned long long *stamp_lds = (unsigned long long *)p; p += SRB_NSTAMP;
    if (tid < 64) stamp_lds[tid] = 0;
#endif
    double *Rt = R + rC * LDR;                          // CoM-CoP rows

    STAMP_BEGIN();
    // ---- inputs (a1/a2/a3: x0, reference window, footholds), null-space basis Z, xbar, term rows
    SRB_AGENT_SETUP;

    // ---- slot constants
    Slot Q[TS];
#pragma unroll
    for (int t = 0; t < TS; t++) {
        slot_init(Q[t], tid + NTH * t, prm, TL, ref, sE, sV, sO, S, rC, rO, K, TT);
        SRB_SLOT_LCK(Q[t], tid + NTH * t);
    }
    double Mi[NZL];                                          // inverse of the reduced Newton matrix (row = lane)
    double dxi[NZL];                                         // Newton direction in xi (uniform)
#pragma unroll
    for (int j = 0; j < NZL; j++) { Mi[j] = (mrow<NZL>(lane) == j) ? 1.0 : 0.0; dxi[j] = 0.0; }
    // LEAN (the N = 20 instances, NZL 24): 1/z, 1/s, dsT and r3 are recomputed where they are used
    // instead of held per slot across the Newton solve (16 VGPRs a slot, 64 at TS = 4: the loop's
    // spills); the same expressions in the same order, so the results are bit-identical
    constexpr bool LEAN = NZL > 16;
    auto IZ = [&](const Slot &q, int r) -> double { if constexpr (LEAN) return rcp_d(q.z[r]); else return q.iz[r]; };
    auto IS = [&](const Slot &q, int r) -> double { if constexpr (LEAN) return rcp_d(q.s[r]); else return q.is[r]; };
    SYNC();
    STAMP_END(0);

    int qp_flag = 3, qp_it = 0, nlp_flag = 0, nlp_it = 0;
#ifdef SRB_DIAG_POLISH_OUT
    double dg_eqr = -1.0;
    int dg_bits = 0;
#endif
    const int nstage = prm.use_nlp ? 2 : 1;
    // One loop over the two stages so that the interior-point iteration exists once in the
    // code object (keeps the hot loop small for the instruction cache).
#pragma clang loop unroll(disable)
    for (int stage = 0; stage < nstage; stage++) {
        const bool nl = stage == 1;
        // the QP stage that the NLP follows runs to qp_warm_tol (its point is only the NLP's warm start)
        const double tolS = (!nl && prm.use_nlp && prm.qp_warm_tol > 0.0) ? prm.qp_warm_tol : tol, thS = tolS / sqrt(3.0);
        STAMP_STAGE(stage);
        const int nts = ((nl ? S : sV) + NTH - 1) / NTH;      // active slot trips
        const int mrows = nl ? (4 * (N - 1) + 12 * N + 2 * C * N + NK + 4 * N) : (4 * (N - 1) + 12 * N + 2 * C * N);
        const int cnt = rU, nko = nl ? NKP : 0;            // MFMA term rows (X, CoM-CoP), obstacle terms
        STAMP_BEGIN();
        // stage activity of each row
        // (written out here rather than through slot_stage: the call form measurably changes the
        // register allocation of the whole loop, 8 -> 72 VGPR spills for 12_4_1)
#pragma unroll
        for (int t = 0; t < TS; t++) {
            Slot &q = Q[t];
            const bool lin = (q.kind == K_VAR && q.i0 < n - 1) || q.kind == K_COP;
            q.m[0] = (lin || (nl && (q.kind == K_VEL || q.kind == K_OBS))) ? 1.0 : 0.0;
            q.m[1] = (lin || (nl && q.kind == K_VEL)) ? 1.0 : 0.0;
            q.wr = (q.kind == K_VAR || q.kind == K_COP || q.kind == K_OBS) ? q.r : TT;
        }
        if (!nl) {
            // ---------------- QP stage setup: kkt_initialize (Auxilary.c:680-755) ----------------
            // [P A' G'; A 0 0; G 0 -I] [x; y; z] = [-c; b; h]:  (Z'(P + G'G)Z) xi = -Z'(P xbar + c) + Z'G'(h - G xbar)
#pragma unroll
            for (int t = 0; t < TS; t++)
                if (t < nts) {
                    Slot &q = Q[t];
                    const double f = slot_f(q, xs, 0.0);
                    const double w0 = q.m[0] * (q.h[0] - f), w1 = q.m[1] * (q.h[1] + f);
                    const bool var = q.kind == K_VAR;
                    const double wgt = (var ? q.a0 : 0.0) + q.m[0] + q.m[1];
                    const double cfv = (var ? -q.a1 - q.a0 * f : 0.0) + (w0 - w1);
                    if (q.kind == K_VAR || q.kind == K_COP) { W[q.r] = wgt; CF[q.r] = cfv; }
                }
            SYNC();
            gram_rhs<NZL, true, NW>(R, W, CF, cnt, OF, nko, H0, vg, nz, tid, part, bmask);
            SYNC();
            gj_load<NZL, NZE>(Mi, H0, ZZ, 0.0, nz, lane);
            if (gj_reduced<NZL, NZE>(Mi, nz, lane, 1) != 0) {
                qp_flag = 1;                                  // x stays xbar (last iterate is returned)
                continue;
            }
            la_solve<NZL, NW, NZE>(Mi, H0, ZZ, 0.0, vg, vy, vr, vd, dxi, nz, lane);
            // x = xbar + Z xi ; zi = h - G x ; s, z shifted (Auxilary.c:716-746)
            double mn = 1e300, mx = -1e300;
#pragma unroll
            for (int t = 0; t < TS; t++)
                if (t < nts) {
                    Slot &q = Q[t];
                    const double f = slot_f(q, xs, 0.0) +
                        ((!SRB_OBS_STORED(NZL) && q.kind == K_OBS) ? 0.0 : row_dot<NZL, NZE>(R + q.r * LDR, dxi));   /* (OBS: masked here) */
                    q.jd = f;                                 // f(x) for the shift below
                    const double z0 = q.h[0] - f, z1 = q.h[1] + f;
                    if (q.m[0] != 0.0) { mn = fmin(mn, z0); mx = fmax(mx, z0); }
                    if (q.m[1] != 0.0) { mn = fmin(mn, z1); mx = fmax(mx, z1); }
                }
            double rv[2] = {-mn, mx};
            wred_x<2, 3u, NW>(rv, red + 0 * 8 * NW, tid);
            mn = -rv[0]; mx = rv[1];
            const double ssh = (-mn < 0) ? 0.0 : 1.0 - mn, zsh = (mx < 0) ? 0.0 : 1.0 + mx;
            SYNC();                                           // every lane has read xs = xbar
            // qp_init 1 (default): the scaled start of oracle/qp_ipm.c, s = max(h - Gx, 0.1), z = 1/s
            // (iSWIFT's z shift by 1 + max(h - Gx) is ~1e3 with the +-1e3 boxes: blocked dual steps,
            // up to 19 iterations on the bench batch against 9); qp_init 0: iSWIFT's start
            const bool scaled = prm.qp_init == 1;
#pragma unroll
            for (int t = 0; t < TS; t++)
                if (t < nts) {
                    Slot &q = Q[t];
                    const double f = q.jd, z0 = q.h[0] - f, z1 = q.h[1] + f;
                    q.s[0] = (q.m[0] != 0.0) ? (scaled ? fmax(z0, 0.1) : z0 + ssh) : 1.0;
                    q.s[1] = (q.m[1] != 0.0) ? (scaled ? fmax(z1, 0.1) : z1 + ssh) : 1.0;
                    q.z[0] = (q.m[0] != 0.0) ? (scaled ? rcp_d(q.s[0]) : -z0 + zsh) : 1.0;
                    q.z[1] = (q.m[1] != 0.0) ? (scaled ? rcp_d(q.s[1]) : -z1 + zsh) : 1.0;
                    if (q.kind == K_VAR) xs[q.i0] = f;
                    // rx = -(P x + c + A'y + G'z) = -G'(z - (G x - h)) at the least-squares start: 0 for
                    // iSWIFT's z (the shift is the same on the two rows of every +- pair), below for the
                    // scaled one (each row's z + (h - Gx) scattered onto its variables)
                    q.rx = 0.0;
                }
            if (scaled) {
                SYNC();
#pragma unroll
                for (int t = 0; t < TS; t++)              // the VAR rows' own bounds first (plain stores)
                    if (t < nts && Q[t].kind == K_VAR) {
                        const Slot &q = Q[t];
                        CF[q.r] = q.m[0] * (q.z[0] + q.h[0] - q.jd) - q.m[1] * (q.z[1] + q.h[1] + q.jd);
                    }
                SYNC();
#pragma unroll
                for (int t = 0; t < TS; t++)              // CoM-CoP rows +-(p_i - u_i+1): onto p_i and u_i+1
                    if (t < nts && Q[t].kind == K_COP) {
                        const Slot &q = Q[t];
                        const double g = q.m[0] * (q.z[0] + q.h[0] - q.jd) - q.m[1] * (q.z[1] + q.h[1] + q.jd);
                        __hip_atomic_fetch_add(&CF[TL.zr(q.i0)], g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        __hip_atomic_fetch_add(&CF[TL.zr(q.i1)], -g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                SYNC();
#pragma unroll
                for (int t = 0; t < TS; t++)
                    if (t < nts && Q[t].kind == K_VAR) Q[t].rx = -CF[Q[t].r];
            }
            SYNC();
            STAMP_END(1);
        } else {
            // ---------------- NLP stage setup (replaces SnoptSolver::Solve, MPC_dist.cpp:402-427) ----------------
            if (x_qp_out)
                for (int v = tid; v < n; v += NTH) x_qp_out[(size_t)agent * n + v] = xs[v];
            // obstacles per grid: the K_obs nearest static obstacles (MPC_dist.cpp:371-396,
            // generalised to K) and the K_nbr nearest other agents (get_lastState() rows),
            // predicted at constant velocity o_k = p + v Ts (k+1); query point = own CoM.
            // (selected by srb_knn_kernel, launched just before this kernel on the same stream)
            STAMP_END(6);                                     // NLP slot 6 (obstacle positions: loaded in the setup)
            SYNC();
            // slacks: shifted h - g(x) over every NLP row; duals 1
            const double s_var = xs[n - 1];
            double mn = 1e300;
#pragma unroll
            for (int t = 0; t < TS; t++)
                if (t < nts) {
                    Slot &q = Q[t];
                    if (q.kind == K_OBS) {
                        const int o = tid + NTH * t - sO;
                        LCK(o >= 0 && o < NK, 5);
                        q.a0 = obs[2 * o]; q.a1 = obs[2 * o + 1]; q.h[0] = -eps[o % K];
                    }
                    const double f = slot_f(q, xs, s_var);
                    q.jd = f;
                    if (q.m[0] != 0.0) mn = fmin(mn, q.h[0] - f);
                    if (q.m[1] != 0.0) mn = fmin(mn, q.h[1] + f);
                }
            {
                double rv[1] = {-mn};
                wred_x<1, 1u, NW>(rv, red + 1 * 8 * NW, tid);
                mn = -rv[0];
            }
            const double ssh = (-mn < 0) ? 0.0 : 1.0 - mn;
#pragma unroll
            for (int t = 0; t < TS; t++)
                if (t < nts) {
                    Slot &q = Q[t];
                    const double f = q.jd;
                    q.s[0] = (q.m[0] != 0.0) ? q.h[0] - f + ssh : 1.0;
                    q.s[1] = (q.m[1] != 0.0) ? q.h[1] + f + ssh : 1.0;
                    // z = Z0 / max(s, 1): rows far from their bound start at complementarity Z0, the
                    // others at Z0 (oracle/nlp_ipm.c, same rule)
                    q.z[0] = SRB_NLP_Z0 * rcp_d(fmax(q.s[0], 1.0));
                    q.z[1] = SRB_NLP_Z0 * rcp_d(fmax(q.s[1], 1.0));
                    if (q.kind == K_OBS) {                     // M_o = J_o Z at the current x (gram_rhs)
                        const int o = q.r - rO;
                        obs_relin<NZL>(R, OJ, rO, o, q.i0, q.i1, -2.0 * (xs[q.i0] - q.a0), -2.0 * (xs[q.i1] - q.a1));
                    }
                    // Z'Z (delta shifts) and rx0 = -Z (Z'Z)^-1 Z'(P x + c + J'z): each row's J'z on its
                    // term row (the velocity rows' below, onto their variables' rows)
                    const double jz = q.m[0] * q.z[0] - q.m[1] * q.z[1];
                    if (q.kind == K_VAR) { W[q.r] = 1.0; CF[q.r] = fma(q.a0, f, q.a1) + jz; }
                    else if (q.kind == K_COP) { W[q.r] = 0.0; CF[q.r] = jz; }
                    else if (q.kind == K_OBS) { W[q.r] = 0.0; CF[q.r] = q.z[0]; }
                }
            if (NW > 1) SYNC();                               // the VAR rows' plain stores land before the VEL adds
#pragma unroll
            for (int t = 0; t < TS; t++)
                if (t < nts && Q[t].kind == K_VEL)
                    __hip_atomic_fetch_add(&CF[Q[t].r], Q[t].m[0] * Q[t].z[0] - Q[t].m[1] * Q[t].z[1], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
            SYNC();
            // the first write of ZZ: the obstacle positions it may alias (SRB_OBS_IN_ZZ) were read by the slots'
            // setup above, and until here every ZZ operand was scaled by a zero shift, never read (gj_load / la_solve
            // test delta != 0; the LDS-check build asserts it, bit 7)
            gram_rhs<NZL, true, NW>(R, W, CF, cnt, OF, nko, ZZ, vg, nz, tid, part, bmask);
            SYNC();
            gj_load<NZL, NZE>(Mi, ZZ, ZZ, 0.0, nz, lane);
            gj_reduced<NZL, NZE>(Mi, nz, lane, 0);
            la_solve<NZL, NW, NZE>(Mi, ZZ, ZZ, 0.0, vg, vy, vr, vd, dxi, nz, lane);
#pragma unroll
            for (int t = 0; t < TS; t++)
                if (t < nts) {
                    Slot &q = Q[t];
                    q.rx = (q.kind == K_VAR) ? -row_dot<NZL, NZE>(R + q.r * LDR, dxi) : 0.0;
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
        double dxl = 1e300;              // this lane's max |ap dx| over its variable slots, last update
        int npassed = 0;                 // NLP: near-optimal iterates so far
        bool saved = false, restore = false;   // NLP: xsv holds the best near-optimal iterate
        bool prov = false;                     // NLP: OPTIMAL by the loosened tests only (-> 4 until polished)
        double best_rx = 1e300;                // its dual residual / max(1, ||Q x + f||_inf)
        // the polish kernel (srb_polish_kernel, launched next) starts from the NLP result: its active
        // set and multipliers -- rows with s * KAPPA < z keep z (as float: the Newton iteration's
        // starting guess, corrected by its first step; measured no different from double), the
        // others -min(z/s, OMCAP), their barrier weight, as a proximal term
        // -- go to HBM, zpol_g[agent][2 slot + row], with the iterate the result is taken from
        // (the saved one on a restore)
        // (LDS or global by a uniform branch, not a pointer select: a generic pointer would make these flat stores)
        auto export_zpol = [&]() {
            const bool to_lds = SRB_FUSED_POLISH_OK(NZL) && prm.polish_fused;
            // address-space-typed pointers: the two stores cannot be merged into one through a select
            __attribute__((address_space(1))) float *zg = (__attribute__((address_space(1))) float *)(zpol_g + (size_t)agent * zstride);
            __attribute__((address_space(3))) float *zl = (__attribute__((address_space(3))) float *)zpl;
#pragma unroll
            for (int t = 0; t < TS; t++)
                if (t < nts && tid + NTH * t < S)
#pragma unroll
                    for (int r = 0; r < 2; r++) {
                        const float v = Q[t].m[r] == 0.0 ? 0.0f
                            : (float)(Q[t].s[r] * SRB_POLISH_KAPPA < Q[t].z[r] ? Q[t].z[r] : -fmin(Q[t].z[r] / Q[t].s[r], SRB_POLISH_OMCAP));
                        if (to_lds) zl[2 * (tid + NTH * t) + r] = v;
                        else zg[2 * (tid + NTH * t) + r] = v;
                    }
        };
        for (int v = tid; v < n; v += NTH) xprev[v] = xs[v];
        for (int iter = 0; iter < maxit; iter++) {
            STAMP_BEGIN();
            // ---- residuals (computeresiduals, Auxilary.c:524-553), norms, reciprocals
            const double s_var = xs[n - 1];
            double nrx = 0.0, nrz = 0.0, sz = 0.0, gm = 1.0, zmx = 0.0;
            double fv[TS];
#pragma unroll
            for (int t = 0; t < TS; t++) {
                fv[t] = 0.0;
                if (t < nts) {
                    Slot &q = Q[t];
                    const double f = slot_f(q, xs, s_var);
                    fv[t] = f;
                    if (kind_of(q) == K_VAR) {
                        nrx = fma(q.rx, q.rx, nrx);
                        gm = fmax(gm, fabs(fma(q.a0, f, q.a1)));
                    }
                    const double rz0 = q.h[0] - q.s[0] - f, rz1 = q.h[1] - q.s[1] + f;
                    nrz = fma(q.m[0] * rz0, rz0, fma(q.m[1] * rz1, rz1, nrz));
                    sz = fma(q.m[0] * q.s[0], q.z[0], fma(q.m[1] * q.s[1], q.z[1], sz));
                    zmx = fmax(zmx, fmax(q.m[0] * q.z[0], q.m[1] * q.z[1]));
                    if constexpr (!LEAN)
#pragma unroll
                        for (int r = 0; r < 2; r++) { q.iz[r] = rcp_d(q.z[r]); q.is[r] = rcp_d(q.s[r]); }
                    if (nl && kind_of(q) == K_OBS) {              // re-linearise: M_o = J_o(x) Z (gram_rhs)
                        const int o = q.r - rO;
                        obs_relin<NZL>(R, OJ, rO, o, q.i0, q.i1, -2.0 * (xs[q.i0] - q.a0), -2.0 * (xs[q.i1] - q.a1));
                        zo[o] = q.z[0];
                    }
                }
            }
            STAMP_END(18);                                    // stamps build: residual loop | reduction
            double dxm;
            {
                double rv[6] = {nrx, nrz, sz, gm, dxl, zmx};
                wred_x<6, 56u, NW>(rv, red + 2 * 8 * NW, tid);
                nrx = sqrt(rv[0]); nrz = sqrt(rv[1]); sz = rv[2]; gm = rv[3]; dxm = rv[4]; zmx = rv[5];
            }
            const double mu = sz * inv_m;
            const bool f32 = KF && mu > prm.kkt32_mu;          // KF instances: fp32 factor this iteration
            (void)f32;
            STAMP_END(3);
            // divergence: a dual beyond SRB_Z_DIV means infeasible rows (converging solves keep their duals
            // below ~1e4; infeasible ones pass 1e10 within a few iterations and then overflow): FATAL at
            // this finite iterate (oracle/qp_ipm.c, nlp_ipm.c: the same rule).  A non-finite iterate
            // (nothing else should produce one) returns the previous iterate, so no FATAL solve hands the
            // caller NaN or inf
            if (!isfinite(nrx) || !isfinite(nrz) || !isfinite(sz) || !(zmx <= SRB_Z_DIV)) {
                flag = 3;
                if (!isfinite(nrx) || !isfinite(nrz) || !isfinite(sz)) {
                    SYNC();
                    for (int v = tid; v < n; v += NTH) xs[v] = xprev[v];
                    SYNC();
                }
                break;
            }
            // NLP: dual residual scaled by max(1, ||Q x + f||_inf) (QP: iSWIFT's absolute test)
            const double thx = nl ? SRB_NLP_EXITF * th * gm : thS;
            const double mtol = nl ? SRB_NLP_EXITF * tol : tolS;
            NLPDBG(iter, 0, nrx); NLPDBG(iter, 1, thx); NLPDBG(iter, 2, nrz); NLPDBG(iter, 3, sz * inv_m);
            const bool pass = nrx < thx && nrz < thS && sz * inv_m < mtol;
            if (pass && (!nl || dxm < SRB_NLP_DXTOL)) {
                // NLP: met only by the loosened tests (SRB_NLP_EXITF, which rely on the polish), the result
                // is provisional -- ACCEPTABLE (4) unless the polish kernel accepts its polish (oracle, same rule)
                prov = nl && !(nrx < th * gm && sz * inv_m < tol);
                flag = 0; break;
            }
            // NLP near the optimum (primal and complementarity met, dual residual within 100x):
            // an inertia shift or a blocked step from here is round-off of the condensed
            // system (W = z/s ~ 1e14 swamps the soft curvature in Z'HZ), not progress -> exit
            // ACCEPTABLE (4) at this iterate (oracle/nlp_ipm.c, the same rule)
            const bool near = nl && nrz < th && sz * inv_m < mtol && nrx < 100.0 * thx;
            // a solve that reached the near-optimal region and then left it is past its round-off
            // floor: ACCEPTABLE at the best near-optimal iterate (oracle, same rule)
            if (nl && saved && !near) { restore = true; flag = 4; break; }
            if (near && nrx / gm <= best_rx) {     // each thread copies the variables it owns
                best_rx = nrx / gm;
                for (int v = tid; v < n; v += NTH) xsv[v] = xs[v];
                if (zpol_g || prm.polish_fused) export_zpol();
                saved = true;
            }
            if (near && ++npassed >= SRB_NLP_NEARWAIT) { flag = 4; break; }
            bool acc = false;
            const bool pc = nl || (sigma > sigma_d);
            double delta = 0.0;
            // right-hand side of pass (0 predictor, 1 corrector / centring):
            //   dsT, r3 = rz - dsT / z, w = om r3, coefficient of term row r = rx + J'w
            auto set_rhs = [&](int pass) {
                const double smu = (pass == 0) ? 0.0 : (pc ? sigma * mu : sigma_d * mu);
                const bool corr = pass == 1 && pc;
                double cfs[TS];
#pragma unroll
                for (int t = 0; t < TS; t++) {
                    cfs[t] = 0.0;
                    if (t < nts) {
                        Slot &q = Q[t];
                        const double f = fv[t];
                        double cf = (kind_of(q) == K_VAR) ? q.rx : 0.0;
#pragma unroll
                        for (int r = 0; r < 2; r++) {
                            double dsT = -q.s[r] * q.z[r];
                            if (corr) dsT -= q.ds[r] * q.dz[r];
                            dsT += smu;
                            const double rz = r ? (q.h[1] - q.s[1] + f) : (q.h[0] - q.s[0] - f);
                            const double r3 = fma(-dsT, IZ(q, r), rz);
                            if constexpr (!LEAN) { q.dsT[r] = dsT; q.r3[r] = r3; }
                            cf = fma((r ? -q.m[1] : q.m[0]) * q.z[r] * IS(q, r), r3, cf);
                        }
                        cfs[t] = cf;
                        CF[q.wr] = cf;
                    }
                }
                if (NW > 1) SYNC();             // other waves' plain stores land before the VEL adds
                if (nl)
#pragma unroll
                    for (int t = 0; t < TS; t++)
                        if (t < nts && kind_of(Q[t]) == K_VEL)
                            __hip_atomic_fetch_add(&CF[Q[t].r], cfs[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            };
            if (pc) {
                // ---- weights W^-1 = z/s (updatekktmatrix, Auxilary.c:197-205), Lagrangian
                //      Hessian -2 sum_j z_kj on (x_k, y_k) (NLP), and the predictor right-hand
                //      side; one pass over the term rows assembles Z'HZ and Z'(rx + J'w)
                SYNC();
#pragma unroll
                for (int t = 0; t < TS; t++)
                    if (t < nts) {
                        Slot &q = Q[t];
                        const double om = fma(q.m[0] * q.z[0], IS(q, 0), q.m[1] * q.z[1] * IS(q, 1));
                        double hs = 0.0;
                        if (nl && kind_of(q) == K_VAR && q.i0 < 4 * N && !(q.i0 & 1)) {
                            const int k = q.i0 >> 2;
                            hs = zo_sum(zo, k, K);
                            hs *= -2.0;
                        }
                        W[q.wr] = om + ((kind_of(q) == K_VAR) ? q.a0 + hs : 0.0);
                    }
                if (NW > 1) SYNC();
                if (nl)
#pragma unroll
                    for (int t = 0; t < TS; t++)
                        if (t < nts && kind_of(Q[t]) == K_VEL)
                            __hip_atomic_fetch_add(&W[Q[t].r], Q[t].z[0] * IS(Q[t], 0) + Q[t].z[1] * IS(Q[t], 1), __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_WORKGROUP);
                STAMP_END(16);
                set_rhs(0);
                SYNC();
                STAMP_END(17);
                gram_rhs<NZL, true, NW>(R, W, CF, cnt, OF, nko, H0, vg, nz, tid, part, bmask);
                SYNC();
                STAMP_END(4);
                double dstart = 0.0;
                int ok = 0;
                for (int tries = 0; tries < (nl ? 14 : 1); tries++) {
                    if (tries == 0) {       // scale-aware first shift: 1e-10 * max(1, max diag of Z'HZ)
                        const double dm = (lane < nz) ? H0[lane * LDH + lane] : 1.0;
                        dstart = 1e-10 * fmax(1.0, wmax(dm));
                    }
                    // the QP stage never shifts: ZZ may still hold the obstacle positions there (SRB_OBS_IN_ZZ)
                    LCK(nl || delta == 0.0, 7);
                    gj_load<NZL, NZE>(Mi, H0, ZZ, delta, nz, lane);    // H0 + delta Z'Z (the solves shift on the fly too)
                    // KF instances: the inverse in fp32 while mu > kkt32_mu (then nref fp64 refinement steps per solve)
                    const int cf = (KF && f32) ? gj_invert_f32<NZL>(Mi, mrow<NZL>(lane), !nl) : gj_reduced<NZL, NZE>(Mi, nz, lane, !nl);
                    if (cf == 0) { ok = 1; break; }
                    delta = (delta == 0.0) ? dstart : delta * 10.0;
                }
                STAMP_END(5);
                if (!ok) { flag = 1; break; }
                if (near && delta != 0.0) { flag = 4; break; }
            }

            // ---- predictor (pc) or centring step (Prime.c:193-196), then corrector
            double ap = 1.0, ad = 1.0;
#pragma clang loop unroll(disable)
            for (int pass = (pc ? 0 : 1); pass < 2; pass++) {
                if (pass == 1 || !pc) {
                    set_rhs(pass);
                    SYNC();
                    STAMP_END(6 + 4 * pass);
                    rhs_only<NZL, NW>(R, CF, cnt, OF, nko, vg, nz, tid, part, bmask);
                    SYNC();
                    STAMP_END(7 + 4 * pass);
                }
                la_solve<NZL, NW, NZE, KF>(Mi, H0, ZZ, delta, vg, vy, vr, vd, dxi, nz, lane, (KF && f32) ? prm.kkt32_ref : SRB_REFINE);
                STAMP_END(8 + 4 * pass);
                // J dx per slot; dz = om (J dx - r3); ds = (dsT - s dz) / z; step-length maxima
                double mxs = 0.0, mxz = 0.0;
                // folded instances (N = 20): dx = Z dxi of every variable once (dxv; ceil(n / NTH) row dots a
                // lane instead of one per slot), then each slot's J dx from it: VAR / VEL dx_v, CoM-CoP
                // dx_p - dx_u, obstacle rows jx dx_px + jy dx_py - dx_s (config 5 1.81 -> 1.80 ms).  The
                // stored-row instances dot each slot's own row inside the slot loop (the separate pass measured
                // slower there: configs[2] 0.327 -> 0.340 ms)
                if constexpr (!SRB_OBS_STORED(NZL)) {
                    for (int v = tid; v < n; v += NTH) dxv[v] = row_dot<NZL, NZE>(R + TL.zr(v) * LDR, dxi);
                    SYNC();
                }
#pragma unroll
                for (int t = 0; t < TS; t++)
                    if (t < nts) {
                        Slot &q = Q[t];
                        const int kd = kind_of(q);
                        if constexpr (SRB_OBS_STORED(NZL)) {
                            LCK(q.r >= 0 && q.r < RROWS, 1);
                            q.jd = row_dot<NZL, NZE>(R + q.r * LDR, dxi);
                        } else if (kd == K_OBS) {                     /* (QP stage: masked rows, 0) */
                            const int o = q.r - rO;
                            q.jd = nl ? fma(OJ[2 * o], dxv[q.i0], fma(OJ[2 * o + 1], dxv[q.i1], -dxv[n - 1])) : 0.0;
                        } else {
                            q.jd = (kd == K_COP) ? dxv[q.i0] - dxv[q.i1] : dxv[q.i0];
                        }
#pragma unroll
                        for (int r = 0; r < 2; r++) {
                            const double izr = IZ(q, r), isr = IS(q, r);
                            double dsT, r3;
                            if constexpr (LEAN) {                    // set_rhs(pass)'s terms, recomputed
                                dsT = -q.s[r] * q.z[r];
                                if (pass == 1 && pc) dsT -= q.ds[r] * q.dz[r];
                                dsT += (pass == 0) ? 0.0 : (pc ? sigma * mu : sigma_d * mu);
                                const double rz = r ? (q.h[1] - q.s[1] + fv[t]) : (q.h[0] - q.s[0] - fv[t]);
                                r3 = fma(-dsT, izr, rz);
                            } else {
                                dsT = q.dsT[r]; r3 = q.r3[r];
                            }
                            q.dz[r] = q.m[r] * q.z[r] * isr * fma(r ? -1.0 : 1.0, q.jd, -r3);
                            q.ds[r] = q.m[r] * fma(-q.s[r], q.dz[r], dsT) * izr;
                            mxs = fmax(mxs, -q.ds[r] * isr); mxz = fmax(mxz, -q.dz[r] * izr);
                        }
                    }
                STAMP_END(21 + pass);
                // findsteplength (Auxilary.c:271-294): 1 / max(-dv / v), 1 when no dv < 0
                {
                    double rv[2] = {mxs, mxz};
                    wred_x<2, 3u, NW>(rv, red + (3 + 2 * pass) * 8 * NW, tid);
                    mxs = rv[0]; mxz = rv[1];
                }
                ap = (mxs > 0.0) ? 1.0 / mxs : 1.0;
                ad = (mxz > 0.0) ? 1.0 / mxz : 1.0;
                STAMP_END(9 + 4 * pass);
                if (pass == 0) {
                    // rho = (s + ap ds)'(z + ad dz) / s'z ; sigma = min(1, rho)^3  (formrho, Prime.c:160-170)
                    double num = 0.0;
#pragma unroll
                    for (int t = 0; t < TS; t++)
                        if (t < nts) {
                            const Slot &q = Q[t];
                            num = fma(q.m[0] * fma(ap, q.ds[0], q.s[0]), fma(ad, q.dz[0], q.z[0]), num);
                            num = fma(q.m[1] * fma(ap, q.ds[1], q.s[1]), fma(ad, q.dz[1], q.z[1]), num);
                        }
                    {
                        double rv[1] = {num};
                        wred_x<1, 0u, NW>(rv, red + 4 * 8 * NW, tid);
                        num = rv[0];
                    }
                    const double rho = num / sz, mr = rho < 1.0 ? rho : 1.0;
                    sigma = mr * mr * mr; if (sigma < sigma_d) sigma = sigma_d;
                    continue;
                }
                if (near && (ap < SRB_NLP_BLOCKED || ad < SRB_NLP_BLOCKED)) { acc = true; break; }
                // ---- update (Prime.c:208-216): step 0.99 alpha capped at 1
                ap = (0.99 * ap < 1.0) ? 0.99 * ap : 1.0;
                ad = (0.99 * ad < 1.0) ? 0.99 * ad : 1.0;
                dxl = 0.0;
                NLPDBG(iter, 4, ap); NLPDBG(iter, 5, ad); NLPDBG(iter, 6, delta); NLPDBG(iter, 7, sigma);
                // rx' = (1-ad) rx + (ad-ap) P dx + ad (hess + delta) dx - (J(x') - J(x))' z'
                // (hess from the old obstacle duals in zo, the Jacobian change from the new ones)
                double hso[TS];
#pragma unroll
                for (int t = 0; t < TS; t++) {
                    hso[t] = 0.0;
                    if (t < nts) {
                        Slot &q = Q[t];
                        if (nl && kind_of(q) == K_VAR && q.i0 < 4 * N && !(q.i0 & 1)) {
                            const int k = q.i0 >> 2;
                            hso[t] = zo_sum(zo, k, K);
                        }
#pragma unroll
                        for (int r = 0; r < 2; r++) { q.s[r] = fma(ap, q.ds[r], q.s[r]); q.z[r] = fma(ad, q.dz[r], q.z[r]); }
                    }
                }
                SYNC();          // every lane has read the old duals and x
                STAMP_END(19);
#pragma unroll
                for (int t = 0; t < TS; t++)
                    if (t < nts) {
                        Slot &q = Q[t];
                        if (nl && kind_of(q) == K_OBS) zo[q.r - rO] = q.z[0];
                        if (kind_of(q) == K_VAR) {
                            dxl = fmax(dxl, fabs(ap * q.jd));
                            q.rx = (1.0 - ad) * q.rx + ((ad - ap) * q.a0) * q.jd;
                            if (nl) q.rx = fma(ad * (delta - 2.0 * hso[t]), q.jd, q.rx);
                            xprev[q.i0] = fv[t];                 // the iterate a non-finite step falls back to
                            xs[q.i0] = fma(ap, q.jd, fv[t]);
                        }
                    }
                SYNC();
                STAMP_END(20);
                if (nl)
#pragma unroll
                    for (int t = 0; t < TS; t++)
                        if (t < nts) {
                            Slot &q = Q[t];
                            if (kind_of(q) == K_VAR && q.i0 < 4 * N && !(q.i0 & 1)) {   // +2 ap dx sum_j z'_kj on (x_k, y_k)
                                const int k = q.i0 >> 2;
                                double hs_new = 0.0;
                                hs_new = zo_sum(zo, k, K);
                                q.rx = fma(2.0 * ap * hs_new, q.jd, q.rx);
                            }
                        }
                STAMP_END(14);
            }
            if (acc) { flag = 4; break; }
            it++;
        }
        if (flag == 0 && prov) flag = 4;
        if (nl && saved && !prov && (restore || flag == 2 || flag == 4)) {      // ACCEPTABLE / MAXIT: the best saved iterate
            for (int v = tid; v < n; v += NTH) xs[v] = xsv[v];     // owner threads, as saved
            flag = 4;                                               // (zpol_g: exported at the save)
        } else if ((zpol_g || prm.polish_fused) && nl) {
            export_zpol();
        }
        // a QP stage that stopped at the warm-start tolerance reports 4 (its point is the NLP's warm start, not
        // iSWIFT's 1e-6 point), never OPTIMAL (oracle/batch.c, the same rule)
        if (stage == 0) { qp_flag = (flag == 0 && tolS > tol) ? 4 : flag; qp_it = it; } else { nlp_flag = flag; nlp_it = it; }
    }
    SYNC();
    if (x_qp_out && nstage == 1)
        for (int v = tid; v < n; v += NTH) x_qp_out[(size_t)agent * n + v] = xs[v];
    // ---- fused active-set polish (prm.polish_fused; otherwise srb_polish_kernel runs next): the same
    // passes on the LDS state the NLP stage left (term rows, iterate) with the interior-point slots
    // reused as the polish's (their state is dead here), so an agent that finishes early polishes on
    // its own SIMD while slower agents still iterate, and nothing goes through HBM.  Compiled for the
    // instances up to SRB_FUSED_POLISH_MAX (NZL 24 since round 5: N = 20 included, 28 B of scratch per lane
    // in 24_4_2_20_2_11, config 5 2.49 -> 2.12 ms with the compiled horizon; NZL 32 keeps the kernel)
    if constexpr (SRB_FUSED_POLISH_OK(NZL))
    if (prm.polish_fused && prm.use_nlp && nlp_flag != 1 && nlp_flag != 3) {
        const int nts = (S + NTH - 1) / NTH;
        const int cnt = rU, nko = NKP;
        for (int v = tid; v < n; v += NTH) xsv[v] = xs[v];
#pragma unroll
        for (int t = 0; t < TS; t++) {
            const int sl = tid + NTH * t;
#pragma unroll
            for (int r = 0; r < 2; r++) {
                LCK(!(t < nts && sl < S) || 2 * sl + r < 2 * rnd4(S), 6);
                const double v = (t < nts && sl < S) ? (double)zpl[2 * sl + r] : 0.0;
                Q[t].ds[r] = (v > 0.0) ? 1.0 : 0.0;
                Q[t].dz[r] = fmax(v, 0.0);
                Q[t].s[r] = fmax(-v, 0.0);
            }
        }
        bool accepted = false;
#ifdef SRB_DIAG_CORRUPT_COST       // diagnostic builds only: the defect class of the round-5 generic-pointer build --
#ifndef SRB_DIAG_BUILD             // the polish's cost registers off (here c_v of the X rows by 1 %), its data intact
#error "SRB_DIAG_CORRUPT_COST is a diagnostic-build option"
#endif
#pragma unroll
        for (int t = 0; t < TS; t++)
            if (Q[t].kind == K_VAR && Q[t].i0 < 4 * N) Q[t].a1 *= 1.01;
#endif
        SRB_POLISH_PASSES_LOOP(Q);
        SYNC();
        if (accepted) nlp_flag = 0;
        else
            for (int v = tid; v < n; v += NTH) xs[v] = xsv[v];
        SYNC();
        STAMP_END(26);                                      // stamps build: the fused polish
    }

    // ---- outputs: x, objective (ExCost::GetCost, dec_vars_constr_cost.h:423-438), alpha_COM
    SRB_AGENT_OUTPUTS;
    STAMP_END(15);
    STAMP_FLUSH(agent);
    if (tid == 0) {
        obj_out[agent] = f;
        status_out[2 * agent] = qp_flag; status_out[2 * agent + 1] = nlp_flag;
        iters_out[2 * agent] = qp_it; iters_out[2 * agent + 1] = nlp_it;
#ifdef SRB_DIAG_POLISH_OUT
        obj_out[agent] = dg_eqr; iters_out[2 * agent] = dg_bits;
#endif
    }
    LCK_REPORT(2 * agent);
}


// --------------------------------------------------------------------------- polish kernel
// Launched right after the solve kernel on the same stream, same instance geometry.  It rebuilds
// the agent's basis and term rows (SRB_AGENT_SETUP), takes the NLP result from x_out and the
// interior-point active set / multipliers from zpol_g, and replaces x, obj, alpha and the NLP
// status (-> OPTIMAL) only when the polish is accepted.  A kernel of its own: inside the solve
// kernel the polish's registers competed with the interior-point loop's and pushed its spills
// from 8 to 100-200 (configs[2] 0.40 -> 0.47-0.66 ms); here the loop is untouched.
template <int NZL, int TS, int NW, int NC, int CC, int KC>
__device__ __forceinline__ void polish_agent(const SrbKParams &prm, int agent,
                const double *__restrict__ x0g, const double *__restrict__ refg, const double *__restrict__ footg,
                const double *__restrict__ obstacles, const double *__restrict__ nbr_state,
                double *__restrict__ x_out, double *__restrict__ obj_out, int *__restrict__ status_out,
                const double *__restrict__ alpha_buf, double *__restrict__ alpha_out,
                const int *__restrict__ sel_g, const float *__restrict__ zpol_g, int zstride, double *lds)
{
    SRB_AGENT_LAYOUT;
#ifdef SRB_STAMPS
    unsigned long long *stamp_lds = nullptr;                // (the stamps build times the solve kernel only)
#endif
    double *Rt = R + rC * LDR;
    (void)xb; (void)dxv; (void)th; (void)tol; (void)wv;
    const int st1 = status_out[2 * agent + 1];
    if (!prm.use_nlp || st1 == 1 || st1 == 3) return;          // the whole workgroup: no usable iterate to polish
    // the solve's outputs first (x into xsv, which the setup does not clear; the exported active set
    // / multipliers into registers), so their HBM latency overlaps the setup
    const float *zp = zpol_g + (size_t)agent * zstride;
    float zv[TS][2];
#pragma unroll
    for (int t = 0; t < TS; t++) {
        const int sl = tid + NTH * t;
#pragma unroll
        for (int r = 0; r < 2; r++) zv[t][r] = (sl < S) ? zp[2 * sl + r] : 0.0f;
    }
    for (int v = tid; v < n; v += NTH) xsv[v] = x_out[(size_t)agent * n + v];
    SRB_AGENT_SETUP;
    SYNC();
    for (int v = tid; v < n; v += NTH) xs[v] = xsv[v];
    SYNC();
    POLDBG_IN(zp, S, xs, n);
    double Mi[NZL], dxi[NZL];
    // ---------------- active-set polish of the NLP result (oracle/nlp_ipm.c `polish`, the same rules) ----------------
    // Near its round-off floor the barrier system's active rows carry z/s ~ 1e14, so the
    // interior-point iterate stops up to ~1e-4 from the optimum along soft directions.  Rows
    // with s * KAPPA < z are taken as the active set A and min f s.t. Aeq x = beq, g_A(x) = h_A
    // is solved by Newton steps on its KKT system regularised by 1 / RHO:
    //   Z'(H_L + RHO J_A'J_A)Z dxi = -Z'(grad f + J_A'(z_A + RHO c_A)),  z_A += RHO (c_A + J_A Z dxi)
    // -- the interior-point machinery with weight RHO on the active rows, 0 on the others --
    // whose fixed point is the exact KKT point of that active set; at most SRB_POLISH_IT steps,
    // fewer once a correction is below SRB_POLISH_DXTOL.  Accepted (OPTIMAL) only when primal
    // feasible, dual feasible and converged; otherwise the most negative multiplier leaves A,
    // violated rows join, and the next pass starts again from the interior-point result (at
    // most SRB_POLISH_PASSES); a rejected polish leaves that result.  The slots are rebuilt
    // here (the interior-point slot state is dead); their fields ds = active mask, dz = z_A,
    // r3 = row value g - h, jd = g(x), s = the inactive rows' interior-point weight z/s, kept in
    // the Hessian only (a proximal term: the fixed point is unchanged, and the reduced matrix
    // stays definite along directions no active row pins, lambda with four contacts).
    {
        const int nts = (S + NTH - 1) / NTH;
        const int cnt = rU, nko = NKP;
        Slot P[TS];
#pragma unroll
        for (int t = 0; t < TS; t++) {
            Slot &q = P[t];
            const int sl = tid + NTH * t;
            slot_init(q, sl, prm, TL, ref, sE, sV, sO, S, rC, rO, K, TT);
            SRB_SLOT_LCK(q, sl);
            slot_stage(q, n, true, TT);
            if (q.kind == K_OBS) { const int o = sl - sO; q.a0 = obs[2 * o]; q.a1 = obs[2 * o + 1]; q.h[0] = -eps[o % K]; }
#pragma unroll
            for (int r = 0; r < 2; r++) {
                const double v = (t < nts && sl < S) ? (double)zv[t][r] : 0.0;
                q.ds[r] = (v > 0.0) ? 1.0 : 0.0;
                q.dz[r] = fmax(v, 0.0);
                q.s[r] = fmax(-v, 0.0);
            }
        }
        bool accepted = false;
#ifdef SRB_DIAG_POLISH_OUT
        double dg_eqr = -1.0;
        int dg_bits = 0;
#endif
        SRB_POLISH_PASSES_LOOP(P);
        SYNC();
        if (accepted) {
            SRB_AGENT_OUTPUTS;
            if (tid == 0) { obj_out[agent] = f; status_out[2 * agent + 1] = 0; }
        }
    }
    LCK_REPORT(2 * agent);

}

#define SRB_NMPC_KERNEL(NZL, TS, NW, NC, CC, KC)                                                               \
    extern "C" __global__ void __launch_bounds__(64 * NW) SRB_WPE                                              \
    srb_nmpc_kernel_##NZL##_##TS##_##NW##_##NC##_##CC##_##KC(                                                 \
        SrbKParams prm, int n_agents, const double *__restrict__ x0g, const double *__restrict__ refg,          \
        const double *__restrict__ footg, const double *__restrict__ obstacles, int n_obs,                       \
        const double *__restrict__ nbr_state, int n_all, int agent_offset, double *__restrict__ x_qp_out,        \
        double *__restrict__ x_out, double *__restrict__ obj_out, int *__restrict__ status_out,                 \
        int *__restrict__ iters_out, const double *__restrict__ alpha_buf, double *__restrict__ alpha_out,       \
        const int *__restrict__ sel_g, float *__restrict__ zpol_g, int zstride)                               \
    {                                                                                                          \
        extern __shared__ __attribute__((aligned(16))) double lds[];                                           \
        const int agent = xcd_agent(blockIdx.x, gridDim.x);                                                   \
        if (agent >= n_agents) return;                                                                         \
        nmpc_agent<NZL, TS, NW, NC, CC, KC>(prm, agent, x0g, refg, footg, obstacles, n_obs, nbr_state, n_all, agent_offset, \
                                x_qp_out, x_out, obj_out, status_out, iters_out, alpha_buf, alpha_out, sel_g, \
                                zpol_g, zstride, lds);                                                         \
    }                                                                                                          \
    extern "C" __global__ void __launch_bounds__(64 * NW) SRB_WPE                                              \
    srb_polish_kernel_##NZL##_##TS##_##NW##_##NC##_##CC##_##KC(                                               \
        SrbKParams prm, int n_agents, const double *__restrict__ x0g, const double *__restrict__ refg,          \
        const double *__restrict__ footg, const double *__restrict__ obstacles,                                 \
        const double *__restrict__ nbr_state, double *__restrict__ x_out, double *__restrict__ obj_out,          \
        int *__restrict__ status_out, const double *__restrict__ alpha_buf, double *__restrict__ alpha_out,     \
        const int *__restrict__ sel_g, const float *__restrict__ zpol_g, int zstride)                         \
    {                                                                                                          \
        extern __shared__ __attribute__((aligned(16))) double lds[];                                           \
        const int agent = xcd_agent(blockIdx.x, gridDim.x);                                                   \
        if (agent >= n_agents) return;                                                                         \
        polish_agent<NZL, TS, NW, NC, CC, KC>(prm, agent, x0g, refg, footg, obstacles, nbr_state, x_out, obj_out,          \
                                  status_out, alpha_buf, alpha_out, sel_g, zpol_g, zstride, lds);             \
    }

// fp32-factor instances (KF = 1; SRB_OPT_KKT_FP32_MU > 0 selects them): configs[4]'s "fp32 KKT with fp64
// iterative-refine residuals" -- the reduced Newton matrix assembled and refined against in fp64, inverted in
// fp32 while the complementarity mu is above prm.kkt32_mu, in fp64 below
#define SRB_NMPC_KERNEL_F32(NZL, TS, NW, NC, CC, KC)                                                           \
    extern "C" __global__ void __launch_bounds__(64 * NW) SRB_WPE                                              \
    srb_nmpc_kernel_f32_##NZL##_##TS##_##NW##_##NC##_##CC##_##KC(                                             \
        SrbKParams prm, int n_agents, const double *__restrict__ x0g, const double *__restrict__ refg,          \
        const double *__restrict__ footg, const double *__restrict__ obstacles, int n_obs,                       \
        const double *__restrict__ nbr_state, int n_all, int agent_offset, double *__restrict__ x_qp_out,        \
        double *__restrict__ x_out, double *__restrict__ obj_out, int *__restrict__ status_out,                 \
        int *__restrict__ iters_out, const double *__restrict__ alpha_buf, double *__restrict__ alpha_out,       \
        const int *__restrict__ sel_g, float *__restrict__ zpol_g, int zstride)                               \
    {                                                                                                          \
        extern __shared__ __attribute__((aligned(16))) double lds[];                                           \
        const int agent = xcd_agent(blockIdx.x, gridDim.x);                                                   \
        if (agent >= n_agents) return;                                                                         \
        nmpc_agent<NZL, TS, NW, NC, CC, KC, 1>(prm, agent, x0g, refg, footg, obstacles, n_obs, nbr_state, n_all, agent_offset, \
                                x_qp_out, x_out, obj_out, status_out, iters_out, alpha_buf, alpha_out, sel_g, \
                                zpol_g, zstride, lds);                                                         \
    }

#if defined(SRB_PART) && !defined(SRB_DEV_INSTANCES)
#if SRB_PART == 0
SRB_KI_PART0(SRB_NMPC_KERNEL)
#elif SRB_PART == 1
SRB_KI_PART1(SRB_NMPC_KERNEL)
#elif SRB_PART == 2
SRB_KI_PART2(SRB_NMPC_KERNEL)
SRB_KF32_PART2(SRB_NMPC_KERNEL_F32)
#else
SRB_KI_PART3(SRB_NMPC_KERNEL)
SRB_KF32_PART3(SRB_NMPC_KERNEL_F32)
#endif
#else
SRB_KERNEL_INSTANCES(SRB_NMPC_KERNEL)
#ifndef SRB_DEV_INSTANCES
SRB_KF32_INSTANCES(SRB_NMPC_KERNEL_F32)
#endif
#endif

#if !defined(SRB_PART) || SRB_PART == 0

// Obstacle and neighbour selection (MPC_dist.cpp:371-396, generalised to K): one workgroup per
// agent, the K_obs nearest static obstacles (with the reference's 1000 m sentinel) and the
// K_nbr nearest other agents to the agent's own CoM, indices to sel_out[agent][K_obs + K_nbr]
// (-1: no neighbour row).  A kernel of its own rather than a phase of the solve: there the
// scan ran at the solve kernel's occupancy, one or two waves per CU, and took a quarter of
// the solve (profiles/r01_c3_stamps.txt).  Tables of SRB_GRID_MIN_ROWS rows or more come with
// a uniform grid (srb_grid_build_kernel) and only the cells around the agent are scanned.
extern "C" __global__ void __launch_bounds__(64 * SRB_KNN_WAVES) srb_knn_kernel(int n_agents,
                const double *__restrict__ x0g, const double *__restrict__ obstacles, int n_obs,
                const double *__restrict__ nbr_state, int n_all, int agent_offset, int K_obs, int K_nbr,
                int *__restrict__ sel_out, int sel_stride, const SrbGrid *__restrict__ gob, const int *__restrict__ oob,
                const double2 *__restrict__ pob, const int *__restrict__ iob, const SrbGrid *__restrict__ gnb,
                const int *__restrict__ onb, const double2 *__restrict__ pnb, const int *__restrict__ inb)
{
    __shared__ double wd_lds[SRB_KNN_WAVES];
    __shared__ int wi_lds[SRB_KNN_WAVES];
    const int agent = xcd_agent(blockIdx.x, gridDim.x), tid = threadIdx.x;
    if (agent >= n_agents) return;                 // whole workgroup: the barriers stay uniform
    const double px = x0g[4 * (size_t)agent], py = x0g[4 * (size_t)agent + 2];
    // sel_stride = Ko + Kn of the whole selection; a pass over one table (srb_select_device) hands over
    // K_obs or K_nbr alone and sel_out already offset to its columns
    int *sel = sel_out + (size_t)agent * sel_stride;
    if (SRB_KNN_WAVES == 2 && K_obs > 0 && K_nbr > 0) {
        // the two tables on the two waves at once, each selection wave-local (DPP argmins, no barrier):
        // configs[2] selection 23.5 -> 20.9 us a step (HIP events, round 5; round 6's thresholded scan and ballot
        // argmin in srb_wave.h: 20.5 -> 13.4 us); the same rows.  (Selecting
        // inside the solve kernel's setup instead measured no faster at configs[2] -- the solve kernel
        // grew by what the launch saved -- and 4.6 % slower at N = 20, where four rounds of agents each
        // wait for their selection; round 5)
        const int lane = tid & 63;
        if (tid < 64)
            knn_select<1>(lane, px, py, obstacles, 2, n_obs, -1, K_obs, 1, sel, wd_lds, wi_lds, gob, oob, pob, iob);
        else
            knn_select<1>(lane, px, py, nbr_state, 4, n_all, agent_offset + agent, K_nbr, 0, sel + K_obs, wd_lds, wi_lds,
                          gnb, onb, pnb, inb);
        return;
    }
    // one table (srb_select_device's passes, or a batch without neighbour rows): a table that one wave scans
    // with the threshold pass (knn_thresh) or through a grid runs on wave 0 alone -- the two-wave form pays two
    // barriers per pop round (round 6: the neighbour pass of the multi-GPU step 19.3 us with both waves)
    if (SRB_KNN_WAVES == 2 && (K_obs > 0) != (K_nbr > 0)) {
        const bool o = K_obs > 0;
        const SrbGrid *g = o ? gob : gnb;
        if ((o ? n_obs : n_all) <= 64 * SRB_KNN_RB || (g && g->ok)) {
            if (tid >= 64) return;                     // whole wave: no barrier follows on the one-wave path
            if (o) knn_select<1>(tid, px, py, obstacles, 2, n_obs, -1, K_obs, 1, sel, wd_lds, wi_lds, gob, oob, pob, iob);
            else knn_select<1>(tid, px, py, nbr_state, 4, n_all, agent_offset + agent, K_nbr, 0, sel + K_obs, wd_lds, wi_lds,
                               gnb, onb, pnb, inb);
            return;
        }
    }
    if (K_obs > 0)
        knn_select<SRB_KNN_WAVES>(tid, px, py, obstacles, 2, n_obs, -1, K_obs, 1, sel, wd_lds, wi_lds, gob, oob, pob, iob);
    if (K_nbr > 0)
        knn_select<SRB_KNN_WAVES>(tid, px, py, nbr_state, 4, n_all, agent_offset + agent, K_nbr, 0, sel + K_obs, wd_lds,
                                  wi_lds, gnb, onb, pnb, inb);
}

// Uniform grid over one table per workgroup (block 0: table 0, block 1: table 1), rebuilt every
// launch (the neighbour snapshot moves every cycle): bounds of the finite rows, about two rows
// per cell (at most SRB_GRID_CELLS cells), counts by LDS atomics, one exclusive scan, scatter of
// the rows into cell order.  One workgroup of 1024 threads per table: a few microseconds for the
// tens of thousands of rows of an 8-GPU swarm, against a brute-force scan per agent.
__device__ __forceinline__ int grid_cell(double x, double y, double x0, double y0, double inv_h, int nx, int ny)
{
    const int cx = min(max((int)((x - x0) * inv_h), 0), nx - 1);
    const int cy = min(max((int)((y - y0) * inv_h), 0), ny - 1);
    return cy * nx + cx;
}

extern "C" __global__ void __launch_bounds__(1024) srb_grid_build_kernel(
    const double *__restrict__ tab0, int stride0, int n0, SrbGrid *g0, int *off0, double2 *spos0, int *sidx0,
    const double *__restrict__ tab1, int stride1, int n1, SrbGrid *g1, int *off1, double2 *spos1, int *sidx1)
{
    __shared__ int cnt[SRB_GRID_CELLS];
    __shared__ double red[4][16];
    __shared__ int part[1024];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const double *tab = blockIdx.x ? tab1 : tab0;
    const int stride = blockIdx.x ? stride1 : stride0, n = blockIdx.x ? n1 : n0;
    SrbGrid *g = blockIdx.x ? g1 : g0;
    int *off = blockIdx.x ? off1 : off0;
    double2 *spos = blockIdx.x ? spos1 : spos0;
    int *sidx = blockIdx.x ? sidx1 : sidx0;
    if (!g) return;
    // bounds of the finite rows
    double mnx = __builtin_inf(), mny = __builtin_inf(), mxx = -__builtin_inf(), mxy = -__builtin_inf();
    for (int i = tid; i < n; i += 1024) {
        const double x = tab[(size_t)stride * i], y = tab[(size_t)stride * i + 1];
        if (isfinite(x) && isfinite(y)) { mnx = fmin(mnx, x); mny = fmin(mny, y); mxx = fmax(mxx, x); mxy = fmax(mxy, y); }
    }
    mnx = wmin(mnx); mny = wmin(mny); mxx = wmax(mxx); mxy = wmax(mxy);
    if (lane == 0) { red[0][wv] = mnx; red[1][wv] = mny; red[2][wv] = mxx; red[3][wv] = mxy; }
    __syncthreads();
    mnx = red[0][0]; mny = red[1][0]; mxx = red[2][0]; mxy = red[3][0];
    for (int w = 1; w < 16; w++) {
        mnx = fmin(mnx, red[0][w]); mny = fmin(mny, red[1][w]); mxx = fmax(mxx, red[2][w]); mxy = fmax(mxy, red[3][w]);
    }
    if (!(mnx <= mxx)) {                           // no finite row: selection falls back to the scan
        if (tid == 0) g->ok = 0;
        return;
    }
    const double W = mxx - mnx, H = mxy - mny;
    const int target = min(max(n / 2, 1), SRB_GRID_CELLS);
    double h = sqrt(fmax(W * H, 1e-300) / target);
    if (!(h > 0.0) || !isfinite(h)) h = 1.0;
    h = fmax(h, fmax(W, H) / 4096.0);             // keeps nx, ny in range
    int nx = (int)(W / h) + 1, ny = (int)(H / h) + 1;
    while ((long long)nx * ny > SRB_GRID_CELLS) { h *= 1.25; nx = (int)(W / h) + 1; ny = (int)(H / h) + 1; }
    const double inv_h = 1.0 / h;
    const int C = nx * ny;
    for (int c = tid; c < C; c += 1024) cnt[c] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += 1024) {
        const double x = tab[(size_t)stride * i], y = tab[(size_t)stride * i + 1];
        if (isfinite(x) && isfinite(y)) atomicAdd(&cnt[grid_cell(x, y, mnx, mny, inv_h, nx, ny)], 1);
    }
    __syncthreads();
    // exclusive scan: per-thread chunk sums, a scan of the 1024 partials, chunk-local offsets
    const int chunk = (C + 1023) / 1024, c0 = tid * chunk, c1 = min(c0 + chunk, C);
    int sum = 0;
    for (int c = c0; c < c1; c++) sum += cnt[c];
    part[tid] = sum;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const int v = (tid >= o) ? part[tid - o] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    int run = part[tid] - sum;                     // exclusive prefix of this chunk
    for (int c = c0; c < c1; c++) { const int v = cnt[c]; cnt[c] = run; off[c] = run; run += v; }
    if (tid == 1023) off[C] = part[1023];
    __syncthreads();
    for (int i = tid; i < n; i += 1024) {
        const double x = tab[(size_t)stride * i], y = tab[(size_t)stride * i + 1];
        if (isfinite(x) && isfinite(y)) {
            const int at = atomicAdd(&cnt[grid_cell(x, y, mnx, mny, inv_h, nx, ny)], 1);
            spos[at] = make_double2(x, y);
            sidx[at] = i;
        }
    }
    if (tid == 0) {
        SrbGrid r;
        r.x0 = mnx; r.y0 = mny; r.inv_h = inv_h; r.h = h; r.nx = nx; r.ny = ny; r.n = part[1023]; r.ok = 1;
        *g = r;
    }
}
#endif   // SRB_PART 0: selection kernels
