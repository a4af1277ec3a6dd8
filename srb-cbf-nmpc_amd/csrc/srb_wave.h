// Wavefront helpers shared by the gfx950 kernels of this library (NMPC solve, low-level
// CLF-QP): DPP/permlane reductions, readlane broadcasts, a refined reciprocal and the
// register Gauss-Jordan inverse.  Header-only, device code.
#pragma once
#include <hip/hip_runtime.h>

#ifndef WAVE
#define WAVE 64
#endif
#ifndef SRB_USE_DPP     // DPP row_newbcast broadcasts in the reduced solve (0: readlane / LDS forms)
#define SRB_USE_DPP 1
#endif

typedef double d4 __attribute__((ext_vector_type(4)));

// Agent of workgroup b in a grid of n one-agent workgroups, XCD-aware: the dispatcher deals
// workgroups round-robin over the 8 XCDs (MI355X_MICROARCH.md, "Workgroup dispatch"; observed, not
// promised -- only the traffic depends on it), so b and b + 8 share an L2.  Workgroups b = 8 j + x take
// the x-th contiguous block of agents: neighbouring agents' inputs share 128-B lines, which a
// round-robin assignment fetched once into each of up to four L2s (configs[2]: x0, ref, foot and the
// selection rows 1.09 -> 0.73 MB per launch, tools/ubench/kernarg_fetch.hip).
// A bijection of [0, n) for every n.
__device__ __forceinline__ int xcd_agent(int b, int n)
{
    const int q = n >> 3, r = n & 7, x = b & 7;
    return x * q + min(x, r) + (b >> 3);
}

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
// NV independent wave reductions interleaved stage by stage (one DPP/permlane latency per
// stage for all of them); bit i of MX selects max (1) or sum (0) for v[i].
template <int NV, unsigned MX>
__device__ __forceinline__ void wred(double (&v)[NV])
{
#define SRB_RED_STAGE(GET)                                                                      \
    _Pragma("unroll") for (int i = 0; i < NV; i++) {                                            \
        const double t_ = GET;                                                                  \
        v[i] = ((MX >> i) & 1u) ? fmax(v[i], t_) : v[i] + t_;                                   \
    }
    SRB_RED_STAGE(dpp_d<0xB1>(v[i]))
    SRB_RED_STAGE(dpp_d<0x4E>(v[i]))
    SRB_RED_STAGE(dpp_d<0x141>(v[i]))
    SRB_RED_STAGE(dpp_d<0x140>(v[i]))
#undef SRB_RED_STAGE
#pragma unroll
    for (int i = 0; i < NV; i++) {
        double a, b;
        swap_d<16>(v[i], a, b);
        v[i] = ((MX >> i) & 1u) ? fmax(a, b) : a + b;
    }
#pragma unroll
    for (int i = 0; i < NV; i++) {
        double a, b;
        swap_d<32>(v[i], a, b);
        v[i] = ((MX >> i) & 1u) ? fmax(a, b) : a + b;
    }
}
// wred over all NW waves of the workgroup: per-wave DPP reduction, then lane 0 of every wave
// publishes to `scr` (NW x NV doubles, one scratch block per call site) and every thread
// combines the NW partials in the same order (identical results on every lane and wave).
template <int NV, unsigned MX, int NW>
__device__ __forceinline__ void wred_x(double (&v)[NV], double *scr, int tid)
{
    wred<NV, MX>(v);
    if constexpr (NW > 1) {
        if ((tid & 63) == 0)
#pragma unroll
            for (int i = 0; i < NV; i++) scr[(tid >> 6) * NV + i] = v[i];
        __syncthreads();
#pragma unroll
        for (int i = 0; i < NV; i++) {
            double r = scr[i];
#pragma unroll
            for (int w = 1; w < NW; w++) r = ((MX >> i) & 1u) ? fmax(r, scr[w * NV + i]) : r + scr[w * NV + i];
            v[i] = r;
        }
    }
}
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

// value of lane k of this lane's 16-lane row: one v_mov_b64_dpp row_newbcast:k (gfx90a+),
// a VALU result the next instruction can consume -- no SGPR round trip as with readlane.
// k must fold to a constant (unrolled loops).
// (row_newbcast writes every lane, so the "old" operand is never used: passing v with bound_ctrl
// lets the compiler emit the DPP move alone, without first zeroing its destination)
__device__ __forceinline__ double bc16(double v, int k)
{
    switch (k) {
#define SRB_BC(K) case K: return __builtin_amdgcn_update_dpp(v, v, 0x150 + K, 0xf, 0xf, true);
    SRB_BC(0) SRB_BC(1) SRB_BC(2) SRB_BC(3) SRB_BC(4) SRB_BC(5) SRB_BC(6) SRB_BC(7)
    SRB_BC(8) SRB_BC(9) SRB_BC(10) SRB_BC(11) SRB_BC(12) SRB_BC(13) SRB_BC(14) default: SRB_BC(15)
#undef SRB_BC
    }
}

// --------------------------------------------------------------------------- Gauss-Jordan
// In-place inverse of the nz x nz SPD matrix held one row per lane (lane i: A[0..NZL)),
// rows/columns >= nz padded with the identity.  Step k broadcasts the pivot row by
// v_readlane and every other lane eliminates column k from its row; the pivot row itself is
// not scaled (each lane keeps 1 / its own pivot and scales its row once at the end), so a
// step is one multiplier and one FMA per entry.  The pivots are those of LDL' in natural
// order, so pivot <= 0 <=> not positive definite; regularise != 0 applies iSWIFT's dynamic
// pivot regularisation (ldl.c:320-321: |D_kk| <= 1e-14 -> 1e-7).  Returns 0 on success.
// Rows may be replicated: with NZL <= 16 (and SRB_USE_DPP) every 16-lane row of the wave holds
// the whole matrix (lane l: matrix row l & 15) for the DPP solves that follow (la_solve); the
// broadcasts read the first copy, and each copy applies the same operations (bit-identical).
// A DPP row_newbcast form of this elimination (gj_invert_dpp) measured slower on MI355X: 3546
// against 3062 cycles for NZL = 12 (tools/ubench/gj_bench.hip), since readlane broadcasts land
// in SGPRs that the row updates read for free while the DPP copies cost a VALU move each.
#ifndef SRB_KKT_FP32          // diagnostic build: reduced Newton matrix inverted in fp32 (make fp32)
#define SRB_KKT_FP32 0
#endif
__device__ __forceinline__ float readlane_f(float v, int lane)
{
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
// the fp32 form of gj_invert below (same steps), on the matrix rounded to fp32
template <int NZL>
__device__ __forceinline__ int gj_invert_f32(double (&Ad)[NZL], int lane, int regularise)
{
    float A[NZL];
#pragma unroll
    for (int j = 0; j < NZL; j++) A[j] = (float)Ad[j];
    int fail = 0;
    float cs = 1.0f;
#pragma unroll
    for (int k = 0; k < NZL; k++) {
        float piv = readlane_f(A[k], k);
        if (regularise && piv <= 1e-14f && piv == piv) piv = 1e-7f;
        fail |= !(piv > 0.0f);
        const float inv = 1.0f / piv;
        float rk[NZL];
#pragma unroll
        for (int j = 0; j < NZL; j++) rk[j] = (j == k) ? 0.0f : readlane_f(A[j], k);
        const bool me = lane == k;
        const float f = me ? 0.0f : A[k] * inv;
#pragma unroll
        for (int j = 0; j < NZL; j++)
            if (j != k) A[j] = fmaf(-f, rk[j], A[j]);
        A[k] = me ? 1.0f : -f;
        cs = me ? inv : cs;
    }
#pragma unroll
    for (int j = 0; j < NZL; j++) Ad[j] = (double)(A[j] * cs);
    return fail;
}

template <int NZL, int NZE = NZL>
__device__ __forceinline__ int gj_invert(double (&A)[NZL], int nz, int lane, int regularise)
{
    if constexpr (NZL <= 16 && SRB_USE_DPP) lane &= 15;
    if constexpr (SRB_KKT_FP32) return gj_invert_f32<NZL>(A, lane, regularise);
    // All NZE steps run (the identity padding makes steps >= nz exact no-ops), so the whole
    // elimination is one basic block: the scheduler overlaps step k's row updates with the
    // broadcast of row k+1, whose entries are updated first.  NZE: the instance's nz when its shape
    // is compiled in (columns >= NZE are identity padding, never touched), else NZL.
    static_assert(NZE <= NZL, "NZE");
    int fail = 0;
    double cs = 1.0;
#pragma unroll
    for (int k = 0; k < NZE; k++) {
        double piv = readlane_d(A[k], k);
        if (regularise && piv <= 1e-14 && piv == piv) piv = 1e-7;
        fail |= !(piv > 0.0);
        const double inv = rcp_d(piv);
        double rk[NZL];
#pragma unroll
        for (int j = 0; j < NZE; j++) rk[j] = (j == k) ? 0.0 : readlane_d(A[j], k);
        const bool me = lane == k;
        const double f = me ? 0.0 : A[k] * inv;
#pragma unroll
        for (int jj = 0; jj < NZE; jj++) {
            const int j = (k + 1 + jj) % NZE;           // next pivot row's entries first
            if (j != k) A[j] = fma(-f, rk[j], A[j]);
        }
        A[k] = me ? 1.0 : -f;
        cs = me ? inv : cs;
    }
#pragma unroll
    for (int j = 0; j < NZL; j++) A[j] *= cs;
    return fail;
}

// value of v in 16-lane row G (compile-time) of the wave, same position in the row: two
// permlane swap stages (32-lane halves, then row pairs) with compile-time half selection
template <int G>
__device__ __forceinline__ double from_row(double v)
{
    double a, b;
    swap_d<32>(v, a, b);                    // a: lane l & 31, b: lane (l & 31) | 32
    const double t = (G & 2) ? b : a;
    swap_d<16>(t, a, b);                    // a: lane l & ~16, b: lane l | 16
    return (G & 1) ? b : a;
}

// The same elimination as gj_invert on a matrix replicated in each 16-lane row (NZL <= 16,
// lane l: row i = l & 15), with the columns split over the four copies instead of repeated:
// row g of the wave (g = l >> 4) updates only columns j = 4c + g, c < NZL / 4.  A step is then
// NZL / 4 DPP row_newbcast reads of the pivot row and NZL / 4 FMAs per lane, plus one
// cross-row fetch of column k (from_row, overlapping the pivot reciprocal), where gj_invert
// issues 2 NZL readlanes and NZL FMAs.  Every entry sees the same operations in the same
// order (bit-identical to gj_invert); the rows are reassembled at the end, so the result is
// replicated exactly as gj_invert leaves it.  Callers must hold the replicated layout.
template <int NZL>
__device__ __forceinline__ int gj_invert_split(double (&A)[NZL], int lane, int regularise)
{
    static_assert(NZL <= 16 && NZL % 4 == 0, "four column groups of a 16-lane row");
    constexpr int NC = NZL / 4;
    const int i = lane & 15, g = lane >> 4;
    double B[NC];
#pragma unroll
    for (int c = 0; c < NC; c++)
        B[c] = (g == 0) ? A[4 * c] : (g == 1) ? A[4 * c + 1] : (g == 2) ? A[4 * c + 2] : A[4 * c + 3];
    int fail = 0;
    double cs = 1.0;
#pragma unroll
    for (int k = 0; k < NZL; k++) {
        const int gk = k & 3, ck = k >> 2;
        // column k of this lane's row (held by row gk of the wave), fetched while the pivot's
        // reciprocal is formed
        double colk;
        switch (gk) {
        case 0: colk = from_row<0>(B[ck]); break;
        case 1: colk = from_row<1>(B[ck]); break;
        case 2: colk = from_row<2>(B[ck]); break;
        default: colk = from_row<3>(B[ck]); break;
        }
        double piv = readlane_d(B[ck], 16 * gk + k);
        if (regularise && piv <= 1e-14 && piv == piv) piv = 1e-7;
        fail |= !(piv > 0.0);
        const double inv = rcp_d(piv);
        const bool me = i == k;
        const double f = me ? 0.0 : colk * inv;
#pragma unroll
        for (int cc = 0; cc < NC; cc++) {
            const int c = (((k + 1) >> 2) + cc) % NC;       // the next pivot's column first
            const double upd = fma(-f, bc16(B[c], k), B[c]);
            B[c] = (c == ck && g == gk) ? (me ? 1.0 : -f) : upd;
        }
        cs = me ? inv : cs;
    }
#pragma unroll
    for (int c = 0; c < NC; c++) {
        const double v = B[c] * cs;
        A[4 * c + 0] = from_row<0>(v);
        A[4 * c + 1] = from_row<1>(v);
        A[4 * c + 2] = from_row<2>(v);
        A[4 * c + 3] = from_row<3>(v);
    }
    return fail;
}

// NZL <= 16: the matrix is replicated in each 16-lane row of the wave (lane l holds matrix
// row l & 15) and step k broadcasts the pivot row by DPP row_newbcast:k -- one VALU move per
// entry that the row update consumes directly, so a step's critical path is the pivot's
// broadcast, reciprocal and multiplier, not the v_readlane -> SGPR -> VALU latency.  Same
// arithmetic as the readlane form above (bit-identical results).
template <int NZL>
__device__ __forceinline__ int gj_invert_dpp(double (&A)[NZL], int lane, int regularise)
{
    static_assert(NZL <= 16, "row_newbcast reaches within 16 lanes");
    const int r = lane & 15;
    int fail = 0;
    double cs = 1.0;
#pragma unroll
    for (int k = 0; k < NZL; k++) {
        double piv = bc16(A[k], k);
        if (regularise && piv <= 1e-14 && piv == piv) piv = 1e-7;
        fail |= !(piv > 0.0);
        const double inv = rcp_d(piv);
        const bool me = r == k;
        const double f = me ? 0.0 : A[k] * inv;
#pragma unroll
        for (int jj = 0; jj < NZL; jj++) {
            const int j = (k + 1 + jj) % NZL;           // next pivot row's entries first
            if (j != k) A[j] = fma(-f, bc16(A[j], k), A[j]);
        }
        A[k] = me ? 1.0 : -f;
        cs = me ? inv : cs;
    }
#pragma unroll
    for (int j = 0; j < NZL; j++) A[j] *= cs;
    return fail;
}

// --------------------------------------------------------------------------- kNN
// (d, index) lexicographic wave argmin; every lane gets the winner
__device__ __forceinline__ void lexmin(double &d, int &idx, double od, int oi)
{
    if (od < d || (od == d && oi < idx)) { d = od; idx = oi; }
}
__device__ __forceinline__ void wargmin(double &d, int &idx)
{
    // the wsum pattern (DPP within 16-lane rows, permlane swaps across them) on the pair
#define SRB_ARG_DPP(CTRL) lexmin(d, idx, dpp_d<CTRL>(d), __builtin_amdgcn_update_dpp(0, idx, CTRL, 0xf, 0xf, false))
    SRB_ARG_DPP(0xB1); SRB_ARG_DPP(0x4E); SRB_ARG_DPP(0x141); SRB_ARG_DPP(0x140);
#undef SRB_ARG_DPP
    double a, b;
    swap_d<16>(d, a, b);
    auto i16 = __builtin_amdgcn_permlane16_swap((unsigned)idx, (unsigned)idx, false, false);
    d = a; idx = (int)i16[0]; lexmin(d, idx, b, (int)i16[1]);
    swap_d<32>(d, a, b);
    auto i32 = __builtin_amdgcn_permlane32_swap((unsigned)idx, (unsigned)idx, false, false);
    d = a; idx = (int)i32[0]; lexmin(d, idx, b, (int)i32[1]);
}

// The same (d, index) lexicographic wave argmin as wargmin, by a double minimum and a ballot (round 6,
// tools/ubench/knn_phase.hip): one fmin per stage instead of the pair's three compares and three selects;
// the index comes from the one lane holding the minimum (v_readlane), or -- when several lanes hold it: an
// exact distance tie, or every head exhausted (+inf) -- from an integer minimum over those lanes' indices.
// Every lane ends with the same (d, idx).  d is never NaN here (knn_select_k offers no NaN keys).
__device__ __forceinline__ int wmin_i(int v)
{
    v = min(v, __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_update_dpp(0, v, 0x141, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_update_dpp(0, v, 0x140, 0xf, 0xf, false));
    auto p16 = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
    v = min((int)p16[0], (int)p16[1]);
    auto p32 = __builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false);
    return min((int)p32[0], (int)p32[1]);
}
__device__ __forceinline__ void wargmin_b(double &d, int &idx)
{
    const double m = wmin(d);
    const unsigned long long tie = __ballot(d == m);
    int w;
    if (__popcll(tie) == 1) w = __builtin_amdgcn_readlane(idx, __ffsll((long long)tie) - 1);
    else w = wmin_i((d == m) ? idx : 0x7fffffff);
    d = m; idx = w;
}

// wargmin over the NW waves of the workgroup: per-wave DPP argmin, lane 0 of every wave
// publishes (d, idx) to scr[2 NW], every thread combines the partials in wave order
template <int NW>
__device__ __forceinline__ void wargmin_x(double &d, int &idx, double *scr, int tid)
{
    wargmin(d, idx);
    if constexpr (NW > 1) {
        if ((tid & 63) == 0) { scr[2 * (tid >> 6)] = d; scr[2 * (tid >> 6) + 1] = (double)idx; }
        __syncthreads();
        d = scr[0]; idx = (int)scr[1];
#pragma unroll
        for (int w = 1; w < NW; w++) lexmin(d, idx, scr[2 * w], (int)scr[2 * w + 1]);
    }
}

// Uniform grid over the rows of a table (SURVEY 8(a) row a10 at swarm scale): built on the
// device each launch by srb_grid_build_kernel for tables of SRB_GRID_MIN_ROWS rows or more.
// Cells row-major (cy * nx + cx), rows of finite coordinates sorted by cell (the order inside
// a cell is arbitrary -- the selection order below is exact whatever it is).
struct SrbGrid {
    double x0, y0, inv_h, h;       // origin and cell size
    int nx, ny, n;                 // cells per axis, rows in the grid
    int ok;                        // 0: not built (brute-force scan)
};

// rows a lane holds in registers on the thresholded brute-force path of knn_select_k (larger tables: the
// batched scan); 32: the neighbour snapshot of a 2048-agent shard on one wave
#ifndef SRB_KNN_RB
#define SRB_KNN_RB 32
#endif

// per-lane insertion of candidate (cd = sqrt distance, ci = row) into the sorted top-K
// (bd, bi), ordered lexicographically by (distance, index)
template <int KM>
__device__ __forceinline__ void knn_insert(double (&bd)[KM], int (&bi)[KM], double cd, int ci, int K)
{
#pragma unroll
    for (int j = 0; j < KM; j++) {
        const bool lt = (j < K) && (cd < bd[j] || (cd == bd[j] && ci < bi[j]));
        const double td = bd[j]; const int ti = bi[j];
        bd[j] = lt ? cd : td; bi[j] = lt ? ci : ti;
        cd = lt ? td : cd; ci = lt ? ti : ci;
    }
}

// The thresholded brute-force pass of knn_select_k (round 6) over a table of at most RB rows a lane: every
// row's d^2 kept in registers (row tid + r STEP in slot r; NaN for the agent itself, rows past the table and
// rows with NaN coordinates, which are never selected), then a bound T on the K-th smallest d^2 from the lanes'
// minima -- the K-th smallest of them: at least K rows of this wave lie within it -- and only the rows with
// d^2 <= T (1 + 1e-14) (the filter's padding: a row beyond cannot round to a sqrt at or below the K-th's)
// enter the lanes' sorted lists, each lane taking its candidates one per trip.  The per-row insertion was
// three quarters of the neighbour scan (tools/ubench/knn_phase.hip); configs[2] selection 20.6 -> 14.5 us.
template <int KM, int RB, int STEP>
__device__ __forceinline__ void knn_thresh(int tid, double px, double py, const double *__restrict__ tab, int stride,
                                           int n_rows, int self, int K, double (&bd)[KM], int (&bi)[KM])
{
#pragma clang fp contract(off)
    double key[RB];
#pragma unroll
    for (int r = 0; r < RB; r++) {
        const int i = tid + r * STEP;
        const bool in = i < n_rows;
        const double tx = in ? tab[(size_t)stride * i] : 0.0, ty = in ? tab[(size_t)stride * i + 1] : 0.0;
        const double dx = px - tx, dy = py - ty;
        key[r] = (in && i != self) ? dx * dx + dy * dy : __builtin_nan("");
    }
    double lm = __builtin_inf();
#pragma unroll
    for (int r = 0; r < RB; r++) lm = fmin(lm, key[r]);      // NaN keys ignored
    double T = __builtin_inf();
    for (int cnt = 0; cnt < K;) {                  // uniform: every lane holds the same t
        const double t = wmin(lm);
        if (!(t < __builtin_inf())) { T = __builtin_inf(); break; }
        cnt += __popcll(__ballot(lm == t));
        T = t;
        lm = (lm == t) ? __builtin_inf() : lm;
    }
    const double wT = (T < __builtin_inf()) ? T * (1.0 + 1e-14) : __builtin_inf();
    unsigned long long cm = 0;
#pragma unroll
    for (int r = 0; r < RB; r++)
        if (key[r] <= wT) cm |= 1ull << r;         // NaN keys fail
    while (__ballot(cm != 0)) {
        if (cm) {
            const int rr = __ffsll((long long)cm) - 1;
            cm &= cm - 1;
            double kd = key[0];
#pragma unroll
            for (int r = 1; r < RB; r++) kd = (rr == r) ? key[r] : kd;
            knn_insert<KM>(bd, bi, sqrt(kd), tid + rr * STEP, K);
        }
    }
}

// K nearest rows of a table (row i at tab[stride*i], x at +0, y at +1) to (px, py),
// ascending in (sqrt distance, index) -- the order of the reference's strict-'<' scan over
// sqrt(pow(dx,2)+pow(dy,2)) (MPC_dist.cpp:373-382; two rows whose squared distances differ
// but round to the same sqrt keep index order, as there) -- excluding row `self`; indices to
// sel[0..K).  cap != 0 applies the reference's min_dist = 1000 / min_i = 0 start: a round
// whose winner is not closer than 1000 m selects row 0.  NaN rows are never selected.
// KW waves (one workgroup) gather candidates -- every row (brute force), or with a grid the
// rows of the cells around the query that must hold the K nearest -- and each lane keeps a
// sorted top-K of its candidates; then K rounds pop the global order: a wave argmin over the
// lane heads, the KW wave winners through LDS (wd_lds, wi_lds: KW entries each), the owning
// lane drops its head (measured faster than per-wave pops followed by one merge of the KW K
// wave winners: two barriers per round cost less than K extra wave-argmin rounds).  The sqrt
// is taken only for rows that can enter a lane's list: d^2 above its K-th entry's squared key
// by more than a relative 1e-14 cannot round to a smaller sqrt.
template <int KW, int KM>
__device__ __forceinline__ void knn_select_k(int tid, double px, double py, const double *__restrict__ tab,
                                           int stride, int n_rows, int self, int K, int cap, int *sel,
                                           double *wd_lds, int *wi_lds, const SrbGrid *grid = nullptr,
                                           const int *__restrict__ cell_off = nullptr,
                                           const double2 *__restrict__ spos = nullptr,
                                           const int *__restrict__ sidx = nullptr)
{
#pragma clang fp contract(off)
    const int lane = tid & 63, wv = tid >> 6;
    double bd[KM]; int bi[KM];
#pragma unroll
    for (int j = 0; j < KM; j++) { bd[j] = __builtin_inf(); bi[j] = 0x7fffffff; }
    double wq = __builtin_inf();                   // filter bound on d^2 (K-th key squared, padded)
    constexpr int STEP = 64 * KW;
    auto offer = [&](double tx, double ty, int i) {
        const double dx = px - tx, dy = py - ty;
        const double d2 = dx * dx + dy * dy;
        if (i == self || !(d2 <= wq)) return;
        knn_insert<KM>(bd, bi, sqrt(d2), i, K);
#pragma unroll
        for (int j = 0; j < KM; j++)
            if (j == K - 1) wq = bd[j] * bd[j] * (1.0 + 1e-14);
    };
    // ---- grid search: the smallest Chebyshev ring r0 of cells around the query cell holding
    // K candidates bounds the K-th distance by (r0 + 1) sqrt(2) h, so every row closer than
    // that lies in the ring R = ceil((r0 + 1) sqrt 2) + 1; queries far outside the grid (or a
    // grid that cannot supply K rows) fall back to the brute-force scan
    bool done = false;
    if (grid && grid->ok) {
        const SrbGrid g = *grid;
        const double fx = floor((px - g.x0) * g.inv_h), fy = floor((py - g.y0) * g.inv_h);
        const int keff = K + (self >= 0 ? 1 : 0);
        if (g.n >= keff && fx > -64.0 && fy > -64.0 && fx < g.nx + 64.0 && fy < g.ny + 64.0) {
            const int cx = (int)fx, cy = (int)fy, rmax = max(g.nx, g.ny) + 64;
            auto rows_in = [&](int r, int y) -> int {        // rows of cell-row y within x-range of ring r
                const int xl = max(cx - r, 0), xr = min(cx + r, g.nx - 1);
                if (y < 0 || y >= g.ny || xl > xr) return 0;
                return cell_off[y * g.nx + xr + 1] - cell_off[y * g.nx + xl];
            };
            // rings 0..3 in one pass (lane l < 16 counts cell row y = cy + l - r(r+1) of ring
            // r = floor(sqrt(l))), then ring by ring from 4 if none of them holds keff rows
            int r0 = 4;
            {
                const int rr = (lane < 1) ? 0 : (lane < 4) ? 1 : (lane < 9) ? 2 : (lane < 16) ? 3 : -1;
                const int v = (rr >= 0) ? rows_in(rr, cy + lane - rr * rr - rr) : 0;
#pragma unroll
                for (int r = 3; r >= 0; r--) {
                    int cr = (rr == r) ? v : 0;
                    for (int o = 32; o > 0; o >>= 1) cr += __shfl_xor(cr, o, 64);
                    if (cr >= keff) r0 = r;
                }
            }
            for (; r0 >= 4 && r0 < rmax; r0++) {            // uniform: every thread computes the same count
                int cnt = 0;
                for (int y = cy - r0 + lane; y <= cy + r0; y += 64) cnt += rows_in(r0, y);
                for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
                if (cnt >= keff) break;
            }
            if (r0 < rmax) {
                const int R = (int)ceil((r0 + 1) * 1.4142135623730951) + 1;
                const int ylo = max(cy - R, 0), yhi = min(cy + R, g.ny - 1);
                const int xl = max(cx - R, 0), xr = min(cx + R, g.nx - 1);
                // up to 64 cell rows at a time: lane y loads its row's range [a, a + len), a wave
                // scan numbers the candidates, and every thread takes candidates c, c + STEP, ..
                // (segment found by a binary search over the scan), so the cell-offset loads and
                // the row loads are two dependent round trips instead of two per cell row
                for (int yb = ylo; xl <= xr && yb <= yhi; yb += 64) {
                    const int y = yb + lane;
                    int a = 0, len = 0;
                    if (y <= yhi) { a = cell_off[y * g.nx + xl]; len = cell_off[y * g.nx + xr + 1] - a; }
                    int inc = len;
#pragma unroll
                    for (int o = 1; o < 64; o <<= 1) { const int v = __shfl_up(inc, o, 64); if (lane >= o) inc += v; }
                    const int total = __shfl(inc, 63, 64), exc = inc - len;
                    for (int c0 = 64 * wv; c0 < total; c0 += STEP) {      // wave-uniform trip count
                        const int c = c0 + lane;
                        int j = 0;                                        // last lane with exc <= c
#pragma unroll
                        for (int st = 32; st > 0; st >>= 1) j += (__shfl(exc, j + st, 64) <= c) ? st : 0;
                        const int i = __shfl(a, j, 64) + (c - __shfl(exc, j, 64));
                        if (c < total) {
                            const double2 q = spos[i];
                            offer(q.x, q.y, sidx[i]);
                        }
                    }
                }
                done = true;
            }
        }
    }
    if (!done && n_rows <= STEP * SRB_KNN_RB) {
        // ---- brute force with a threshold (knn_thresh), as many register slots as the table needs
        if (n_rows <= STEP * 4) knn_thresh<KM, 4, STEP>(tid, px, py, tab, stride, n_rows, self, K, bd, bi);
        else if (n_rows <= STEP * 16) knn_thresh<KM, 16, STEP>(tid, px, py, tab, stride, n_rows, self, K, bd, bi);
        else knn_thresh<KM, SRB_KNN_RB, STEP>(tid, px, py, tab, stride, n_rows, self, K, bd, bi);
        done = true;
    }
    if (!done) {
        // ---- brute force: KNN_U rows per lane per batch, all loads issued before the first use
#ifndef SRB_KNN_U
#define SRB_KNN_U 4
#endif
        constexpr int KNN_U = SRB_KNN_U;
        for (int i0 = tid; i0 < n_rows; i0 += KNN_U * STEP) {
            double tx[KNN_U], ty[KNN_U];
#pragma unroll
            for (int u = 0; u < KNN_U; u++) {
                const int i = i0 + u * STEP;
                const bool in = i < n_rows;
                tx[u] = in ? tab[(size_t)stride * i] : 0.0;
                ty[u] = in ? tab[(size_t)stride * i + 1] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < KNN_U; u++)
                if (i0 + u * STEP < n_rows) offer(tx[u], ty[u], i0 + u * STEP);
        }
    }
    // round j's winner is kept by lane j and stored after the last round: a store inside the
    // loop would make every barrier wait for it (s_waitcnt vmcnt(0) before s_barrier)
    int mine = -1;
#pragma clang loop unroll(disable)
    for (int j = 0; j < K; j++) {
        double d = bd[0]; int idx = bi[0];
        wargmin_b(d, idx);
        if (KW > 1) {
            if (lane == 0) { wd_lds[wv] = d; wi_lds[wv] = idx; }
            __syncthreads();
#pragma unroll
            for (int w = 0; w < KW; w++) {
                const double od = wd_lds[w]; const int oi = wi_lds[w];
                if (od < d || (od == d && oi < idx)) { d = od; idx = oi; }
            }
            __syncthreads();                       // every wave has read the winners
        }
        if (bi[0] == idx) {
#pragma unroll
            for (int t = 0; t + 1 < KM; t++) { bd[t] = bd[t + 1]; bi[t] = bi[t + 1]; }
            bd[KM - 1] = __builtin_inf(); bi[KM - 1] = 0x7fffffff;
        }
        if (tid == j) mine = cap ? ((d < 1000.0) ? idx : 0) : ((idx == 0x7fffffff) ? -1 : idx);
    }
    if (tid < K) sel[tid] = mine;
}
// the insertion network as deep as K needs (K <= KM): 4, 8 or SRB_KNN_MAX entries
template <int KW>
__device__ __forceinline__ void knn_select(int tid, double px, double py, const double *__restrict__ tab,
                                           int stride, int n_rows, int self, int K, int cap, int *sel,
                                           double *wd_lds, int *wi_lds, const SrbGrid *grid = nullptr,
                                           const int *cell_off = nullptr, const double2 *spos = nullptr,
                                           const int *sidx = nullptr)
{
    if (K <= 4) knn_select_k<KW, 4>(tid, px, py, tab, stride, n_rows, self, K, cap, sel, wd_lds, wi_lds, grid, cell_off, spos, sidx);
    else if (K <= 8) knn_select_k<KW, 8>(tid, px, py, tab, stride, n_rows, self, K, cap, sel, wd_lds, wi_lds, grid, cell_off, spos, sidx);
    else knn_select_k<KW, SRB_KNN_MAX>(tid, px, py, tab, stride, n_rows, self, K, cap, sel, wd_lds, wi_lds, grid, cell_off, spos, sidx);
}
