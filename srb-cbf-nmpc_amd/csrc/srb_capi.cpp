// Host side of the C ABI declared in include/srbnmpc.h.
//
// The context owns device staging buffers sized for max_agents, one HIP stream and a
// pair of events around each kernel, so bench.py can time the kernels on the stream
// they actually run on.  Per-call work on the host is only the (tiny) LIP
// discretisation shared by every agent and the launch.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <string>
#include "srbnmpc.h"
#include "srb_kernel_params.h"

#define DECL_NMPC(NZL, TS, NW, NC, CC, KC)                                                                    \
    extern "C" __global__ void srb_nmpc_kernel_##NZL##_##TS##_##NW##_##NC##_##CC##_##KC(                     \
        SrbKParams prm, int n_agents, const double *x0g, const double *refg, const double *footg,              \
        const double *obstacles, int n_obs, const double *nbr_state, int n_all, int agent_offset,              \
        double *x_qp_out, double *x_out, double *obj_out, int *status_out, int *iters_out,                    \
        const double *alpha_buf, double *alpha_out, const int *sel_g, float *zpol_g, int zstride);            \
    extern "C" __global__ void srb_polish_kernel_##NZL##_##TS##_##NW##_##NC##_##CC##_##KC(                   \
        SrbKParams prm, int n_agents, const double *x0g, const double *refg, const double *footg,              \
        const double *obstacles, const double *nbr_state, double *x_out, double *obj_out, int *status_out,     \
        const double *alpha_buf, double *alpha_out, const int *sel_g, const float *zpol_g, int zstride);
SRB_KERNEL_INSTANCES(DECL_NMPC)
#undef DECL_NMPC
#define DECL_NMPC_F32(NZL, TS, NW, NC, CC, KC)                                                                \
    extern "C" __global__ void srb_nmpc_kernel_f32_##NZL##_##TS##_##NW##_##NC##_##CC##_##KC(                 \
        SrbKParams prm, int n_agents, const double *x0g, const double *refg, const double *footg,              \
        const double *obstacles, int n_obs, const double *nbr_state, int n_all, int agent_offset,              \
        double *x_qp_out, double *x_out, double *obj_out, int *status_out, int *iters_out,                    \
        const double *alpha_buf, double *alpha_out, const int *sel_g, float *zpol_g, int zstride);
SRB_KF32_INSTANCES(DECL_NMPC_F32)
#undef DECL_NMPC_F32

typedef void (*srb_kernel_fn)(SrbKParams, int, const double *, const double *, const double *, const double *, int,
                              const double *, int, int, double *, double *, double *, int *, int *, const double *,
                              double *, const int *, float *, int);
typedef void (*srb_polish_fn)(SrbKParams, int, const double *, const double *, const double *, const double *,
                              const double *, double *, double *, int *, const double *, double *, const int *,
                              const float *, int);
struct SrbGrid;
extern "C" __global__ void srb_knn_kernel(int n_agents, const double *x0g, const double *obstacles, int n_obs,
                                          const double *nbr_state, int n_all, int agent_offset, int K_obs, int K_nbr,
                                          int *sel_out, int sel_stride, const SrbGrid *gob, const int *oob, const double2 *pob,
                                          const int *iob, const SrbGrid *gnb, const int *onb, const double2 *pnb,
                                          const int *inb);
extern "C" __global__ void srb_grid_build_kernel(const double *tab0, int stride0, int n0, SrbGrid *g0, int *off0,
                                                 double2 *spos0, int *sidx0, const double *tab1, int stride1, int n1,
                                                 SrbGrid *g1, int *off1, double2 *spos1, int *sidx1);
struct srb_instance { int nzl, ts, nw, nc, cc, kc; srb_kernel_fn fn; srb_polish_fn polish; };
#define ENTRY_NMPC(NZL, TS, NW, NC, CC, KC)                                                                   \
    {NZL, TS, NW, NC, CC, KC, srb_nmpc_kernel_##NZL##_##TS##_##NW##_##NC##_##CC##_##KC,                       \
     srb_polish_kernel_##NZL##_##TS##_##NW##_##NC##_##CC##_##KC},
static const srb_instance g_instances[] = {SRB_KERNEL_INSTANCES(ENTRY_NMPC)};
#undef ENTRY_NMPC
// the fp32-factor variant of an instance (SRB_OPT_KKT_FP32_MU > 0), or null
struct srb_instance_f32 { int nzl, ts, nw, nc, cc, kc; srb_kernel_fn fn; };
#define ENTRY_F32(NZL, TS, NW, NC, CC, KC) {NZL, TS, NW, NC, CC, KC, srb_nmpc_kernel_f32_##NZL##_##TS##_##NW##_##NC##_##CC##_##KC},
static const srb_instance_f32 g_instances_f32[] = {SRB_KF32_INSTANCES(ENTRY_F32)};
#undef ENTRY_F32
static srb_kernel_fn f32_variant(const srb_instance *in)
{
    for (const srb_instance_f32 &v : g_instances_f32)
        if (v.nzl == in->nzl && v.ts == in->ts && v.nw == in->nw && v.nc == in->nc && v.cc == in->cc && v.kc == in->kc) return v.fn;
    return nullptr;
}

// Waves per agent: small batches (up to one agent per CU) spread each agent over the four
// SIMDs of a CU (NW = 4) for latency; larger batches run one wave per agent so that agents,
// not waves of one agent, fill the SIMDs.
static int g_cu_count = 0;
static size_t g_lds_max = 160 * 1024;   // gfx950 LDS per CU; the device's sharedMemPerBlock once known
// Waves per agent: small batches (up to one agent per CU) spread each agent over the four
// SIMDs of a CU (NW = 4) for latency; larger batches run one wave per agent so that agents,
// not waves of one agent, fill the SIMDs -- except large problems (more than five row slots per
// lane with one wave, e.g. N = 20), where one wave spills its registers and two waves per agent
// are 1.8x faster (profiles/r01_nw_tuning.txt).  srb_ctx_set_waves overrides.  (No environment
// variable changes what the product library computes: every knob is a context setting.)
static int wanted_waves(int n_agents, int slots, int ctx_nw)
{
    if (ctx_nw == 1 || ctx_nw == 2 || ctx_nw == 4) return ctx_nw;
    if (g_cu_count > 0 && n_agents <= g_cu_count) return 4;
    return (slots > 5 * 64) ? 2 : 1;
}

static const srb_instance *pick_instance(const SrbKParams &k, int nw = 1)
{
    const int S = srb_slots(k.N, k.C, k.K_obs + k.K_nbr);
    for (int pass = 0; pass < 3; pass++) {
        const int want = pass == 0 ? nw : pass == 1 ? (nw == 4 ? 2 : 1) : 1;
        for (const srb_instance &in : g_instances)
            if (in.nw == want && in.nzl >= k.nz && 64 * in.nw * in.ts >= S &&
                (in.nc == 0 || in.nc == k.N) && (in.cc == 0 || in.cc == k.C) &&
                (in.kc == 0 || in.kc == k.K_obs + k.K_nbr) &&
                (size_t)srb_lds_doubles(k, in.nzl, in.nw) * sizeof(double) <= g_lds_max)
                return &in;
    }
    return nullptr;
}

static thread_local std::string g_err;

static int fail(int code, const std::string &msg)
{
    g_err = msg;
    return code;
}

// shared with srb_ll_capi.cpp
int srb_internal_fail(int code, const char *msg) { return fail(code, msg); }

#define HIPCHK(expr)                                                                   \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess) return fail(SRB_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

struct srb_ctx {
    srb_params p;
    int max_agents, device;
    hipStream_t stream;
    hipEvent_t ev[4];
    hipEvent_t done;               // recorded after every call's work (submission-order chaining)
    hipStream_t last;              // stream of the previous call
    bool any;                      // a call has been submitted (done is valid)
    // device staging
    double *x0, *ref, *foot, *obstacles, *nbr, *x_qp, *x, *obj, *abuf, *alpha;
    int *status, *iters;
    int *sel;                      // [max_agents][2 SRB_KNN_MAX] selected obstacle / neighbour rows
    size_t cap_obs, cap_nbr;
    float knn_ms, solve_ms;
    bool timed;
    int last_nw;
    int nw;                        // waves per agent forced by srb_ctx_set_waves (0: automatic)
    int qp_init;                   // QP starting point (srb_ctx_set_qp_init): 1 scaled (default), 0 iSWIFT
    // srb_ctx_set_option (SRB_OPT_*): the polish of the NLP result on/off, its penalty and waves per
    // agent, the selection-grid thresholds
    int polish, polish_waves, grid_min_rows, grid_min_rows_static, polish_fused;
    int last_polish;               // how the last launch polished: 0 no, 1 polish kernel, 2 fused
    int timing;                    // 1: HIP events around the kernels (srb_last_kernel_ms); 0: none
    int selection;                 // SRB_OPT_SELECTION: 1 the solve launches the selection, 0 the caller did
    int last_f32;                  // the last launch ran an fp32-factor instance (SRB_OPT_LAST_KKT_FP32, read only)
    double polish_rho;
    double qp_warm_tol;            // SRB_OPT_QP_WARM_TOL
    double kkt32_mu;               // SRB_OPT_KKT_FP32_MU: fp32 factor while mu > this (0: off, the fp64 instances)
    int kkt32_ref;                 // SRB_OPT_KKT_FP32_REFINE: fp64 refinement steps per solve with the fp32 factor
    float *zpol;                   // [max_agents][zstride] NLP active set / multipliers for the polish kernel
    int zstride;
    float polish_ms;
    // selection grids (table 0: static obstacles, 1: neighbour snapshot), rebuilt per launch
    struct grid_buf { void *g; int *off; double2 *spos; int *sidx; size_t cap; } grid[2];
    const double *grid_src;        // obstacle table, row count and version the obstacle grid was built from
    int grid_n, grid_ver;
};

// Calls on one context run in submission order (include/srbnmpc.h, "Ordering"): a call on
// another stream than the previous one first waits for that call's work, so the context's
// scratch (grids, the default sel buffer, staging, timing events) never serves two launches
// in flight.
static int order_after_last(srb_ctx *c, hipStream_t s)
{
    if (c->any && s != c->last) HIPCHK(hipStreamWaitEvent(s, c->done, 0));
    return SRB_OK;
}

static int mark_done(srb_ctx *c, hipStream_t s)
{
    HIPCHK(hipEventRecord(c->done, s));
    c->last = s; c->any = true;
    return SRB_OK;
}

// device buffers of selection grid t for a table of n rows (grown on demand; the header
// starts with ok = 0, so a grid is never read before a build has filled it)
static int grid_reserve(srb_ctx *c, int t, size_t n)
{
    srb_ctx::grid_buf &b = c->grid[t];
    if (!b.g) {
        HIPCHK(hipMalloc(&b.g, 64));
        HIPCHK(hipMemset(b.g, 0, 64));
        HIPCHK(hipMalloc(&b.off, (SRB_GRID_CELLS + 1) * sizeof(int)));
    }
    if (n > b.cap) {
        if (c->any) HIPCHK(hipEventSynchronize(c->done));   // the previous launch may still read them
        if (b.spos) HIPCHK(hipFree(b.spos));
        if (b.sidx) HIPCHK(hipFree(b.sidx));
        HIPCHK(hipMalloc(&b.spos, n * sizeof(double2)));
        HIPCHK(hipMalloc(&b.sidx, n * sizeof(int)));
        b.cap = n;
    }
    return SRB_OK;
}

extern "C" void srb_params_default(srb_params *p, int N, int C)
{
    std::memset(p, 0, sizeof(*p));
    p->N = N; p->C = C; p->K_obs = 1; p->K_nbr = 0;
    p->grav = 9.81; p->hcom = 0.29; p->Ts = 43 * 0.001; p->mu = 0.7;
    p->Qw = 3e2; p->Pw = 2e3; p->Rw = 1e-1; p->Sw = 0.3e4;
    p->box = 1e3;
    p->eps_obs = (double)1.9f; p->eps_nbr = (double)2.2f; p->vsat = (double)0.35f;
    p->tol = 1e-6; p->qp_maxit = 25; p->nlp_maxit = 50; p->use_nlp = 1;
}

extern "C" int srb_nv(const srb_params *p) { return (6 + p->C) * p->N + 1; }

extern "C" int srb_abi_version(void) { return SRB_ABI_VERSION; }

static void mm4(const double *X, const double *Y, double *Z)
{
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            double s = 0;
            for (int k = 0; k < 4; k++) s += X[i * 4 + k] * Y[k * 4 + j];
            Z[i * 4 + j] = s;
        }
}

// Inverse of the 5x5 Bernstein matrix B[i][j] = C(4,j) s_i^j (1-s_i)^(4-j), s_i = i/4
// (fitComTrajectory_eventbase, MPC_dist.cpp:801-806), Gauss-Jordan with partial pivoting.
static void bernstein_inverse(double Binv[25])
{
    static const double binom[5] = {1, 4, 6, 4, 1};
    double M[5][10];
    for (int i = 0; i < 5; i++) {
        const double s = i * 0.25;
        for (int j = 0; j < 5; j++) { M[i][j] = binom[j] * std::pow(s, j) * std::pow(1 - s, 4 - j); M[i][5 + j] = (i == j); }
    }
    for (int k = 0; k < 5; k++) {
        int piv = k;
        for (int i = k + 1; i < 5; i++) if (std::fabs(M[i][k]) > std::fabs(M[piv][k])) piv = i;
        for (int j = 0; j < 10; j++) std::swap(M[k][j], M[piv][j]);
        const double inv = 1.0 / M[k][k];
        for (int j = 0; j < 10; j++) M[k][j] *= inv;
        for (int i = 0; i < 5; i++)
            if (i != k) {
                const double f = M[i][k];
                for (int j = 0; j < 10; j++) M[i][j] -= f * M[k][j];
            }
    }
    for (int i = 0; i < 5; i++)
        for (int j = 0; j < 5; j++) Binv[i * 5 + j] = M[i][5 + j];
}

// LIP discretisation MPC_dist.cpp:99-127 (Ad by third-order series, Bd = A^-1 (Ad - I) B)
static SrbKParams make_kparams(const srb_params *p, int use_nlp)
{
    SrbKParams k;
    std::memset(&k, 0, sizeof k);
    k.N = p->N; k.C = p->C; k.K_obs = p->K_obs; k.K_nbr = p->K_nbr;
    k.n = (6 + p->C) * p->N + 1;
    k.nz = p->N * (p->C - 1) + 1;
    k.mq = 4 * (p->N - 1) + 12 * p->N + 2 * p->C * p->N;
    k.use_nlp = use_nlp;
    k.qp_maxit = p->qp_maxit; k.nlp_maxit = p->nlp_maxit;
    const double w2 = p->grav / p->hcom, T = p->Ts;
    double A[16] = {0}, B[8] = {0}, A2[16], A3[16];
    A[1] = 1; A[4] = w2; A[11] = 1; A[14] = w2;
    B[2] = -w2; B[7] = -w2;
    mm4(A, A, A2); mm4(A2, A, A3);
    for (int i = 0; i < 16; i++) k.Ad[i] = (i % 5 == 0 ? 1.0 : 0.0) + A[i] * T + 0.5 * A2[i] * T * T + A3[i] * T * T * T / 6;
    double Ai[16] = {0}, AdI[16], M[16];
    Ai[1] = 1.0 / w2; Ai[4] = 1.0; Ai[11] = 1.0 / w2; Ai[14] = 1.0;
    for (int i = 0; i < 16; i++) AdI[i] = k.Ad[i] - (i % 5 == 0 ? 1.0 : 0.0);
    mm4(Ai, AdI, M);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 2; j++) {
            double s = 0;
            for (int q = 0; q < 4; q++) s += M[i * 4 + q] * B[q * 2 + j];
            k.Bd[i * 2 + j] = s;
        }
    k.Qw = p->Qw; k.Pw = p->Pw; k.Rw = p->Rw; k.Sw = p->Sw; k.box = p->box;
    k.fr = p->mu * p->hcom / std::sqrt(2.0);
    k.eps_obs = p->eps_obs; k.eps_nbr = p->eps_nbr; k.vsat = p->vsat; k.tol = p->tol; k.Ts = p->Ts;
    bernstein_inverse(k.Binv);
    return k;
}

static int validate(const srb_params *p)
{
    if (!p) return fail(SRB_ERR_ARG, "null params");
    if (p->N < 2 || p->C < 2 || p->C > 4) return fail(SRB_ERR_ARG, "need N >= 2 and 2 <= C <= 4");
    if (p->N > SRB_MAX_N) return fail(SRB_ERR_SIZE, "N exceeds 33 (CoM-CoP slots in one 64-lane trip)");
    if (p->K_obs < 0 || p->K_nbr < 0 || p->K_obs > SRB_KNN_MAX || p->K_nbr > SRB_KNN_MAX)
        return fail(SRB_ERR_ARG, "K_obs, K_nbr out of range (each <= 16)");
    if (p->N * (p->C - 1) + 1 > SRB_MAX_NZ) return fail(SRB_ERR_SIZE, "N(C-1)+1 exceeds 32 (reduced Newton system bound)");
    SrbKParams k = make_kparams(p, p->use_nlp);
    const srb_instance *in = pick_instance(k);
    if (!in) return fail(SRB_ERR_SIZE, "no kernel instance covers the row slots (n + 4N - 2 + N K <= 512)");
    if ((size_t)srb_lds_doubles(k, in->nzl, in->nw) * sizeof(double) > 160 * 1024) return fail(SRB_ERR_SIZE, "per-agent LDS exceeds 160 KiB");
    return SRB_OK;
}

extern "C" int srb_lds_bytes(const srb_params *p)
{
    SrbKParams k = make_kparams(p, p->use_nlp);
    const srb_instance *in = pick_instance(k);
    return in ? srb_lds_doubles(k, in->nzl, in->nw) * (int)sizeof(double) : -1;
}

extern "C" int srb_ctx_create(const srb_params *p, int max_agents, int device, srb_ctx **out)
{
    if (!out || max_agents <= 0) return fail(SRB_ERR_ARG, "bad arguments");
    int rc = validate(p);                 // parameter checks first (no device needed)
    if (rc) return rc;
    int ndev = 0;
    HIPCHK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(SRB_ERR_ARG, "device index out of range");
    HIPCHK(hipSetDevice(device));
    if (g_cu_count == 0) {
        hipDeviceProp_t prop;
        HIPCHK(hipGetDeviceProperties(&prop, device));
        g_cu_count = prop.multiProcessorCount;
        g_lds_max = prop.sharedMemPerBlock;
    }
    rc = validate(p);                     // again against this device's LDS per workgroup
    if (rc) return rc;
    srb_ctx *c = new srb_ctx();           // value-initialised: every buffer null until allocated
    // a failure after this point unwinds through srb_ctx_destroy; *out stays untouched
#define CREATE_CHK(expr)                                                                               \
    do {                                                                                               \
        hipError_t e_ = (expr);                                                                        \
        if (e_ != hipSuccess) {                                                                        \
            const int rc_ = fail(SRB_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_));          \
            srb_ctx_destroy(c);                                                                        \
            return rc_;                                                                                \
        }                                                                                              \
    } while (0)
    c->p = *p; c->max_agents = max_agents; c->device = device;
    c->cap_obs = 0; c->cap_nbr = 0; c->obstacles = nullptr; c->nbr = nullptr; c->timed = false; c->nw = 0; c->last_nw = 0;
    for (auto &g : c->grid) g = srb_ctx::grid_buf{nullptr, nullptr, nullptr, nullptr, 0};
    c->grid_src = nullptr; c->grid_n = 0; c->grid_ver = 0;
    c->last = nullptr; c->any = false;
    c->qp_init = 1; c->polish_ms = 0.0f;
    c->polish = SRB_POLISH_ON; c->polish_rho = SRB_POLISH_RHO; c->qp_warm_tol = SRB_QP_WARM_TOL; c->polish_waves = 0; c->polish_fused = 1; c->last_polish = 0; c->timing = 1; c->selection = 1;
    c->kkt32_mu = 0.0; c->kkt32_ref = 3;
    c->grid_min_rows = SRB_GRID_MIN_ROWS; c->grid_min_rows_static = SRB_GRID_MIN_ROWS_STATIC;
    c->zstride = 2 * srb_r4(srb_slots(p->N, p->C, p->K_obs + p->K_nbr));
    const int N = p->N, C = p->C, nv = srb_nv(p);
    const size_t A = (size_t)max_agents;
    CREATE_CHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    for (int i = 0; i < 4; i++) CREATE_CHK(hipEventCreate(&c->ev[i]));
    CREATE_CHK(hipEventCreateWithFlags(&c->done, hipEventDisableTiming));
    CREATE_CHK(hipMalloc(&c->x0, A * 4 * sizeof(double)));
    CREATE_CHK(hipMalloc(&c->ref, A * 4 * N * sizeof(double)));
    CREATE_CHK(hipMalloc(&c->foot, A * 2 * C * N * sizeof(double)));
    CREATE_CHK(hipMalloc(&c->x_qp, A * nv * sizeof(double)));
    CREATE_CHK(hipMalloc(&c->x, A * nv * sizeof(double)));
    CREATE_CHK(hipMalloc(&c->obj, A * sizeof(double)));
    CREATE_CHK(hipMalloc(&c->status, A * 2 * sizeof(int)));
    CREATE_CHK(hipMalloc(&c->iters, A * 2 * sizeof(int)));
    CREATE_CHK(hipMalloc(&c->abuf, A * 4 * sizeof(double)));
    CREATE_CHK(hipMalloc(&c->alpha, A * 20 * sizeof(double)));
    CREATE_CHK(hipMalloc(&c->sel, A * 2 * SRB_KNN_MAX * sizeof(int)));
    CREATE_CHK(hipMalloc(&c->zpol, A * (size_t)c->zstride * sizeof(float)));
#undef CREATE_CHK
    *out = c;
    return SRB_OK;
}

extern "C" int srb_ctx_destroy(srb_ctx *c)
{
    if (!c) return SRB_OK;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->any) (void)hipEventSynchronize(c->done);     // the last launch may be on another stream
    void *bufs[] = {c->x0, c->ref, c->foot, c->x_qp, c->x, c->obj, c->status, c->iters, c->obstacles, c->nbr,
                    c->abuf, c->alpha, c->sel, c->zpol};
    for (void *b : bufs)
        if (b) (void)hipFree(b);
    for (auto &g : c->grid)
        for (void *b : {g.g, (void *)g.off, (void *)g.spos, (void *)g.sidx})
            if (b) (void)hipFree(b);
    for (int i = 0; i < 4; i++)
        if (c->ev[i]) (void)hipEventDestroy(c->ev[i]);
    if (c->done) (void)hipEventDestroy(c->done);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return SRB_OK;
}

// Obstacle / neighbour selection for a batch (srb_knn_kernel; with a uniform grid per long table,
// srb_grid_build_kernel): K_obs, K_nbr already clamped to the tables.  x0 rows are [x, ., y, .]
// (stride 4); shared with the SRB-12 mode (srb12_capi.cpp), which hands over its CoM positions so.
static int launch_select(srb_ctx *c, int n_agents, const double *x0, const double *obstacles, int n_obs,
                         const double *nbr_state, int n_all, int agent_offset, int K_obs, int K_nbr,
                         int obstacles_version, int *sel, hipStream_t s, int sel_stride = -1)
{
    if (sel_stride < 0) sel_stride = K_obs + K_nbr;
    // long tables (a swarm sharded over GPUs: the whole neighbour snapshot, obstacles scaled
    // with the arena) get a uniform grid so each agent scans only the cells around it
    // (a versioned static obstacle table builds its grid once, so it pays off at fewer rows;
    // SRB_OPT_GRID_MIN_ROWS / _STATIC set the thresholds)
    const int min_rows = c->grid_min_rows, min_rows_static = c->grid_min_rows_static;
    const bool go = K_obs > 0 && n_obs >= (obstacles_version != 0 ? min_rows_static : min_rows);
    const bool gn = K_nbr > 0 && n_all >= min_rows;
    if (go) { int rc = grid_reserve(c, 0, n_obs); if (rc) return rc; }
    if (gn) { int rc = grid_reserve(c, 1, n_all); if (rc) return rc; }
    const srb_ctx::grid_buf &G0 = c->grid[0], &G1 = c->grid[1];
    // a static obstacle table (same version, pointer and size) keeps its grid
    const bool go_build = go && !(obstacles_version != 0 && obstacles_version == c->grid_ver &&
                                  obstacles == c->grid_src && n_obs == c->grid_n);
    if (go_build || gn) {
        hipLaunchKernelGGL(srb_grid_build_kernel, dim3(2), dim3(1024), 0, s,
                           obstacles, 2, n_obs, go_build ? (SrbGrid *)G0.g : nullptr, G0.off, G0.spos, G0.sidx,
                           nbr_state, 4, n_all, gn ? (SrbGrid *)G1.g : nullptr, G1.off, G1.spos, G1.sidx);
        HIPCHK(hipGetLastError());
    }
    if (go_build) { c->grid_src = obstacles; c->grid_n = n_obs; c->grid_ver = obstacles_version; }
    hipLaunchKernelGGL(srb_knn_kernel, dim3(n_agents), dim3(64 * SRB_KNN_WAVES), 0, s, n_agents, x0, obstacles, n_obs,
                       nbr_state, n_all, agent_offset, K_obs, K_nbr, sel, sel_stride,
                       go ? (const SrbGrid *)G0.g : nullptr, G0.off, G0.spos, G0.sidx,
                       gn ? (const SrbGrid *)G1.g : nullptr, G1.off, G1.spos, G1.sidx);
    HIPCHK(hipGetLastError());
    return SRB_OK;
}

int srb_internal_select(srb_ctx *c, int n_agents, const double *x0, const double *obstacles, int n_obs,
                        const double *nbr_state, int n_all, int agent_offset, int K_obs, int K_nbr,
                        int obstacles_version, int *sel, hipStream_t s)
{
    return launch_select(c, n_agents, x0, obstacles, n_obs, nbr_state, n_all, agent_offset, K_obs, K_nbr,
                         obstacles_version, sel, s);
}

int srb_internal_mark_done(srb_ctx *c, hipStream_t s) { return mark_done(c, s); }

static int launch(srb_ctx *c, int n_agents, const srb_batch *d, hipStream_t s, int use_nlp)
{
    if (n_agents < 0 || n_agents > c->max_agents) return fail(SRB_ERR_ARG, "n_agents exceeds max_agents");
    if (n_agents == 0) return SRB_OK;
    const srb_params *p = &c->p;
    if (!d->x0 || !d->ref || !d->foot || !d->x || !d->obj || !d->status || !d->iters)
        return fail(SRB_ERR_ARG, "missing buffer");
    if ((d->alpha != nullptr) != (d->alpha_buf != nullptr))
        return fail(SRB_ERR_ARG, "alpha and alpha_buf go together (both or neither)");
    if (d->alpha && p->N < 4) return fail(SRB_ERR_ARG, "the Bezier fit needs N >= 4 (X_0..X_3)");
    if (use_nlp && p->K_obs > 0 && (d->n_obs < 0 || (d->n_obs > 0 && !d->obstacles)))
        return fail(SRB_ERR_ARG, "obstacles missing");
    if (use_nlp && p->K_nbr > 0 && d->nbr_state && (d->agent_offset < 0 || d->agent_offset + n_agents > d->n_all))
        return fail(SRB_ERR_ARG, "agent_offset out of range of the neighbour table");
    SrbKParams k = make_kparams(p, use_nlp);
    k.qp_init = c->qp_init;
    k.polish_rho = c->polish_rho;
    k.qp_warm_tol = c->qp_warm_tol;
    k.kkt32_mu = c->kkt32_mu;
    k.kkt32_ref = c->kkt32_ref;
    // "up to K nearest": clamp to what exists (batch-uniform), so no row is ever a dummy
    if (k.K_obs > d->n_obs) k.K_obs = d->n_obs > 0 ? d->n_obs : 0;
    const int others = d->nbr_state ? d->n_all - 1 : 0;
    if (k.K_nbr > others) k.K_nbr = others > 0 ? others : 0;
    const srb_instance *in = pick_instance(k, wanted_waves(n_agents, srb_slots(k.N, k.C, k.K_obs + k.K_nbr), c->nw));
    if (!in) return fail(SRB_ERR_SIZE, "no kernel instance covers this problem");
    const size_t lds = (size_t)srb_lds_doubles(k, in->nzl, in->nw) * sizeof(double);
    c->last_nw = in->nw;
    HIPCHK(hipSetDevice(c->device));
    const int n_obs = k.K_obs > 0 ? d->n_obs : 0, n_all = k.K_nbr > 0 ? d->n_all : 0;
    // timing events (SRB_OPT_TIMING): each record is a marker the queue drains to, a few us a step
    c->timed = c->timing != 0;
    if (c->timing) HIPCHK(hipEventRecord(c->ev[0], s));
    // two launches: nearest obstacle / neighbour selection, then QP and NLP stages per agent
    int *sel = d->sel ? d->sel : c->sel;
    // SRB_OPT_SELECTION 0: the caller filled d->sel by srb_select_device (its two tables may then be selected
    // around a collective, bench.py's multi-GPU step)
    if (use_nlp && k.K_obs + k.K_nbr > 0 && c->selection) {
        int rc = launch_select(c, n_agents, d->x0, d->obstacles, n_obs, d->nbr_state, n_all, d->agent_offset, k.K_obs,
                               k.K_nbr, d->obstacles_version, sel, s);
        if (rc) return rc;
    }
    if (c->timing) HIPCHK(hipEventRecord(c->ev[2], s));
    // the solve kernel, then (NLP stage) the active-set polish of its result: fused into the solve
    // kernel's end (SRB_OPT_POLISH_FUSED, instances up to SRB_FUSED_POLISH_MAX = NZL 24), else srb_polish_kernel (same instance
    // geometry; it rewrites x / obj / alpha / status only where the polish is accepted)
    const bool fused = use_nlp && c->polish && c->polish_fused && SRB_FUSED_POLISH_OK(in->nzl);
    const bool polish = use_nlp && c->polish && !fused;
    k.polish_fused = fused ? 1 : 0;
    c->last_polish = fused ? 2 : polish ? 1 : 0;
    // SRB_OPT_KKT_FP32_MU > 0: the instance's fp32-factor variant where one is compiled (else the fp64 one)
    srb_kernel_fn fn = in->fn;
    c->last_f32 = 0;
    if (c->kkt32_mu > 0.0) {
        srb_kernel_fn f = f32_variant(in);
        if (f) { fn = f; c->last_f32 = 1; }
    }
    hipLaunchKernelGGL(fn, dim3(n_agents), dim3(64 * in->nw), lds, s, k, n_agents, d->x0, d->ref, d->foot, d->obstacles,
                       n_obs, d->nbr_state, n_all, d->agent_offset, d->x_qp, d->x, d->obj, d->status, d->iters,
                       d->alpha ? d->alpha_buf : nullptr, d->alpha_buf ? d->alpha : nullptr, (const int *)sel,
                       polish ? c->zpol : nullptr, c->zstride);
    HIPCHK(hipGetLastError());
    if (c->timing) HIPCHK(hipEventRecord(c->ev[3], s));
    if (polish) {
        // the polish kernel reads only the solve's outputs (x, status, sel, zpol by global slot
        // index), so it runs at its own waves per agent: at least two (its registers fit two
        // waves per SIMD, and a polish step's latency halves): configs[2] polish 0.067 -> 0.053 ms,
        // configs[1] (solve at 4 waves) and N = 20 (2 waves) unchanged, one wave slower everywhere
        // (profiles/r03_polish_nw_ab.txt).  SRB_OPT_POLISH_WAVES = 1 | 2 | 4 overrides.
        const int pnw = c->polish_waves ? c->polish_waves : (in->nw < 2 ? 2 : in->nw);
        const srb_instance *pin = pnw == in->nw ? in : pick_instance(k, pnw);
        if (!pin || pin->nzl != in->nzl) pin = in;
        const size_t plds = (size_t)srb_lds_doubles(k, pin->nzl, pin->nw) * sizeof(double);
        hipLaunchKernelGGL(pin->polish, dim3(n_agents), dim3(64 * pin->nw), plds, s, k, n_agents, d->x0, d->ref, d->foot,
                           d->obstacles, d->nbr_state, d->x, d->obj, d->status, d->alpha ? d->alpha_buf : nullptr,
                           d->alpha_buf ? d->alpha : nullptr, (const int *)sel, (const float *)c->zpol, c->zstride);
        HIPCHK(hipGetLastError());
    }
    if (c->timing) HIPCHK(hipEventRecord(c->ev[1], s));
    return SRB_OK;
}

extern "C" int srb_ctx_set_waves(srb_ctx *c, int nw)
{
    if (!c) return fail(SRB_ERR_ARG, "null ctx");
    if (nw != 0 && nw != 1 && nw != 2 && nw != 4) return fail(SRB_ERR_ARG, "waves per agent: 0 (automatic), 1, 2 or 4");
    c->nw = nw;
    return SRB_OK;
}

extern "C" int srb_ctx_waves(srb_ctx *c) { return c ? c->last_nw : 0; }

extern "C" int srb_ctx_set_option(srb_ctx *c, int opt, double v)
{
    if (!c) return fail(SRB_ERR_ARG, "null ctx");
    const bool whole = v == (double)(long long)v;
    switch (opt) {
    case SRB_OPT_POLISH:
        if (v != 0.0 && v != 1.0) return fail(SRB_ERR_ARG, "SRB_OPT_POLISH: 0 or 1");
        c->polish = (int)v; return SRB_OK;
    case SRB_OPT_POLISH_RHO:
        if (!(v >= 1e3 && v <= 1e12)) return fail(SRB_ERR_ARG, "SRB_OPT_POLISH_RHO: 1e3 .. 1e12");
        c->polish_rho = v; return SRB_OK;
    case SRB_OPT_POLISH_WAVES:
        if (v != 0.0 && v != 1.0 && v != 2.0 && v != 4.0) return fail(SRB_ERR_ARG, "SRB_OPT_POLISH_WAVES: 0 (automatic), 1, 2 or 4");
        c->polish_waves = (int)v; return SRB_OK;
    case SRB_OPT_POLISH_FUSED:
        if (v != 0.0 && v != 1.0) return fail(SRB_ERR_ARG, "SRB_OPT_POLISH_FUSED: 0 or 1");
        c->polish_fused = (int)v; return SRB_OK;
    case SRB_OPT_LAST_POLISH:
        return fail(SRB_ERR_ARG, "SRB_OPT_LAST_POLISH is read only");
    case SRB_OPT_QP_WARM_TOL:
        if (!(v >= 0.0 && v <= 1e3)) return fail(SRB_ERR_ARG, "SRB_OPT_QP_WARM_TOL: 0 (the full tolerance) .. 1e3");
        c->qp_warm_tol = v; return SRB_OK;
    case SRB_OPT_TIMING:
        if (v != 0.0 && v != 1.0) return fail(SRB_ERR_ARG, "SRB_OPT_TIMING: 0 or 1");
        c->timing = (int)v; return SRB_OK;
    case SRB_OPT_SELECTION:
        if (v != 0.0 && v != 1.0) return fail(SRB_ERR_ARG, "SRB_OPT_SELECTION: 0 or 1");
        c->selection = (int)v; return SRB_OK;
    case SRB_OPT_KKT_FP32_MU:
        if (!(v >= 0.0 && v <= 1e30)) return fail(SRB_ERR_ARG, "SRB_OPT_KKT_FP32_MU: 0 (off) .. 1e30");
        c->kkt32_mu = v; return SRB_OK;
    case SRB_OPT_KKT_FP32_REFINE:
        if (!whole || v < 1.0 || v > 8.0) return fail(SRB_ERR_ARG, "SRB_OPT_KKT_FP32_REFINE: 1 .. 8");
        c->kkt32_ref = (int)v; return SRB_OK;
    case SRB_OPT_LAST_KKT_FP32:
        return fail(SRB_ERR_ARG, "SRB_OPT_LAST_KKT_FP32 is read only");
    case SRB_OPT_GRID_MIN_ROWS:
    case SRB_OPT_GRID_MIN_ROWS_STATIC:
        if (!whole || v < 1.0 || v > 2147483647.0) return fail(SRB_ERR_ARG, "SRB_OPT_GRID_MIN_ROWS*: a row count >= 1");
        (opt == SRB_OPT_GRID_MIN_ROWS ? c->grid_min_rows : c->grid_min_rows_static) = (int)v;
        return SRB_OK;
    default:
        return fail(SRB_ERR_ARG, "unknown option");
    }
}

extern "C" int srb_ctx_get_option(srb_ctx *c, int opt, double *v)
{
    if (!c || !v) return fail(SRB_ERR_ARG, "null argument");
    switch (opt) {
    case SRB_OPT_POLISH: *v = c->polish; return SRB_OK;
    case SRB_OPT_POLISH_RHO: *v = c->polish_rho; return SRB_OK;
    case SRB_OPT_POLISH_WAVES: *v = c->polish_waves; return SRB_OK;
    case SRB_OPT_GRID_MIN_ROWS: *v = c->grid_min_rows; return SRB_OK;
    case SRB_OPT_GRID_MIN_ROWS_STATIC: *v = c->grid_min_rows_static; return SRB_OK;
    case SRB_OPT_POLISH_FUSED: *v = c->polish_fused; return SRB_OK;
    case SRB_OPT_LAST_POLISH: *v = c->last_polish; return SRB_OK;
    case SRB_OPT_TIMING: *v = c->timing; return SRB_OK;
    case SRB_OPT_QP_WARM_TOL: *v = c->qp_warm_tol; return SRB_OK;
    case SRB_OPT_SELECTION: *v = c->selection; return SRB_OK;
    case SRB_OPT_KKT_FP32_MU: *v = c->kkt32_mu; return SRB_OK;
    case SRB_OPT_KKT_FP32_REFINE: *v = c->kkt32_ref; return SRB_OK;
    case SRB_OPT_LAST_KKT_FP32: *v = c->last_f32; return SRB_OK;
    default: return fail(SRB_ERR_ARG, "unknown option");
    }
}

extern "C" int srb_ctx_set_qp_init(srb_ctx *c, int mode)
{
    if (!c) return fail(SRB_ERR_ARG, "null ctx");
    if (mode != 0 && mode != 1) return fail(SRB_ERR_ARG, "QP start: 1 (scaled, default) or 0 (iSWIFT kkt_initialize)");
    c->qp_init = mode;
    return SRB_OK;
}

extern "C" int srb_solve_batch_device(srb_ctx *c, int n_agents, const srb_batch *dev_io, void *stream)
{
    // the layout check comes first: it needs no context (tests/test_abi.py runs it without a GPU)
    if (dev_io && dev_io->struct_size != (int)sizeof(srb_batch))
        return fail(SRB_ERR_ARG, "srb_batch.struct_size != sizeof(srb_batch): caller built against another ABI");
    if (!c || !dev_io) return fail(SRB_ERR_ARG, "null argument");
    hipStream_t s = (hipStream_t)stream;          // NULL: the HIP null stream (ordered with blocking streams)
    HIPCHK(hipSetDevice(c->device));
    int rc = order_after_last(c, s);
    if (!rc) rc = launch(c, n_agents, dev_io, s, c->p.use_nlp);
    if (!rc && n_agents > 0) rc = mark_done(c, s);
    return rc;
}

// One or both tables of the selection into dev_io->sel (required; [A][Ko + Kn], the layout the solve reads):
// tables bit 0 the static obstacles (its columns 0 .. Ko - 1), bit 1 the neighbour snapshot (Ko .. Ko + Kn - 1).
// With SRB_OPT_SELECTION = 0 the solve then uses sel as it is, so a caller can select the static obstacles
// while the neighbour all-gather is in flight and the neighbours after it (bench.py).
extern "C" int srb_select_device(srb_ctx *c, int n_agents, const srb_batch *d, int tables, void *stream)
{
    if (d && d->struct_size != (int)sizeof(srb_batch))
        return fail(SRB_ERR_ARG, "srb_batch.struct_size != sizeof(srb_batch): caller built against another ABI");
    if (!c || !d) return fail(SRB_ERR_ARG, "null argument");
    if (tables < 1 || tables > 3) return fail(SRB_ERR_ARG, "tables: 1 (static obstacles), 2 (neighbours) or 3 (both)");
    if (n_agents < 0 || n_agents > c->max_agents) return fail(SRB_ERR_ARG, "n_agents exceeds max_agents");
    if (!d->x0 || !d->sel) return fail(SRB_ERR_ARG, "missing buffer (x0, sel)");
    if (n_agents == 0) return SRB_OK;
    const srb_params *p = &c->p;
    int Ko = p->K_obs, Kn = p->K_nbr;                     // clamped exactly as the solve does
    if (Ko > d->n_obs) Ko = d->n_obs > 0 ? d->n_obs : 0;
    const int others = d->nbr_state ? d->n_all - 1 : 0;
    if (Kn > others) Kn = others > 0 ? others : 0;
    if ((tables & 1) && Ko > 0 && !d->obstacles) return fail(SRB_ERR_ARG, "obstacles missing");
    if ((tables & 2) && Kn > 0 && (d->agent_offset < 0 || d->agent_offset + n_agents > d->n_all))
        return fail(SRB_ERR_ARG, "agent_offset out of range of the neighbour table");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipSetDevice(c->device));
    int rc = order_after_last(c, s);
    const int ko = (tables & 1) ? Ko : 0, kn = (tables & 2) ? Kn : 0;
    if (!rc && ko + kn > 0)
        rc = launch_select(c, n_agents, d->x0, d->obstacles, ko ? d->n_obs : 0, d->nbr_state, kn ? d->n_all : 0,
                           d->agent_offset, ko, kn, d->obstacles_version, d->sel + (ko ? 0 : Ko), s, Ko + Kn);
    if (!rc) rc = mark_done(c, s);
    return rc;
}

extern "C" __global__ void srb_prepare_kernel(int n_agents, int N, int C, int n_rows, int T, int agent_offset,
                                              const double *Pr, const double *Prd, const int *agent_id,
                                              const int *gait_domain, const int *contact, const double *toe,
                                              const double *start, const double *q, const double *dq, double *x0,
                                              double *ref, double *foot, double *last_state, int *status);

extern "C" int srb_prepare_batch_device(srb_ctx *c, int n_agents, const srb_prep *d, void *stream)
{
    // the layout check comes first: it needs no context (tests/test_abi.py runs it without a GPU)
    if (d && d->struct_size != (int)sizeof(srb_prep))
        return fail(SRB_ERR_ARG, "srb_prep.struct_size != sizeof(srb_prep): caller built against another ABI");
    if (!c || !d) return fail(SRB_ERR_ARG, "null argument");
    if (n_agents < 0) return fail(SRB_ERR_ARG, "negative n_agents");
    if (n_agents == 0) return SRB_OK;
    if (!d->Pr || !d->Prd || !d->gait_domain || !d->contact || !d->toe || !d->start || !d->q || !d->dq || !d->x0 ||
        !d->ref || !d->foot || !d->last_state || !d->status)
        return fail(SRB_ERR_ARG, "missing buffer");
    if (d->n_rows < 2 || d->T < 1) return fail(SRB_ERR_ARG, "empty HL path");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;          // NULL: the HIP null stream (ordered with blocking streams)
    hipLaunchKernelGGL(srb_prepare_kernel, dim3((n_agents + 255) / 256), dim3(256), 0, s, n_agents, c->p.N, c->p.C,
                       d->n_rows, d->T, d->agent_offset, d->Pr, d->Prd, d->agent_id, d->gait_domain, d->contact,
                       d->toe, d->start, d->q, d->dq, d->x0, d->ref, d->foot, d->last_state, d->status);
    HIPCHK(hipGetLastError());
    return SRB_OK;
}

extern "C" __global__ void srb_hlplan_kernel(int NA, const double *Pstart, const double *Pobs, int n_obs, int loop,
                                             double *Pr, double *Prd);

extern "C" __global__ void srb_hlplan_step_kernel(int NA, int i, int loop, const double *Pobs, int n_obs,
                                                  const double *pos_cur, double *pos_next, double *st, double *Pr,
                                                  double *Prd);

// swarms up to this many agents run as one persistent workgroup (srb_hlplan_kernel); larger ones
// one launch per step over NA / 64 workgroups (srb_hlplan_step_kernel)
#define SRB_HL_ONE_WG 1024

extern "C" int srb_hl_plan(int device, int NA, const double *Pstart, const double *Pobs, int n_obs, int loop, double *Pr,
                           double *Prd)
{
    if (NA < 1 || NA > (1 << 20)) return fail(SRB_ERR_SIZE, "HL planner: 1 <= NA <= 2^20");
    if (n_obs < 0 || n_obs > 2048 || (n_obs > 0 && !Pobs)) return fail(SRB_ERR_ARG, "HL planner: bad obstacle table");
    if (loop < 80 || !Pstart || !Pr || !Prd) return fail(SRB_ERR_ARG, "HL planner: bad arguments (loop >= 80)");
    int ndev = 0;
    HIPCHK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(SRB_ERR_ARG, "device index out of range");
    HIPCHK(hipSetDevice(device));
    const int T = loop / 40;
    const size_t out = (size_t)T * 2 * NA * sizeof(double);
    double *dPs = nullptr, *dOb = nullptr, *dPr = nullptr, *dPrd = nullptr;
    int rc = SRB_OK;
    auto chk = [&](hipError_t e, const char *what) {
        if (e != hipSuccess && rc == SRB_OK) rc = fail(SRB_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
    };
    chk(hipMalloc(&dPs, 2 * NA * sizeof(double)), "hipMalloc");
    chk(hipMalloc(&dOb, (n_obs > 0 ? n_obs : 1) * 2 * sizeof(double)), "hipMalloc");
    chk(hipMalloc(&dPr, out), "hipMalloc");
    chk(hipMalloc(&dPrd, out), "hipMalloc");
    if (rc == SRB_OK) {
        chk(hipMemcpy(dPs, Pstart, 2 * NA * sizeof(double), hipMemcpyHostToDevice), "hipMemcpy");
        if (n_obs > 0) chk(hipMemcpy(dOb, Pobs, n_obs * 2 * sizeof(double), hipMemcpyHostToDevice), "hipMemcpy");
    }
    if (rc == SRB_OK && NA <= SRB_HL_ONE_WG) {
        const int threads = ((NA + 63) / 64) * 64;
        const size_t lds = (4 * (size_t)NA + 2 * (size_t)n_obs) * sizeof(double);
        hipLaunchKernelGGL(srb_hlplan_kernel, dim3(1), dim3(threads), lds, 0, NA, dPs, dOb, n_obs, loop, dPr, dPrd);
        chk(hipGetLastError(), "srb_hlplan_kernel");
        chk(hipDeviceSynchronize(), "srb_hlplan_kernel");
    } else if (rc == SRB_OK) {
        // one coupled swarm across the chip: positions double-buffered in global memory
        double *pos[2] = {nullptr, nullptr}, *st = nullptr;
        chk(hipMalloc(&pos[0], 2 * (size_t)NA * sizeof(double)), "hipMalloc");
        chk(hipMalloc(&pos[1], 2 * (size_t)NA * sizeof(double)), "hipMalloc");
        chk(hipMalloc(&st, 4 * (size_t)NA * sizeof(double)), "hipMalloc");
        if (rc == SRB_OK) {
            double *h = (double *)std::calloc(4 * (size_t)NA, sizeof(double));
            for (int a = 0; a < NA; a++) { h[4 * a] = Pstart[2 * a]; h[4 * a + 1] = Pstart[2 * a + 1]; }
            chk(hipMemcpy(st, h, 4 * (size_t)NA * sizeof(double), hipMemcpyHostToDevice), "hipMemcpy");
            chk(hipMemcpy(pos[0], Pstart, 2 * (size_t)NA * sizeof(double), hipMemcpyHostToDevice), "hipMemcpy");
            std::free(h);
        }
        const int blocks = (NA + 63) / 64;
        for (int i = 0; i <= loop && rc == SRB_OK; i++) {
            hipLaunchKernelGGL(srb_hlplan_step_kernel, dim3(blocks), dim3(64), 0, 0, NA, i, loop, dOb, n_obs, pos[i & 1],
                               pos[(i & 1) ^ 1], st, dPr, dPrd);
            if ((i & 1023) == 0) chk(hipGetLastError(), "srb_hlplan_step_kernel");
        }
        chk(hipDeviceSynchronize(), "srb_hlplan_step_kernel");
        for (void *b : {(void *)pos[0], (void *)pos[1], (void *)st})
            if (b) (void)hipFree(b);
    }
    if (rc == SRB_OK) {
        chk(hipMemcpy(Pr, dPr, out, hipMemcpyDeviceToHost), "hipMemcpy");
        chk(hipMemcpy(Prd, dPrd, out, hipMemcpyDeviceToHost), "hipMemcpy");
    }
    for (void *b : {(void *)dPs, (void *)dOb, (void *)dPr, (void *)dPrd})
        if (b) (void)hipFree(b);
    return rc;
}

extern "C" int srb_sync(srb_ctx *c)
{
    if (!c) return fail(SRB_ERR_ARG, "null ctx");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipDeviceSynchronize());
    return SRB_OK;
}

extern "C" int srb_last_kernel_ms(srb_ctx *c, float *knn_ms, float *solve_ms)
{
    if (!c || !c->timed) return fail(SRB_ERR_ARG, "no timed launch");
    HIPCHK(hipEventSynchronize(c->ev[1]));
    float a = 0, b = 0;
    HIPCHK(hipEventElapsedTime(&a, c->ev[0], c->ev[2]));
    HIPCHK(hipEventElapsedTime(&b, c->ev[2], c->ev[3]));
    if (knn_ms) *knn_ms = a;            // srb_knn_kernel (0 when there is nothing to select)
    if (solve_ms) *solve_ms = b;        // srb_nmpc_kernel_*
    return SRB_OK;
}

extern "C" int srb_last_polish_ms(srb_ctx *c, float *polish_ms)
{
    if (!c || !c->timed) return fail(SRB_ERR_ARG, "no timed launch");
    HIPCHK(hipEventSynchronize(c->ev[1]));
    float t = 0;
    if (c->last_polish == 1) HIPCHK(hipEventElapsedTime(&t, c->ev[3], c->ev[1]));
    if (polish_ms) *polish_ms = t;      // srb_polish_kernel_* (0 without it: no NLP stage, or fused)
    return SRB_OK;
}

static int solve_host(srb_ctx *c, int n_agents, const srb_batch *h, int use_nlp)
{
    // the layout check comes first: it needs no context (tests/test_abi.py runs it without a GPU)
    if (h && h->struct_size != (int)sizeof(srb_batch))
        return fail(SRB_ERR_ARG, "srb_batch.struct_size != sizeof(srb_batch): caller built against another ABI");
    if (!c || !h) return fail(SRB_ERR_ARG, "null argument");
    if (n_agents < 0 || n_agents > c->max_agents) return fail(SRB_ERR_ARG, "n_agents exceeds max_agents");
    if (n_agents == 0) return SRB_OK;
    const srb_params *p = &c->p;
    const int N = p->N, C = p->C, nv = srb_nv(p);
    const size_t A = (size_t)n_agents;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    if (int rc0 = order_after_last(c, s)) return rc0;   // after the last device launch on this context
    if (!h->x0 || !h->ref || !h->foot || !h->x || !h->obj || !h->status || !h->iters)
        return fail(SRB_ERR_ARG, "missing buffer");
    HIPCHK(hipMemcpyAsync(c->x0, h->x0, A * 4 * sizeof(double), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->ref, h->ref, A * 4 * N * sizeof(double), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->foot, h->foot, A * 2 * C * N * sizeof(double), hipMemcpyHostToDevice, s));
    srb_batch d = *h;
    d.x0 = c->x0; d.ref = c->ref; d.foot = c->foot;
    d.x_qp = c->x_qp; d.x = c->x; d.obj = c->obj; d.status = c->status; d.iters = c->iters;
    d.alpha_buf = nullptr; d.alpha = nullptr;
    if (h->alpha && h->alpha_buf) {
        HIPCHK(hipMemcpyAsync(c->abuf, h->alpha_buf, A * 4 * sizeof(double), hipMemcpyHostToDevice, s));
        d.alpha_buf = c->abuf; d.alpha = c->alpha;
    } else if (h->alpha || h->alpha_buf) {
        return fail(SRB_ERR_ARG, "alpha and alpha_buf go together (both or neither)");
    }
    d.obstacles = nullptr; d.nbr_state = nullptr;
    if (h->n_obs > 0 && h->obstacles) {
        if ((size_t)h->n_obs > c->cap_obs) {
            if (c->obstacles) HIPCHK(hipFree(c->obstacles));
            HIPCHK(hipMalloc(&c->obstacles, (size_t)h->n_obs * 2 * sizeof(double)));
            c->cap_obs = h->n_obs;
        }
        HIPCHK(hipMemcpyAsync(c->obstacles, h->obstacles, (size_t)h->n_obs * 2 * sizeof(double), hipMemcpyHostToDevice, s));
        d.obstacles = c->obstacles;
    }
    if (h->n_all > 0 && h->nbr_state) {
        if ((size_t)h->n_all > c->cap_nbr) {
            if (c->nbr) HIPCHK(hipFree(c->nbr));
            HIPCHK(hipMalloc(&c->nbr, (size_t)h->n_all * 4 * sizeof(double)));
            c->cap_nbr = h->n_all;
        }
        HIPCHK(hipMemcpyAsync(c->nbr, h->nbr_state, (size_t)h->n_all * 4 * sizeof(double), hipMemcpyHostToDevice, s));
        d.nbr_state = c->nbr;
    }
    d.sel = nullptr;                       // the context's scratch; copied out below when asked for
    d.obstacles_version = 0;               // staged copy: rebuilt every call
    int rc = launch(c, n_agents, &d, s, use_nlp);
    if (!rc) rc = mark_done(c, s);
    if (rc) return rc;
    if (h->sel && use_nlp) {
        const int Ko = std::min(p->K_obs, std::max(h->n_obs, 0)), Kn = h->nbr_state ? std::min(p->K_nbr, std::max(h->n_all - 1, 0)) : 0;
        if (Ko + Kn > 0) HIPCHK(hipMemcpyAsync(h->sel, c->sel, A * (Ko + Kn) * sizeof(int), hipMemcpyDeviceToHost, s));
    }
    if (h->x_qp) HIPCHK(hipMemcpyAsync(h->x_qp, c->x_qp, A * nv * sizeof(double), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(h->x, c->x, A * nv * sizeof(double), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(h->obj, c->obj, A * sizeof(double), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(h->status, c->status, A * 2 * sizeof(int), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(h->iters, c->iters, A * 2 * sizeof(int), hipMemcpyDeviceToHost, s));
    if (d.alpha) HIPCHK(hipMemcpyAsync(h->alpha, c->alpha, A * 20 * sizeof(double), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return SRB_OK;
}

extern "C" int srb_solve_batch(srb_ctx *c, int n_agents, const srb_batch *host_io)
{
    return solve_host(c, n_agents, host_io, c ? c->p.use_nlp : 0);
}

extern "C" int srb_solve_qp(srb_ctx *c, int n_agents, const srb_batch *host_io)
{
    return solve_host(c, n_agents, host_io, 0);
}

// fitComTrajectory_eventbase (MPC_dist.cpp:784-855).  With N == NDOMAIN the reference's
// 24x24 KKT (whose 20x8 -> 20x4 block assignment keeps only the s = 0 end-point row)
// has the unique solution of the 5-point Bernstein interpolation through
// [buf, X0, X1, X2, X3] at s = 0, 1/4, 1/2, 3/4, 1, solved here per state row.
extern "C" void srb_fit_bezier(const double buf[4], const double *X, double alpha[20])
{
    static const double binom[5] = {1, 4, 6, 4, 1};
    for (int d = 0; d < 4; d++) {
        double M[5][6];
        for (int i = 0; i < 5; i++) {
            double s = i * 0.25;
            for (int j = 0; j < 5; j++) M[i][j] = binom[j] * std::pow(s, j) * std::pow(1 - s, 4 - j);
            M[i][5] = (i == 0) ? buf[d] : X[(i - 1) * 4 + d];
        }
        for (int k = 0; k < 5; k++) {           // Gaussian elimination, partial pivoting
            int piv = k;
            for (int i = k + 1; i < 5; i++) if (std::fabs(M[i][k]) > std::fabs(M[piv][k])) piv = i;
            if (piv != k) for (int j = 0; j < 6; j++) std::swap(M[k][j], M[piv][j]);
            for (int i = k + 1; i < 5; i++) {
                double l = M[i][k] / M[k][k];
                for (int j = k; j < 6; j++) M[i][j] -= l * M[k][j];
            }
        }
        double a[5];
        for (int i = 4; i >= 0; i--) {
            double s = M[i][5];
            for (int j = i + 1; j < 5; j++) s -= M[i][j] * a[j];
            a[i] = s / M[i][i];
        }
        for (int j = 0; j < 5; j++) alpha[d * 5 + j] = a[j];
    }
}

extern "C" const char *srb_last_error(void) { return g_err.c_str(); }

#ifdef SRB_NLPDBG
extern __device__ double srb_nlp_dbg[SRB_NLP_DBG_LEN];
extern __device__ int srb_nlp_dbg_agent;
// diagnostic build only: select the traced agent (-1: none) and read/clear the trace
extern "C" int srb_debug_nlp_trace(int agent, double *out)
{
    HIPCHK(hipDeviceSynchronize());
    if (out) HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(srb_nlp_dbg), sizeof(double) * SRB_NLP_DBG_LEN));
    double z[SRB_NLP_DBG_LEN] = {0};
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(srb_nlp_dbg), z, sizeof z));
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(srb_nlp_dbg_agent), &agent, sizeof(int)));
    return SRB_OK;
}
#endif

#ifdef SRB_STAMPS
extern __device__ unsigned long long srb_stamp_buf[64];
extern "C" int srb_debug_stamps(unsigned long long *out, int reset)
{
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(srb_stamp_buf), sizeof(unsigned long long) * 64));
    if (reset) {
        unsigned long long z[64] = {0};
        HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(srb_stamp_buf), z, sizeof z));
    }
    return SRB_OK;
}
#endif
