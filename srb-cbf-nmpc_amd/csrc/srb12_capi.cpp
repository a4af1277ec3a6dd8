// Host side of the SRB-12 extension-mode entry points of include/srbnmpc.h (srb12_*).
//
// The context owns device staging for the host-buffer entry point, a LIP-mode context whose
// selection machinery (srb_knn_kernel and its grids, srb_capi.cpp) it reuses for the obstacle /
// neighbour rows, and events around the two launches.  One 64-lane workgroup per agent runs
// srb12_kernel_<TL>_<TO>_<NC>_<K1> (srb12_kernels.hip): row-slot trips per lane, (N, K) compiled in or 0.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstring>
#include <string>
#include "srbnmpc.h"
#include "srb_kernel_params.h"

#define SRB12_DBG_LEN (2 * 64 * 8 + 16 + 128)   // trace, stamp sums, state checks (srb12_kernels.hip)

int srb_internal_fail(int code, const char *msg);
int srb_internal_select(srb_ctx *c, int n_agents, const double *x0, const double *obstacles, int n_obs,
                        const double *nbr_state, int n_all, int agent_offset, int K_obs, int K_nbr,
                        int obstacles_version, int *sel, hipStream_t s);
int srb_internal_mark_done(srb_ctx *c, hipStream_t s);

typedef void (*srb12_fn)(Srb12KParams, int, const double *, const double *, const double *, const int *,
                         const double *, const double *, const int *, double *, double *, double *, int *, int *);
#define DECL12(TL, TO, NC, K1)                                                                                  \
    extern "C" __global__ void srb12_kernel_##TL##_##TO##_##NC##_##K1(Srb12KParams, int, const double *, const double *,      \
                                                        const double *, const int *, const double *,             \
                                                        const double *, const int *, double *, double *,         \
                                                        double *, int *, int *);
SRB12_INSTANCES(DECL12)
#undef DECL12
extern "C" __global__ void srb12_pos_kernel(int n_agents, const double *x0g, double *pos);
struct srb12_inst { int tl, to, nc, k1; srb12_fn fn; };
#define ENTRY12(TL, TO, NC, K1) {TL, TO, NC, K1, srb12_kernel_##TL##_##TO##_##NC##_##K1},
static const srb12_inst g_inst12[] = {SRB12_INSTANCES(ENTRY12)};
#undef ENTRY12

#define H12CHK(expr)                                                                                    \
    do {                                                                                                \
        hipError_t e_ = (expr);                                                                         \
        if (e_ != hipSuccess)                                                                           \
            return srb_internal_fail(SRB_ERR_HIP, (std::string(#expr ": ") + hipGetErrorString(e_)).c_str()); \
    } while (0)

struct srb12_ctx {
    srb12_params p;
    int max_agents, device;
    srb_ctx *sel_ctx;              // LIP-mode context: selection kernels, grids, default sel buffer
    hipStream_t stream;
    hipEvent_t ev[3];
    hipEvent_t done;
    hipStream_t last;
    bool timed, any;
    int timing;                    // srb12_ctx_set_timing (default 1)
    double *pos;                   // [max_agents][4] CoM rows for the selection
    int *sel;                      // [max_agents][2 SRB_KNN_MAX]
    double *x0, *xref, *foot, *obstacles, *nbr, *x_qp, *x, *obj;
    int *contact, *status, *iters;
    size_t cap_obs, cap_nbr;
    int dbg_agent;                 // diagnostics: srb12_debug_trace
    double *dbg;
};

extern "C" void srb12_params_default(srb12_params *p, int N)
{
    std::memset(p, 0, sizeof(*p));
    p->N = N; p->K_obs = 3; p->K_nbr = 0;
    p->Ts = 43 * 0.001;                     // the LIP grid (MPC_dist.cpp:104): the same neighbour prediction
    p->mass = 12.4530;                      // fast_MPC.cpp:40
    const double Ib[9] = {0.01683993, 8.3902e-5, 0.000597679, 8.3902e-5, 0.056579028, 2.5134e-5,
                          0.000597679, 2.5134e-5, 0.064713601};      // fast_MPC.cpp:41-43
    std::memcpy(p->Ib, Ib, sizeof Ib);
    p->grav = 9.81; p->mu = 0.7; p->fmax = 150.0;                   // mu_MPC (Parameters.cpp:32)
    for (int i = 0; i < 12; i++) { p->q[i] = 1e3; p->qN[i] = 1e3; }  // Parameters.cpp:34-45
    for (int i = 0; i < 3; i++) p->r[i] = 1e-2;                      // Parameters.cpp:50-52
    p->Sw = 3000.0;
    p->eps_obs = (double)1.9f; p->eps_nbr = (double)2.2f;
    p->tol = 1e-6; p->qp_maxit = 25; p->nlp_maxit = 50; p->use_nlp = 1;
    p->z0 = 100.0;
    p->tol_final = 1e-8;
    p->polish = 1;
    p->tol_qp = 1e-3;
}

extern "C" int srb12_nv(const srb12_params *p) { return 24 * p->N + 1; }

// the first instance with enough leg-slot and obstacle-slot trips (the list is ordered by cost) for
// horizon N and K rows per grid -- the rows the launch actually selects (clamp_rows: a compiled-in K
// must equal them, the kernel reads sel at that stride and carves its LDS for them)
static const srb12_inst *pick12(int N, int K)
{
    const int tl = srb12_leg_trips(N), to = srb12_obs_trips(N, K);
    for (const srb12_inst &in : g_inst12)      // the (N, K) compiled in
        if (in.nc == N && in.k1 == K + 1 && in.tl >= tl && in.to >= to) return &in;
    for (const srb12_inst &in : g_inst12)      // run-time (N, K)
        if (in.nc == 0 && in.tl >= tl && in.to >= to) return &in;
    return nullptr;
}

static int validate12(const srb12_params *p)
{
    if (!p) return srb_internal_fail(SRB_ERR_ARG, "null params");
    if (p->N < 1 || p->N > SRB12_MAX_N) return srb_internal_fail(SRB_ERR_SIZE, "SRB-12 mode: need 1 <= N <= 24");
    if (p->K_obs < 0 || p->K_nbr < 0 || p->K_obs > SRB_KNN_MAX || p->K_nbr > SRB_KNN_MAX)
        return srb_internal_fail(SRB_ERR_ARG, "K_obs, K_nbr out of range (each <= 16)");
    if (!(p->mass > 0) || !(p->Ts > 0) || !(p->tol > 0) || !(p->tol_final > 0) || !(p->mu >= 0) || !(p->fmax > 0) ||
        !(p->Sw > 0) || !(p->tol_qp >= 0))
        return srb_internal_fail(SRB_ERR_ARG, "srb12_params out of range (mass, Ts, tol, tol_final, fmax, Sw > 0, tol_qp >= 0)");
    for (int i = 0; i < 12; i++)
        if (!(p->q[i] >= 0) || !(p->qN[i] >= 0)) return srb_internal_fail(SRB_ERR_ARG, "state weights must be >= 0");
    for (int i = 0; i < 3; i++)
        if (!(p->r[i] > 0)) return srb_internal_fail(SRB_ERR_ARG, "force weights must be > 0");
    if (!pick12(p->N, p->K_obs + p->K_nbr)) return srb_internal_fail(SRB_ERR_SIZE, "no SRB-12 kernel instance covers the row slots");
    if ((size_t)srb12_lds_doubles(p->N, p->K_obs + p->K_nbr) * sizeof(double) > 160 * 1024)
        return srb_internal_fail(SRB_ERR_SIZE, "per-agent LDS exceeds 160 KiB");
    return SRB_OK;
}

extern "C" int srb12_lds_bytes(const srb12_params *p)
{
    return p ? srb12_lds_doubles(p->N, p->K_obs + p->K_nbr) * (int)sizeof(double) : -1;
}

static Srb12KParams make_k12(const srb12_params *p, int K_obs, int K_nbr)
{
    Srb12KParams k;
    std::memset(&k, 0, sizeof k);
    k.N = p->N; k.K_obs = K_obs; k.K_nbr = K_nbr; k.use_nlp = p->use_nlp ? 1 : 0;
    k.qp_maxit = p->qp_maxit; k.nlp_maxit = p->nlp_maxit;
    k.Ts = p->Ts; k.mass = p->mass; k.grav = p->grav; k.mus = p->mu / std::sqrt(2.0); k.fmax = p->fmax;
    k.Sw = p->Sw; k.eps_obs = p->eps_obs; k.eps_nbr = p->eps_nbr; k.tol = p->tol; k.z0 = p->z0; k.tol_final = p->tol_final; k.polish = p->polish ? 1 : 0;
    k.tol_qp = p->tol_qp;
    std::memcpy(k.Ib, p->Ib, sizeof k.Ib);
    std::memcpy(k.q, p->q, sizeof k.q); std::memcpy(k.qN, p->qN, sizeof k.qN); std::memcpy(k.r, p->r, sizeof k.r);
    return k;
}

extern "C" int srb12_ctx_create(const srb12_params *p, int max_agents, int device, srb12_ctx **out)
{
    if (!out || max_agents <= 0) return srb_internal_fail(SRB_ERR_ARG, "bad arguments");
    int rc = validate12(p);
    if (rc) return rc;
    int ndev = 0;
    H12CHK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return srb_internal_fail(SRB_ERR_ARG, "device index out of range");
    H12CHK(hipSetDevice(device));
    srb_params sp;
    srb_params_default(&sp, 2, 2);
    sp.K_obs = p->K_obs; sp.K_nbr = p->K_nbr;
    srb_ctx *sc = nullptr;
    if ((rc = srb_ctx_create(&sp, max_agents, device, &sc))) return rc;
    srb12_ctx *c = new srb12_ctx();
    std::memset(c, 0, sizeof *c);
    // a failure after this point unwinds through srb12_ctx_destroy (it null-checks every buffer and
    // destroys the selection context); *out stays untouched
#define CREATE_CHK(expr)                                                                                \
    do {                                                                                                \
        hipError_t e_ = (expr);                                                                         \
        if (e_ != hipSuccess) {                                                                         \
            const int rc_ = srb_internal_fail(SRB_ERR_HIP, (std::string(#expr ": ") + hipGetErrorString(e_)).c_str()); \
            srb12_ctx_destroy(c);   /* sets no error: the message above stays */                      \
            return rc_;                                                                                 \
        }                                                                                               \
    } while (0)
    c->p = *p; c->max_agents = max_agents; c->device = device; c->sel_ctx = sc;
    const size_t A = (size_t)max_agents, N = (size_t)p->N, nv = 24 * N + 1;
    CREATE_CHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    for (int i = 0; i < 3; i++) CREATE_CHK(hipEventCreate(&c->ev[i]));
    CREATE_CHK(hipEventCreateWithFlags(&c->done, hipEventDisableTiming));
    CREATE_CHK(hipMalloc(&c->pos, A * 4 * sizeof(double)));
    CREATE_CHK(hipMalloc(&c->sel, A * 2 * SRB_KNN_MAX * sizeof(int)));
    CREATE_CHK(hipMalloc(&c->x0, A * 12 * sizeof(double)));
    CREATE_CHK(hipMalloc(&c->xref, A * 12 * N * sizeof(double)));
    CREATE_CHK(hipMalloc(&c->foot, A * 12 * N * sizeof(double)));
    CREATE_CHK(hipMalloc(&c->contact, A * 4 * N * sizeof(int)));
    CREATE_CHK(hipMalloc(&c->x_qp, A * nv * sizeof(double)));
    CREATE_CHK(hipMalloc(&c->x, A * nv * sizeof(double)));
    CREATE_CHK(hipMalloc(&c->obj, A * sizeof(double)));
    CREATE_CHK(hipMalloc(&c->status, A * 2 * sizeof(int)));
    CREATE_CHK(hipMalloc(&c->iters, A * 2 * sizeof(int)));
    CREATE_CHK(hipMalloc(&c->dbg, SRB12_DBG_LEN * sizeof(double)));
    c->dbg_agent = -1; c->timing = 1;
#undef CREATE_CHK
    *out = c;
    return SRB_OK;
}

extern "C" int srb12_ctx_destroy(srb12_ctx *c)
{
    if (!c) return SRB_OK;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->any) (void)hipEventSynchronize(c->done);
    void *bufs[] = {c->dbg, c->pos, c->sel, c->x0, c->xref, c->foot, c->contact, c->obstacles, c->nbr, c->x_qp, c->x, c->obj,
                    c->status, c->iters};
    for (void *b : bufs)
        if (b) (void)hipFree(b);
    for (int i = 0; i < 3; i++)
        if (c->ev[i]) (void)hipEventDestroy(c->ev[i]);
    if (c->done) (void)hipEventDestroy(c->done);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    srb_ctx_destroy(c->sel_ctx);
    delete c;
    return SRB_OK;
}

static int order12(srb12_ctx *c, hipStream_t s)
{
    if (c->any && s != c->last) H12CHK(hipStreamWaitEvent(s, c->done, 0));
    return SRB_OK;
}

// "up to K nearest": the rows selected per agent, clamped to what the tables hold (batch-uniform, as
// the LIP mode) and 0 without the NLP stage -- the launch and the host copy-back of sel use this one rule
static void clamp_rows(const srb12_params *p, const srb12_batch *d, int *Ko, int *Kn)
{
    int ko = p->K_obs, kn = p->K_nbr;
    if (ko > d->n_obs) ko = d->n_obs > 0 ? d->n_obs : 0;
    const int others = d->nbr_state ? d->n_all - 1 : 0;
    if (kn > others) kn = others > 0 ? others : 0;
    if (!p->use_nlp) ko = kn = 0;
    *Ko = ko; *Kn = kn;
}

static int launch12(srb12_ctx *c, int n_agents, const srb12_batch *d, hipStream_t s)
{
    if (n_agents < 0 || n_agents > c->max_agents) return srb_internal_fail(SRB_ERR_ARG, "n_agents exceeds max_agents");
    if (n_agents == 0) return SRB_OK;
    const srb12_params *p = &c->p;
    if (!d->x0 || !d->xref || !d->foot || !d->contact || !d->x || !d->obj || !d->status || !d->iters)
        return srb_internal_fail(SRB_ERR_ARG, "missing buffer");
    if (p->use_nlp && p->K_obs > 0 && (d->n_obs < 0 || (d->n_obs > 0 && !d->obstacles)))
        return srb_internal_fail(SRB_ERR_ARG, "obstacles missing");
    if (p->use_nlp && p->K_nbr > 0 && d->nbr_state && (d->agent_offset < 0 || d->agent_offset + n_agents > d->n_all))
        return srb_internal_fail(SRB_ERR_ARG, "agent_offset out of range of the neighbour table");
    int Ko = 0, Kn = 0;
    clamp_rows(p, d, &Ko, &Kn);
    Srb12KParams k = make_k12(p, Ko, Kn);
    k.dbg_agent = c->dbg_agent; k.dbg = c->dbg;
    const srb12_inst *in = pick12(p->N, Ko + Kn);
    if (!in) return srb_internal_fail(SRB_ERR_SIZE, "no SRB-12 kernel instance covers the row slots");
    const size_t lds = (size_t)srb12_lds_doubles(p->N, Ko + Kn) * sizeof(double);
    int *sel = d->sel ? d->sel : c->sel;
    if (c->timing) H12CHK(hipEventRecord(c->ev[0], s));
    if (Ko + Kn > 0) {
        hipLaunchKernelGGL(srb12_pos_kernel, dim3((n_agents + 255) / 256), dim3(256), 0, s, n_agents, d->x0, c->pos);
        H12CHK(hipGetLastError());
        int rc = srb_internal_select(c->sel_ctx, n_agents, c->pos, d->obstacles, Ko > 0 ? d->n_obs : 0, d->nbr_state,
                                     Kn > 0 ? d->n_all : 0, d->agent_offset, Ko, Kn, d->obstacles_version, sel, s);
        if (rc) return rc;
        // the selection context's own ordering event: its grid buffers are reallocated only after
        // this launch (grid_reserve waits on it)
        if ((rc = srb_internal_mark_done(c->sel_ctx, s))) return rc;
    }
    if (c->timing) H12CHK(hipEventRecord(c->ev[1], s));
    hipLaunchKernelGGL(in->fn, dim3(n_agents), dim3(64), lds, s, k, n_agents, d->x0, d->xref, d->foot, d->contact,
                       d->obstacles, d->nbr_state, (const int *)sel, d->x_qp, d->x, d->obj, d->status, d->iters);
    H12CHK(hipGetLastError());
    if (c->timing) H12CHK(hipEventRecord(c->ev[2], s));
    c->timed = c->timing != 0;
    return SRB_OK;
}

extern "C" int srb12_solve_batch_device(srb12_ctx *c, int n_agents, const srb12_batch *d, void *stream)
{
    if (d && d->struct_size != (int)sizeof(srb12_batch))
        return srb_internal_fail(SRB_ERR_ARG, "srb12_batch.struct_size != sizeof(srb12_batch): caller built against another ABI");
    if (!c || !d) return srb_internal_fail(SRB_ERR_ARG, "null argument");
    H12CHK(hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;
    int rc = order12(c, s);
    if (!rc) rc = launch12(c, n_agents, d, s);
    if (!rc && n_agents > 0) {
        H12CHK(hipEventRecord(c->done, s));
        c->last = s; c->any = true;
    }
    return rc;
}

static int reserve(void **buf, size_t *cap, size_t bytes, srb12_ctx *c)
{
    if (bytes <= *cap) return SRB_OK;
    if (c->any) H12CHK(hipEventSynchronize(c->done));
    if (*buf) H12CHK(hipFree(*buf));
    H12CHK(hipMalloc(buf, bytes));
    *cap = bytes;
    return SRB_OK;
}

extern "C" int srb12_solve_batch(srb12_ctx *c, int n_agents, const srb12_batch *h)
{
    if (h && h->struct_size != (int)sizeof(srb12_batch))
        return srb_internal_fail(SRB_ERR_ARG, "srb12_batch.struct_size != sizeof(srb12_batch): caller built against another ABI");
    if (!c || !h) return srb_internal_fail(SRB_ERR_ARG, "null argument");
    if (n_agents < 0 || n_agents > c->max_agents) return srb_internal_fail(SRB_ERR_ARG, "n_agents exceeds max_agents");
    if (n_agents == 0) return SRB_OK;
    if (!h->x0 || !h->xref || !h->foot || !h->contact || !h->x || !h->obj || !h->status || !h->iters)
        return srb_internal_fail(SRB_ERR_ARG, "missing buffer");
    H12CHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    if (int rc0 = order12(c, s)) return rc0;
    const size_t A = (size_t)n_agents, N = (size_t)c->p.N, nv = 24 * N + 1;
    H12CHK(hipMemcpyAsync(c->x0, h->x0, A * 12 * sizeof(double), hipMemcpyHostToDevice, s));
    H12CHK(hipMemcpyAsync(c->xref, h->xref, A * 12 * N * sizeof(double), hipMemcpyHostToDevice, s));
    H12CHK(hipMemcpyAsync(c->foot, h->foot, A * 12 * N * sizeof(double), hipMemcpyHostToDevice, s));
    H12CHK(hipMemcpyAsync(c->contact, h->contact, A * 4 * N * sizeof(int), hipMemcpyHostToDevice, s));
    srb12_batch d = *h;
    d.x0 = c->x0; d.xref = c->xref; d.foot = c->foot; d.contact = c->contact;
    d.x_qp = c->x_qp; d.x = c->x; d.obj = c->obj; d.status = c->status; d.iters = c->iters;
    d.sel = h->sel ? c->sel : nullptr;
    d.obstacles = nullptr; d.nbr_state = nullptr;
    if (h->n_obs > 0 && h->obstacles) {
        size_t cap = c->cap_obs;
        if (int rc = reserve((void **)&c->obstacles, &cap, (size_t)h->n_obs * 2 * sizeof(double), c)) return rc;
        c->cap_obs = cap;
        H12CHK(hipMemcpyAsync(c->obstacles, h->obstacles, (size_t)h->n_obs * 2 * sizeof(double), hipMemcpyHostToDevice, s));
        d.obstacles = c->obstacles;
    }
    if (h->n_all > 0 && h->nbr_state) {
        size_t cap = c->cap_nbr;
        if (int rc = reserve((void **)&c->nbr, &cap, (size_t)h->n_all * 4 * sizeof(double), c)) return rc;
        c->cap_nbr = cap;
        H12CHK(hipMemcpyAsync(c->nbr, h->nbr_state, (size_t)h->n_all * 4 * sizeof(double), hipMemcpyHostToDevice, s));
        d.nbr_state = c->nbr;
    }
    d.obstacles_version = 0;               // staging copies: no grid reuse across calls
    int rc = launch12(c, n_agents, &d, s);
    if (rc) return rc;
    H12CHK(hipEventRecord(c->done, s));
    c->last = s; c->any = true;
    if (h->x_qp) H12CHK(hipMemcpyAsync(h->x_qp, c->x_qp, A * nv * sizeof(double), hipMemcpyDeviceToHost, s));
    H12CHK(hipMemcpyAsync(h->x, c->x, A * nv * sizeof(double), hipMemcpyDeviceToHost, s));
    H12CHK(hipMemcpyAsync(h->obj, c->obj, A * sizeof(double), hipMemcpyDeviceToHost, s));
    H12CHK(hipMemcpyAsync(h->status, c->status, A * 2 * sizeof(int), hipMemcpyDeviceToHost, s));
    H12CHK(hipMemcpyAsync(h->iters, c->iters, A * 2 * sizeof(int), hipMemcpyDeviceToHost, s));
    if (h->sel) {
        int Ko = 0, Kn = 0;
        clamp_rows(&c->p, h, &Ko, &Kn);
        const int Kt = Ko + Kn;
        if (Kt > 0) H12CHK(hipMemcpyAsync(h->sel, c->sel, A * Kt * sizeof(int), hipMemcpyDeviceToHost, s));
    }
    H12CHK(hipStreamSynchronize(s));
    return SRB_OK;
}

extern "C" int srb12_ctx_set_timing(srb12_ctx *c, int on)
{
    if (!c) return srb_internal_fail(SRB_ERR_ARG, "null ctx");
    c->timing = on ? 1 : 0;
    return SRB_OK;
}

extern "C" int srb12_last_kernel_ms(srb12_ctx *c, float *select_ms, float *solve_ms)
{
    if (!c || !c->timed) return srb_internal_fail(SRB_ERR_ARG, "no timed launch");
    H12CHK(hipEventSynchronize(c->ev[2]));
    float a = 0, b = 0;
    H12CHK(hipEventElapsedTime(&a, c->ev[0], c->ev[1]));
    H12CHK(hipEventElapsedTime(&b, c->ev[1], c->ev[2]));
    if (select_ms) *select_ms = a;
    if (solve_ms) *solve_ms = b;
    return SRB_OK;
}

// diagnostics (not in the public header): agent >= 0 records a per-iteration trace on the next
// calls (|r_d|, its threshold, |r_p|, mu, ap, ad, delta, sigma per iteration, QP then NLP);
// out != NULL copies the last trace [2][64][8] + 16 phase-cycle sums (-DSRB12_STAMPS builds) to the host
extern "C" int srb12_debug_trace(srb12_ctx *c, int agent, double *out)
{
    if (!c) return srb_internal_fail(SRB_ERR_ARG, "null ctx");
    H12CHK(hipSetDevice(c->device));
    if (out) {
        if (c->any) H12CHK(hipEventSynchronize(c->done));
        H12CHK(hipMemcpy(out, c->dbg, (2 * 64 * 8 + 16) * sizeof(double), hipMemcpyDeviceToHost));
    }
    c->dbg_agent = agent;
    H12CHK(hipMemset(c->dbg, 0, SRB12_DBG_LEN * sizeof(double)));
    return SRB_OK;
}

// diagnostics (not in the public header): the 128 state checks of the traced agent that a -DSRB12_CHECK
// build records in its polish (srb12_kernels.hip S12CK; tools/srb12_check.py); zeros in other builds
extern "C" int srb12_debug_check(srb12_ctx *c, double *out)
{
    if (!c || !out) return srb_internal_fail(SRB_ERR_ARG, "null argument");
    H12CHK(hipSetDevice(c->device));
    if (c->any) H12CHK(hipEventSynchronize(c->done));
    H12CHK(hipMemcpy(out, c->dbg + (2 * 64 * 8 + 16), 128 * sizeof(double), hipMemcpyDeviceToHost));
    return SRB_OK;
}
