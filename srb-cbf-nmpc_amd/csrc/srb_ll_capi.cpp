// Host side of the low-level CLF-QP entry points of include/srbnmpc.h (srb_ll_*).
//
// The context owns device staging sized for max_agents (used by the host-buffer entry
// point), one HIP stream and an event pair around each kernel launch.  Per call the host
// only folds the CLF constants (LowLevelCtrl.cpp:176-185) and launches srb_ll_kernel with
// one 64-lane workgroup per agent.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstring>
#include <string>
#include "srbnmpc.h"
#include "srb_kernel_params.h"

int srb_internal_fail(int code, const char *msg);

struct SrbLLDev {   // must match srb_llctrl.hip
    const int *ind;
    const double *q, *dq, *Dinv, *B, *Hv, *Jc, *dJc, *Js, *Jtoe, *Jhip, *toePos, *hipPos, *H0, *dH0, *y, *dy, *hd,
        *dhd, *fDes;
    double *tau, *QP_force, *ddq, *dq_out, *q_out, *V, *dV, *x;
    int *status, *iters;
};
extern "C" __global__ void srb_ll_kernel(SrbLLKParams prm, int n_agents, SrbLLDev io);

#define LLCHK(expr)                                                                                     \
    do {                                                                                                \
        hipError_t e_ = (expr);                                                                         \
        if (e_ != hipSuccess)                                                                           \
            return srb_internal_fail(SRB_ERR_HIP, (std::string(#expr ": ") + hipGetErrorString(e_)).c_str()); \
    } while (0)

// per-agent element counts of every srb_ll_io array, in SrbLLDev order
static const int kInCount[] = {18, 18, 18 * 18, 12 * 18, 18, 18 * 12, 12, 18 * 12, 18 * 12, 18 * 12, 12, 12,
                               18 * 18, 18, 18, 18, 18, 18, 12};
static const int kOutCount[] = {18, 12, 18, 18, 18, 1, 1, 32};
#define LL_NIN 19
#define LL_NOUT 8

struct srb_ll_ctx {
    srb_ll_params p;
    int max_agents, device;
    hipStream_t stream;
    hipEvent_t ev[2];
    hipEvent_t done;               // recorded after every call's work (submission-order chaining)
    hipStream_t last;              // stream of the previous call
    bool timed, any;
    int *ind, *status, *iters;
    double *in[LL_NIN], *outb[LL_NOUT];
};

extern "C" void srb_ll_params_default(srb_ll_params *p)
{
    std::memset(p, 0, sizeof(*p));
    p->mu = 0.7; p->kp = 700; p->kd = 40; p->useCLF = 1;
    p->tauPen = 1e0; p->dfPen = 1e-1; p->auxPen = 1e6; p->clfPen = 1e8;
    p->auxMax = 100; p->clfEps = 0.8;
    p->maxit = 25; p->tol = 1e-6;
}

static int validate_ll(const srb_ll_params *p)
{
    if (!p) return srb_internal_fail(SRB_ERR_ARG, "null params");
    if (!(p->kp > 0) || !(p->kd > 0) || !(p->clfEps > 0) || !(p->tauPen > 0) || !(p->dfPen > 0) ||
        !(p->auxPen > 0) || (p->useCLF && !(p->clfPen > 0)) || !(p->mu >= 0) || p->maxit < 0 || !(p->tol > 0))
        return srb_internal_fail(SRB_ERR_ARG, "srb_ll_params out of range (penalties, gains, clfEps, tol > 0)");
    return SRB_OK;
}

// CLF Lyapunov constants of LowLevelCtrl::constraints (:176-190, :233)
static SrbLLKParams make_llk(const srb_ll_params *p)
{
    SrbLLKParams k;
    std::memset(&k, 0, sizeof k);
    const double kp = p->kp, kd = p->kd, e = p->clfEps;
    const double P1 = (kd * kd + kp * kp + kp) / (2 * kp * kd), Pd = 1 / (2 * kp), P2 = (kp + 1) / (2 * kd * kp);
    const double cc = 1.0 / (0.5 * (P1 + P2 + std::sqrt(P1 * P1 - 2 * P1 * P2 + P2 * P2 + 4 * Pd * Pd)));
    k.mus = p->mu / std::sqrt(2.0);
    k.kp = kp; k.kd = kd;
    k.tauPen = p->tauPen; k.dfPen = p->dfPen; k.auxPen = p->auxPen; k.clfPen = p->clfPen;
    k.p1e2 = P1 / (e * e); k.pde = Pd / e; k.p2 = P2;
    k.cce = cc / e;
    k.tol = p->tol;
    k.useCLF = p->useCLF ? 1 : 0;
    k.maxit = p->maxit;
    k.dbg_agent = -1;
    return k;
}

extern "C" int srb_ll_ctx_create(const srb_ll_params *p, int max_agents, int device, srb_ll_ctx **out)
{
    if (!out || max_agents <= 0) return srb_internal_fail(SRB_ERR_ARG, "bad arguments");
    int rc = validate_ll(p);
    if (rc) return rc;
    int ndev = 0;
    LLCHK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return srb_internal_fail(SRB_ERR_ARG, "device index out of range");
    LLCHK(hipSetDevice(device));
    srb_ll_ctx *c = new srb_ll_ctx();
    std::memset(c, 0, sizeof *c);
    c->p = *p; c->max_agents = max_agents; c->device = device;
    const size_t A = (size_t)max_agents;
    LLCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    for (int i = 0; i < 2; i++) LLCHK(hipEventCreate(&c->ev[i]));
    LLCHK(hipEventCreateWithFlags(&c->done, hipEventDisableTiming));
    LLCHK(hipMalloc(&c->ind, A * 4 * sizeof(int)));
    LLCHK(hipMalloc(&c->status, A * sizeof(int)));
    LLCHK(hipMalloc(&c->iters, A * sizeof(int)));
    for (int i = 0; i < LL_NIN; i++) LLCHK(hipMalloc(&c->in[i], A * kInCount[i] * sizeof(double)));
    for (int i = 0; i < LL_NOUT; i++) LLCHK(hipMalloc(&c->outb[i], A * kOutCount[i] * sizeof(double)));
    *out = c;
    return SRB_OK;
}

extern "C" int srb_ll_ctx_destroy(srb_ll_ctx *c)
{
    if (!c) return SRB_OK;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    if (c->any) (void)hipEventSynchronize(c->done);     // the last launch may be on another stream
    (void)hipFree(c->ind); (void)hipFree(c->status); (void)hipFree(c->iters);
    for (int i = 0; i < LL_NIN; i++) (void)hipFree(c->in[i]);
    for (int i = 0; i < LL_NOUT; i++) (void)hipFree(c->outb[i]);
    for (int i = 0; i < 2; i++) (void)hipEventDestroy(c->ev[i]);
    (void)hipEventDestroy(c->done);
    (void)hipStreamDestroy(c->stream);
    delete c;
    return SRB_OK;
}

// diagnostics (srb_llctrl.hip; not part of the public header)
extern "C" int srb_ll_dbg_agent(void);

static SrbLLDev to_dev(const srb_ll_io *d)
{
    SrbLLDev k;
    k.ind = d->ind;
    k.q = d->q; k.dq = d->dq; k.Dinv = d->Dinv; k.B = d->B; k.Hv = d->H; k.Jc = d->Jc; k.dJc = d->dJc; k.Js = d->Js;
    k.Jtoe = d->Jtoe; k.Jhip = d->Jhip; k.toePos = d->toePos; k.hipPos = d->hipPos; k.H0 = d->H0; k.dH0 = d->dH0;
    k.y = d->y; k.dy = d->dy; k.hd = d->hd; k.dhd = d->dhd; k.fDes = d->fDes;
    k.tau = d->tau; k.QP_force = d->QP_force; k.ddq = d->ddq; k.dq_out = d->dq_out; k.q_out = d->q_out;
    k.V = d->V; k.dV = d->dV; k.x = d->x; k.status = d->status; k.iters = d->iters;
    return k;
}

// calls on one context run in submission order (include/srbnmpc.h, "Ordering"): a call on
// another stream than the previous one first waits for that call's work
static int ll_order(srb_ll_ctx *c, hipStream_t s)
{
    if (c->any && s != c->last) LLCHK(hipStreamWaitEvent(s, c->done, 0));
    return SRB_OK;
}

static int ll_done(srb_ll_ctx *c, hipStream_t s)
{
    LLCHK(hipEventRecord(c->done, s));
    c->last = s; c->any = true;
    return SRB_OK;
}

static int ll_launch(srb_ll_ctx *c, int n_agents, SrbLLDev k, hipStream_t s)
{
    const void *need[] = {k.ind, k.q, k.dq, k.Dinv, k.B, k.Hv, k.Jc, k.dJc, k.Js, k.Jtoe, k.Jhip, k.toePos,
                          k.hipPos, k.H0, k.dH0, k.y, k.dy, k.hd, k.dhd, k.fDes, k.tau, k.QP_force, k.ddq,
                          k.dq_out, k.q_out, k.V, k.dV, k.x, k.status, k.iters};
    for (const void *b : need)
        if (!b) return srb_internal_fail(SRB_ERR_ARG, "missing srb_ll_io buffer");
    SrbLLKParams prm = make_llk(&c->p);
    prm.dbg_agent = srb_ll_dbg_agent();
    LLCHK(hipEventRecord(c->ev[0], s));
    hipLaunchKernelGGL(srb_ll_kernel, dim3(n_agents), dim3(64), 0, s, prm, n_agents, k);
    LLCHK(hipGetLastError());
    LLCHK(hipEventRecord(c->ev[1], s));
    c->timed = true;
    return SRB_OK;
}

extern "C" int srb_ll_calc_torque_device(srb_ll_ctx *c, int n_agents, const srb_ll_io *d, void *stream)
{
    if (d && d->struct_size != (int)sizeof(srb_ll_io))    // layout check first (no context needed)
        return srb_internal_fail(SRB_ERR_ARG, "srb_ll_io.struct_size != sizeof(srb_ll_io): caller built against another ABI");
    if (!c || !d) return srb_internal_fail(SRB_ERR_ARG, "null argument");
    if (n_agents < 0 || n_agents > c->max_agents) return srb_internal_fail(SRB_ERR_ARG, "n_agents exceeds max_agents");
    if (n_agents == 0) return SRB_OK;
    LLCHK(hipSetDevice(c->device));
    SrbLLDev k = to_dev(d);
    if (!k.x) k.x = c->outb[7];   // x is optional: the context's buffer absorbs it
    hipStream_t s = (hipStream_t)stream;                         // NULL: the HIP null stream
    int rc = ll_order(c, s);
    if (!rc) rc = ll_launch(c, n_agents, k, s);
    if (!rc) rc = ll_done(c, s);
    return rc;
}

extern "C" int srb_ll_calc_torque(srb_ll_ctx *c, int n_agents, const srb_ll_io *h)
{
    if (h && h->struct_size != (int)sizeof(srb_ll_io))    // layout check first (no context needed)
        return srb_internal_fail(SRB_ERR_ARG, "srb_ll_io.struct_size != sizeof(srb_ll_io): caller built against another ABI");
    if (!c || !h) return srb_internal_fail(SRB_ERR_ARG, "null argument");
    if (n_agents < 0 || n_agents > c->max_agents) return srb_internal_fail(SRB_ERR_ARG, "n_agents exceeds max_agents");
    if (n_agents == 0) return SRB_OK;
    LLCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    if (int rc0 = ll_order(c, s)) return rc0;
    const size_t A = (size_t)n_agents;
    const double *hin[LL_NIN] = {h->q, h->dq, h->Dinv, h->B, h->H, h->Jc, h->dJc, h->Js, h->Jtoe, h->Jhip,
                                 h->toePos, h->hipPos, h->H0, h->dH0, h->y, h->dy, h->hd, h->dhd, h->fDes};
    double *hout[LL_NOUT] = {h->tau, h->QP_force, h->ddq, h->dq_out, h->q_out, h->V, h->dV, h->x};
    if (!h->ind || !h->status || !h->iters) return srb_internal_fail(SRB_ERR_ARG, "missing srb_ll_io buffer");
    for (int i = 0; i < LL_NIN; i++)
        if (!hin[i]) return srb_internal_fail(SRB_ERR_ARG, "missing srb_ll_io input buffer");
    for (int i = 0; i < LL_NOUT - 1; i++)
        if (!hout[i]) return srb_internal_fail(SRB_ERR_ARG, "missing srb_ll_io output buffer");
    LLCHK(hipMemcpyAsync(c->ind, h->ind, A * 4 * sizeof(int), hipMemcpyHostToDevice, s));
    for (int i = 0; i < LL_NIN; i++)
        LLCHK(hipMemcpyAsync(c->in[i], hin[i], A * kInCount[i] * sizeof(double), hipMemcpyHostToDevice, s));
    LLCHK(hipMemcpyAsync(c->outb[0], h->tau, A * 18 * sizeof(double), hipMemcpyHostToDevice, s));   // tau is in/out
    srb_ll_io d;
    d.struct_size = sizeof d;
    d.ind = c->ind;
    d.q = c->in[0]; d.dq = c->in[1]; d.Dinv = c->in[2]; d.B = c->in[3]; d.H = c->in[4]; d.Jc = c->in[5];
    d.dJc = c->in[6]; d.Js = c->in[7]; d.Jtoe = c->in[8]; d.Jhip = c->in[9]; d.toePos = c->in[10];
    d.hipPos = c->in[11]; d.H0 = c->in[12]; d.dH0 = c->in[13]; d.y = c->in[14]; d.dy = c->in[15]; d.hd = c->in[16];
    d.dhd = c->in[17]; d.fDes = c->in[18];
    d.tau = c->outb[0]; d.QP_force = c->outb[1]; d.ddq = c->outb[2]; d.dq_out = c->outb[3]; d.q_out = c->outb[4];
    d.V = c->outb[5]; d.dV = c->outb[6]; d.x = c->outb[7]; d.status = c->status; d.iters = c->iters;
    int rc = ll_launch(c, n_agents, to_dev(&d), s);
    if (!rc) rc = ll_done(c, s);
    if (rc) return rc;
    for (int i = 0; i < LL_NOUT; i++)
        if (hout[i]) LLCHK(hipMemcpyAsync(hout[i], c->outb[i], A * kOutCount[i] * sizeof(double), hipMemcpyDeviceToHost, s));
    LLCHK(hipMemcpyAsync(h->status, c->status, A * sizeof(int), hipMemcpyDeviceToHost, s));
    LLCHK(hipMemcpyAsync(h->iters, c->iters, A * sizeof(int), hipMemcpyDeviceToHost, s));
    LLCHK(hipStreamSynchronize(s));
    return SRB_OK;
}

extern "C" int srb_ll_sync(srb_ll_ctx *c)
{
    if (!c) return srb_internal_fail(SRB_ERR_ARG, "null ctx");
    LLCHK(hipSetDevice(c->device));
    LLCHK(hipDeviceSynchronize());
    return SRB_OK;
}

extern "C" int srb_ll_last_kernel_ms(srb_ll_ctx *c, float *ms)
{
    if (!c || !c->timed) return srb_internal_fail(SRB_ERR_ARG, "no timed launch");
    LLCHK(hipEventSynchronize(c->ev[1]));
    float t = 0;
    LLCHK(hipEventElapsedTime(&t, c->ev[0], c->ev[1]));
    if (ms) *ms = t;
    return SRB_OK;
}
