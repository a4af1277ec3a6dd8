// Kernel-side parameter block (host fills it from srb_params, see srb_capi.cpp).
#pragma once

#define SRB_MAX_K 32      // obstacle rows per grid (K_obs + K_nbr)
#define SRB_KNN_MAX 16    // neighbours per agent (K_nbr)
#define SRB_MAX_N 64      // lanes of one wave hold one xi entry each: nz = N(C-1)+1 <= 64
#define SRB_MAX_OBS 4096  // static obstacles (64 lanes x 64-bit chosen mask)
#define SRB_MAX_NV 256    // z_mul keeps 4 variables per lane

struct SrbKParams {
    int N, C, K_obs, K_nbr;
    int n, nz, mq, use_nlp;
    int qp_maxit, nlp_maxit;
    double Ad[16], Bd[8];                  // LIP discretisation (MPC_dist.cpp:126-127)
    double Qw, Pw, Rw, Sw, box, fr;        // gains (:172-175), box (:317), mu*h/sqrt(2) (:315)
    double eps_obs, eps_nbr, vsat, tol, Ts;
};

// doubles of dynamic LDS one agent needs; must match the carve in srb_nmpc_kernel
static inline int srb_lds_doubles(const SrbKParams &p)
{
    const int N = p.N, C = p.C, K = p.K_obs + p.K_nbr, n = p.n, nz = p.nz;
    const int mmax = p.use_nlp ? (p.mq + N * K + 4 * N) : p.mq;
    return n * nz + 6 * n + 4 * N + 2 * C * N + (2 * (N - 1) + 3 * N) + 11 * mmax +
           (2 * N * K + 2) * 2 + (K + 1) + 4 * nz * nz + 3 * nz;
}
