// Kernel-side parameter block (host fills it from srb_params, see srb_capi.cpp).
#pragma once

#define SRB_MAX_K 32      // obstacle rows per grid (K_obs + K_nbr)
#define SRB_KNN_MAX 16    // neighbours per agent (K_nbr)
#define SRB_MAX_N 32      // reduced Newton system size bound: nz = N(C-1)+1 <= 32
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

// Z'HZ layout helpers: Z is n16 x ldz (rows to a multiple of 16, columns to a multiple of
// 16, zero padded); SRB_NCPL2 = both orientations of every off-diagonal coupling of H.
#define SRB_R16(x) ((((x) + 15) / 16) * 16)     /* term lists: whole 16-term MFMA trips */
#define SRB_LDZ(nz) ((((nz) + 15) / 16) * 16)
#define SRB_NCPL2(N) (2 * (2 * ((N) - 1) + 3 * (N)))

// doubles of dynamic LDS one agent needs; must match the carve in srb_nmpc_kernel
static inline int srb_lds_doubles(const SrbKParams &p)
{
    const int N = p.N, C = p.C, K = p.K_obs + p.K_nbr, n = p.n, nz = p.nz;
    const int mmax = p.use_nlp ? (p.mq + N * K + 4 * N) : p.mq;
    const int cpl16 = SRB_R16(SRB_NCPL2(N));
    return SRB_R16(n) * SRB_LDZ(nz) + 5 * n + SRB_R16(n) + 2 * cpl16 + 4 * N + 2 * C * N + 11 * mmax +
           (2 * N * K + 2) * 2 + (K + 1) + 4 * nz * nz + 6 * 64
#ifdef SRB_STAMPS
           + 64
#endif
        ;
}
