// Diagnostic (not product code): cycles per register Gauss-Jordan inverse of an SPD
// NZL x NZL matrix held one row per lane, pivot-row broadcast by v_readlane (srb_wave.h
// gj_invert) against a 64-bit DPP row_newbcast broadcast (rows replicated in each 16-lane
// row of the wave).  Checks that both give the same inverse.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#define WAVE 64
#include "../../srb-cbf-nmpc_amd/csrc/srb_kernel_params.h"
#include "../../srb-cbf-nmpc_amd/csrc/srb_wave.h"

// value of lane k of this lane's 16-lane row (k folds to an immediate after unrolling)
__device__ __forceinline__ double bc16(double v, int k)
{
    switch (k) {
#define SRB_BC(K) case K: return __builtin_amdgcn_update_dpp(0.0, v, 0x150 + K, 0xf, 0xf, false);
    SRB_BC(0) SRB_BC(1) SRB_BC(2) SRB_BC(3) SRB_BC(4) SRB_BC(5) SRB_BC(6) SRB_BC(7)
    SRB_BC(8) SRB_BC(9) SRB_BC(10) SRB_BC(11) SRB_BC(12) SRB_BC(13) SRB_BC(14) default: SRB_BC(15)
#undef SRB_BC
    }
}

template <int NZL>
__device__ __forceinline__ int gj_dpp(double (&A)[NZL], int nz, int lane)
{
    int fail = 0;
    double cs = 1.0;
    const int r = lane & 15;
#pragma unroll
    for (int k = 0; k < NZL; k++) {
        double piv = bc16(A[k], k);
        fail |= !(piv > 0.0);
        const double inv = rcp_d(piv);
        const bool me = r == k;
        const double f = me ? 0.0 : A[k] * inv;
#pragma unroll
        for (int jj = 0; jj < NZL; jj++) {
            const int j = (k + 1 + jj) % NZL;
            if (j != k) A[j] = fma(-f, bc16(A[j], k), A[j]);
        }
        A[k] = me ? 1.0 : -f;
        cs = me ? inv : cs;
    }
#pragma unroll
    for (int j = 0; j < NZL; j++) A[j] *= cs;
    return fail;
}

template <int NZL, int MODE>
__global__ void kern(const double *M, double *out, unsigned long long *cyc, int reps)
{
    const int lane = threadIdx.x;
    const int row = MODE ? (lane & 15) : lane;
    double A[NZL];
    unsigned long long t0 = 0, t1 = 0;
    for (int rep = 0; rep < reps; rep++) {
#pragma unroll
        for (int j = 0; j < NZL; j++) A[j] = (row < NZL) ? M[row * NZL + j] : (row == j ? 1.0 : 0.0);
        __builtin_amdgcn_sched_barrier(0);
        if (rep == 1) t0 = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
        if (MODE) gj_dpp<NZL>(A, NZL, lane); else gj_invert<NZL>(A, NZL, lane, 0);
        __builtin_amdgcn_sched_barrier(0);
        double s = 0; for (int j = 0; j < NZL; j++) s += A[j];
        if (s == 12345.678) out[1000] = s;              // keep the work
    }
    __builtin_amdgcn_sched_barrier(0);
    t1 = __builtin_amdgcn_s_memtime();
    if (lane < NZL) for (int j = 0; j < NZL; j++) out[lane * NZL + j] = A[j];
    if (lane == 0) cyc[0] = (t1 - t0) / (reps - 1);
}

int main()
{
    constexpr int NZL = 12;
    double hM[NZL * NZL];
    for (int i = 0; i < NZL; i++)
        for (int j = 0; j < NZL; j++) hM[i * NZL + j] = 1.0 / (1 + i + j) + (i == j ? 2.0 + i : 0.0);
    double *dM, *dO; unsigned long long *dC;
    hipMalloc(&dM, sizeof hM); hipMalloc(&dO, 2048 * sizeof(double)); hipMalloc(&dC, 8);
    hipMemcpy(dM, hM, sizeof hM, hipMemcpyHostToDevice);
    double r0[NZL * NZL], r1[NZL * NZL]; unsigned long long c0, c1;
    for (int t = 0; t < 3; t++) {
        hipLaunchKernelGGL((kern<NZL, 0>), dim3(1), dim3(64), 0, 0, dM, dO, dC, 64);
        hipDeviceSynchronize(); hipMemcpy(r0, dO, sizeof r0, hipMemcpyDeviceToHost); hipMemcpy(&c0, dC, 8, hipMemcpyDeviceToHost);
        hipLaunchKernelGGL((kern<NZL, 1>), dim3(1), dim3(64), 0, 0, dM, dO, dC, 64);
        hipDeviceSynchronize(); hipMemcpy(r1, dO, sizeof r1, hipMemcpyDeviceToHost); hipMemcpy(&c1, dC, 8, hipMemcpyDeviceToHost);
    }
    double md = 0, mi = 0;
    for (int i = 0; i < NZL * NZL; i++) { md = fmax(md, fabs(r0[i] - r1[i])); mi = fmax(mi, fabs(r0[i])); }
    // residual of M * inv - I
    double res = 0;
    for (int i = 0; i < NZL; i++) for (int j = 0; j < NZL; j++) { double s = -(i == j); for (int k = 0; k < NZL; k++) s += hM[i * NZL + k] * r1[k * NZL + j]; res = fmax(res, fabs(s)); }
    printf("NZL=%d readlane GJ %llu cyc, dpp GJ %llu cyc, max|diff| %.3e (max|inv| %.3e), |M inv - I| %.3e\n", NZL, c0, c1, md, mi, res);
    return 0;
}
