// Diagnostic (round 6): where the neighbour selection's time goes at configs[2] -- the brute-force path of
// srb_wave.h knn_select_k (1024 agents, one 64-lane wave each, a 1024-row [x, y, xdot, ydot] table, K = 8),
// restated here with switches that remove one piece at a time.  Not product code.
//   hipcc --offload-arch=gfx950 -O3 -I srb-cbf-nmpc_amd/csrc tools/ubench/knn_phase.hip -o tools/ubench/knn_phase
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "srb_kernel_params.h"
#include "srb_wave.h"

// MODE bits: 1 no sqrt (the key is d^2), 2 no insertion (lane min only), 4 no pop rounds, 8 no table loads
// (rows from registers), 16 empty kernel (store only)
template <int MODE, int U>
__global__ void __launch_bounds__(64) kp(int n_agents, const double *x0g, const double *tab, int n_rows, int K, int *sel_out,
                                         unsigned long long *cyc)
{
#pragma clang fp contract(off)
    const int agent = blockIdx.x, lane = threadIdx.x;
    int *sel = sel_out + (size_t)agent * 8;
    if (MODE & 16) { if (lane < K) sel[lane] = lane; return; }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const double px = x0g[4 * (size_t)agent], py = x0g[4 * (size_t)agent + 2];
    constexpr int KM = 8;
    double bd[KM]; int bi[KM];
#pragma unroll
    for (int j = 0; j < KM; j++) { bd[j] = __builtin_inf(); bi[j] = 0x7fffffff; }
    double wq = __builtin_inf();
    const int self = agent;
    for (int i0 = lane; i0 < n_rows; i0 += U * 64) {
        double tx[U], ty[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int i = i0 + u * 64;
            const bool in = i < n_rows;
            if (MODE & 8) { tx[u] = (double)(i & 31); ty[u] = (double)(i >> 5); }
            else { tx[u] = in ? tab[(size_t)4 * i] : 0.0; ty[u] = in ? tab[(size_t)4 * i + 1] : 0.0; }
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int i = i0 + u * 64;
            if (i >= n_rows) continue;
            const double dx = px - tx[u], dy = py - ty[u];
            const double d2 = dx * dx + dy * dy;
            if (MODE & 2) { if (i != self && d2 < bd[0]) { bd[0] = d2; bi[0] = i; } continue; }
            if (i == self || !(d2 <= wq)) continue;
            knn_insert<KM>(bd, bi, (MODE & 1) ? d2 : sqrt(d2), i, K);
#pragma unroll
            for (int j = 0; j < KM; j++)
                if (j == K - 1) wq = (MODE & 1) ? bd[j] : bd[j] * bd[j] * (1.0 + 1e-14);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    int mine = -1;
    if (!(MODE & 4)) {
#pragma clang loop unroll(disable)
        for (int j = 0; j < K; j++) {
            double d = bd[0]; int idx = bi[0];
            wargmin(d, idx);
            if (bi[0] == idx) {
#pragma unroll
                for (int t = 0; t + 1 < KM; t++) { bd[t] = bd[t + 1]; bi[t] = bi[t + 1]; }
                bd[KM - 1] = __builtin_inf(); bi[KM - 1] = 0x7fffffff;
            }
            if (lane == j) mine = idx;
        }
    } else {
        mine = bi[0];
    }
    const unsigned long long t2 = __builtin_amdgcn_s_memtime();
    if (lane < K) sel[lane] = mine;
    if (lane == 0) { cyc[2 * agent] = t1 - t0; cyc[2 * agent + 1] = t2 - t1; }
}

// round 6: the product's functions (srb_wave.h knn_thresh + the ballot-argmin pop rounds), stamped between
// them; BITS 1: skip the pop rounds
template <int BITS>
__global__ void __launch_bounds__(64) kq(int n_agents, const double *x0g, const double *tab, int n_rows, int K, int *sel_out,
                                         unsigned long long *cyc)
{
    const int agent = blockIdx.x, lane = threadIdx.x;
    int *sel = sel_out + (size_t)agent * 8;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const double px = x0g[4 * (size_t)agent], py = x0g[4 * (size_t)agent + 2];
    double bd[8]; int bi[8];
#pragma unroll
    for (int j = 0; j < 8; j++) { bd[j] = __builtin_inf(); bi[j] = 0x7fffffff; }
    knn_thresh<8, 16, 64>(lane, px, py, tab, 4, n_rows, agent, K, bd, bi);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    int mine = -1;
    if (!(BITS & 1)) {
#pragma clang loop unroll(disable)
        for (int j = 0; j < K; j++) {
            double d = bd[0]; int idx = bi[0];
            wargmin_b(d, idx);
            if (bi[0] == idx) {
#pragma unroll
                for (int t = 0; t + 1 < 8; t++) { bd[t] = bd[t + 1]; bi[t] = bi[t + 1]; }
                bd[7] = __builtin_inf(); bi[7] = 0x7fffffff;
            }
            if (lane == j) mine = idx;
        }
    } else mine = bi[0];
    const unsigned long long t2 = __builtin_amdgcn_s_memtime();
    if (lane < K) sel[lane] = mine;
    if (lane == 0) { cyc[2 * agent] = t1 - t0; cyc[2 * agent + 1] = t2 - t1; }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)
template <int MODE, int U>
int run(const char *name, int A, double *x0, double *tab, int n, int *sel, unsigned long long *cyc)
{
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    for (int i = 0; i < 5; i++) hipLaunchKernelGGL((kp<MODE, U>), dim3(A), dim3(64), 0, 0, A, x0, tab, n, 8, sel, cyc);
    CK(hipDeviceSynchronize());
    float best = 1e9f;
    for (int r = 0; r < 50; r++) {
        (void)hipEventRecord(a, 0);
        hipLaunchKernelGGL((kp<MODE, U>), dim3(A), dim3(64), 0, 0, A, x0, tab, n, 8, sel, cyc);
        (void)hipEventRecord(b, 0); (void)hipEventSynchronize(b);
        float ms = 0; (void)hipEventElapsedTime(&ms, a, b);
        best = ms < best ? ms : best;
    }
    std::vector<unsigned long long> h(2 * A);
    CK(hipMemcpy(h.data(), cyc, 2 * A * 8, hipMemcpyDeviceToHost));
    double s1 = 0, s2 = 0, m1 = 0;
    for (int i = 0; i < A; i++) { s1 += h[2 * i]; s2 += h[2 * i + 1]; m1 = h[2 * i] > m1 ? h[2 * i] : m1; }
    printf("%-34s best %7.2f us   scan %8.0f (max %8.0f) pop %7.0f memtime ticks/wave\n", name, best * 1000.0f,
           s1 / A, m1, s2 / A);
    return 0;
}

template <int BITS>
int runq(const char *name, int A, double *x0, double *tab, int n, int *sel, unsigned long long *cyc)
{
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    for (int i = 0; i < 5; i++) hipLaunchKernelGGL((kq<BITS>), dim3(A), dim3(64), 0, 0, A, x0, tab, n, 8, sel, cyc);
    CK(hipDeviceSynchronize());
    float best = 1e9f;
    for (int r = 0; r < 50; r++) {
        (void)hipEventRecord(a, 0);
        hipLaunchKernelGGL((kq<BITS>), dim3(A), dim3(64), 0, 0, A, x0, tab, n, 8, sel, cyc);
        (void)hipEventRecord(b, 0); (void)hipEventSynchronize(b);
        float ms = 0; (void)hipEventElapsedTime(&ms, a, b);
        best = ms < best ? ms : best;
    }
    std::vector<unsigned long long> h(2 * A);
    CK(hipMemcpy(h.data(), cyc, 2 * A * 8, hipMemcpyDeviceToHost));
    double s1 = 0, s2 = 0, m1 = 0;
    for (int i = 0; i < A; i++) { s1 += h[2 * i]; s2 += h[2 * i + 1]; m1 = h[2 * i] > m1 ? h[2 * i] : m1; }
    printf("%-34s best %7.2f us   scan %8.0f (max %8.0f) pop %7.0f memtime ticks/wave\n", name, best * 1000.0f,
           s1 / A, m1, s2 / A);
    return 0;
}

int main()
{
    const int A = 1024, n = 1024;
    std::vector<double> hx(4 * A), ht(4 * n);
    for (int i = 0; i < A; i++) {                   // agents on a jittered grid of a 64 m arena
        hx[4 * i] = (i % 32) * 2.0 + 0.37 * ((i * 7919) % 13) / 13.0;
        hx[4 * i + 2] = (i / 32) * 2.0 + 0.41 * ((i * 104729) % 17) / 17.0;
    }
    for (int i = 0; i < n; i++) { ht[4 * i] = hx[4 * i]; ht[4 * i + 1] = hx[4 * i + 2]; }
    double *x0, *tab; int *sel; unsigned long long *cyc;
    CK(hipMalloc(&x0, hx.size() * 8)); CK(hipMalloc(&tab, ht.size() * 8)); CK(hipMalloc(&sel, A * 8 * 4));
    CK(hipMalloc(&cyc, 2 * A * 8));
    CK(hipMemcpy(x0, hx.data(), hx.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(tab, ht.data(), ht.size() * 8, hipMemcpyHostToDevice));
    if (run<16, 4>("empty kernel", A, x0, tab, n, sel, cyc)) return 1;
    if (run<0, 4>("product shape (U = 4)", A, x0, tab, n, sel, cyc)) return 1;
    if (run<0, 8>("U = 8", A, x0, tab, n, sel, cyc)) return 1;
    if (run<0, 16>("U = 16 (every load first)", A, x0, tab, n, sel, cyc)) return 1;
    if (run<1, 4>("no sqrt", A, x0, tab, n, sel, cyc)) return 1;
    if (run<2, 4>("no insertion", A, x0, tab, n, sel, cyc)) return 1;
    if (run<4, 4>("no pop rounds", A, x0, tab, n, sel, cyc)) return 1;
    if (run<8, 4>("no table loads", A, x0, tab, n, sel, cyc)) return 1;
    if (run<8 | 2, 4>("no loads, no insertion", A, x0, tab, n, sel, cyc)) return 1;
    if (runq<0>("round 6: knn_thresh + ballot pop", A, x0, tab, n, sel, cyc)) return 1;
    if (runq<1>("round 6: knn_thresh only", A, x0, tab, n, sel, cyc)) return 1;
    return 0;
}
