// Diagnostic: time of the obstacle / neighbour selection kernel shape (srb_wave.h knn_select)
// against an empty kernel of the same grid, and against its pieces.  Not product code.
//   hipcc --offload-arch=gfx950 -O3 -I srb-cbf-nmpc_amd/csrc tools/ubench/knn_bench.hip -o /tmp/knn_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "srb_kernel_params.h"
#include "srb_wave.h"

template <int KW, int MODE>
__global__ void __launch_bounds__(64 * KW) kb(int n_agents, const double *x0g, const double *obst, int n_obs,
                                              const double *nbr, int n_all, int Ko, int Kn, int *sel_out)
{
    __shared__ double wd_lds[KW];
    __shared__ int wi_lds[KW];
    const int agent = blockIdx.x, tid = threadIdx.x;
    int *sel = sel_out + (size_t)agent * (Ko + Kn);
    if (MODE == 0) { if (tid < Ko + Kn) sel[tid] = -1; return; }
    const double px = x0g[4 * (size_t)agent], py = x0g[4 * (size_t)agent + 2];
    if (Ko > 0) knn_select<KW>(tid, px, py, obst, 2, n_obs, -1, Ko, sel, wd_lds, wi_lds);
    if (MODE == 2 && Kn > 0) knn_select<KW>(tid, px, py, nbr, 4, n_all, agent, Kn, sel + Ko, wd_lds, wi_lds);
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)
template <int KW, int MODE>
float timeit(int A, double *x0, double *ob, int no, double *nb, int na, int Ko, int Kn, int *sel)
{
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    for (int i = 0; i < 3; i++) hipLaunchKernelGGL((kb<KW, MODE>), dim3(A), dim3(64 * KW), 0, 0, A, x0, ob, no, nb, na, Ko, Kn, sel);
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < 20; i++) hipLaunchKernelGGL((kb<KW, MODE>), dim3(A), dim3(64 * KW), 0, 0, A, x0, ob, no, nb, na, Ko, Kn, sel);
    (void)hipEventRecord(b, 0); (void)hipEventSynchronize(b);
    float ms = 0; (void)hipEventElapsedTime(&ms, a, b);
    return ms / 20 * 1000.0f;
}

int main()
{
    const int A = 1024, na = 1024, no = 20;
    std::vector<double> hx(4 * 4096), ho(2 * no), hn(4 * 4096);
    for (size_t i = 0; i < hx.size(); i++) hx[i] = (double)((i * 7919) % 1000) / 100.0;
    for (size_t i = 0; i < ho.size(); i++) ho[i] = (double)((i * 104729) % 900) / 100.0;
    hn = hx;
    double *x0, *ob, *nb; int *sel;
    CK(hipMalloc(&x0, hx.size() * 8)); CK(hipMalloc(&ob, ho.size() * 8)); CK(hipMalloc(&nb, hn.size() * 8));
    CK(hipMalloc(&sel, 4096 * 32 * 4));
    CK(hipMemcpy(x0, hx.data(), hx.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(ob, ho.data(), ho.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(nb, hn.data(), hn.size() * 8, hipMemcpyHostToDevice));
    printf("empty        KW=4: %8.2f us\n", timeit<4, 0>(A, x0, ob, no, nb, na, 3, 8, sel));
    printf("obst only    KW=4: %8.2f us\n", timeit<4, 1>(A, x0, ob, no, nb, na, 3, 8, sel));
    printf("obst+nbr     KW=4: %8.2f us\n", timeit<4, 2>(A, x0, ob, no, nb, na, 3, 8, sel));
    printf("obst+nbr     KW=1: %8.2f us\n", timeit<1, 2>(A, x0, ob, no, nb, na, 3, 8, sel));
    printf("obst+nbr K=1 KW=4: %8.2f us\n", timeit<4, 2>(A, x0, ob, no, nb, na, 1, 1, sel));
    return 0;
}
