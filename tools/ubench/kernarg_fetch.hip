// Diagnostic (not product code): where the configs[2] solve kernel's per-agent HBM fetch beyond its
// inputs comes from (tools/traffic_ab.py measured 1506 B per agent against 716 B of
// inputs).  Two suspects, each isolated by a kernel pair run at 1024 and 4096 workgroups under
// rocprofv3 --pmc FETCH_SIZE (and WRITE_SIZE in its own pass):
//   karg_byval / karg_byptr   every workgroup reads a 640-B parameter block -- passed by value (the
//                             kernel-argument segment, like SrbKParams) or through a device pointer
//   wr_packed / wr_aligned    every workgroup writes 81 doubles -- packed at an 81-double stride (the
//                             solve kernel's x[A][nv], rows straddle 128-B lines) or at a 96-double stride
// Per-workgroup FETCH_SIZE of byval minus byptr = the argument block fetched per workgroup; packed
// minus aligned = fills of partially written lines.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench/kernarg_fetch tools/ubench/kernarg_fetch.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

struct Big { double v[80]; };

__global__ void __launch_bounds__(64) karg_byval(Big p, double *__restrict__ out)
{
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 80; i++) s += p.v[i] * (double)(i + 1);
    if (threadIdx.x == 0) out[blockIdx.x * 16] = s;
}

__global__ void __launch_bounds__(64) karg_byptr(const Big *__restrict__ p, double *__restrict__ out)
{
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 80; i++) s += p->v[i] * (double)(i + 1);
    if (threadIdx.x == 0) out[blockIdx.x * 16] = s;
}

__global__ void __launch_bounds__(64) wr_packed(double *__restrict__ out, double v)
{
    for (int i = threadIdx.x; i < 81; i += 64) out[blockIdx.x * 81 + i] = v + i;
}

__global__ void __launch_bounds__(64) wr_aligned(double *__restrict__ out, double v)
{
    for (int i = threadIdx.x; i < 81; i += 64) out[blockIdx.x * 96 + i] = v + i;
}

// evicts the L2 lines the previous kernels left (64 MB of writes, 8 MB per XCD)
__global__ void __launch_bounds__(256) l2_sweep(double *__restrict__ a, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = (double)i;
}

int main()
{
    Big h;
    for (int i = 0; i < 80; i++) h.v[i] = 1.0 / (i + 1);
    Big *dp = nullptr;
    double *out = nullptr, *out2 = nullptr, *sw = nullptr;
    const int maxb = 4096;
    const size_t nsw = (size_t)8 << 20;
    CHK(hipMalloc(&sw, nsw * sizeof(double)));
    CHK(hipMalloc(&out2, (size_t)maxb * 96 * sizeof(double)));
    CHK(hipMalloc(&dp, sizeof(Big)));
    CHK(hipMalloc(&out, (size_t)maxb * 96 * sizeof(double)));
    CHK(hipMemcpy(dp, &h, sizeof(Big), hipMemcpyHostToDevice));
    CHK(hipMemset(out, 0, (size_t)maxb * 96 * sizeof(double)));
    CHK(hipDeviceSynchronize());
    const int grids[2] = {1024, 4096};
    for (int g : grids)
        for (int rep = 0; rep < 3; rep++) {
            karg_byval<<<g, 64>>>(h, out);
            karg_byptr<<<g, 64>>>(dp, out);
            l2_sweep<<<2048, 256>>>(sw, nsw);
            wr_packed<<<g, 64>>>(out, 1.0 + rep);
            l2_sweep<<<2048, 256>>>(sw, nsw);
            wr_aligned<<<g, 64>>>(out2, 2.0 + rep);
            CHK(hipGetLastError());
            CHK(hipDeviceSynchronize());
        }
    double r;
    CHK(hipMemcpy(&r, out, sizeof r, hipMemcpyDeviceToHost));
    printf("{\"grids\": [1024, 4096], \"reps\": 3, \"check\": %.3f}\n", r);
    CHK(hipFree(dp));
    CHK(hipFree(out));
    CHK(hipFree(out2));
    CHK(hipFree(sw));
    return 0;
}
