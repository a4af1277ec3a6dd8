// Diagnostic (not product code): single-wave latencies that set the solve kernel's per-iteration
// cycle count at one wave per SIMD (configs[2]):
//   (a) 64 dependent v_mfma_f64_16x16x4f64 on one accumulator (gram_rhs at NZL <= 16),
//   (b) the same 64 MFMAs over 4 independent accumulators,
//   (c) a dependent chain of 64 LDS double loads (index chasing),
//   (d) 64 workgroup barriers of a one-wave workgroup.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/mfma_lat.hip -o /tmp/mfma_lat && /tmp/mfma_lat
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(64) kern(const double *in, double *out, unsigned long long *cyc)
{
    __shared__ double lds[1024];
    __shared__ int idx[1024];
    const int lane = threadIdx.x;
    for (int i = lane; i < 1024; i += 64) { lds[i] = in[i & 63]; idx[i] = (i * 37 + 11) & 1023; }
    __syncthreads();
    double a = in[lane], b = in[(lane + 1) & 63];
    unsigned long long t[8];
    d4 acc = {0, 0, 0, 0}, c0 = acc, c1 = acc, c2 = acc, c3 = acc;
    __builtin_amdgcn_sched_barrier(0);
    t[0] = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 64; i++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    out[lane] = acc[0] + acc[1] + acc[2] + acc[3];     // waits for the chain
    __builtin_amdgcn_sched_barrier(0);
    t[1] = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 16; i++) {
        c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, b, c3, 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    out[64 + lane] = (c0[0] + c1[1]) + (c2[2] + c3[3]);
    __builtin_amdgcn_sched_barrier(0);
    t[2] = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
    int j = lane;
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 64; i++) { j = idx[j]; }
    s = lds[j];
    __builtin_amdgcn_sched_barrier(0);
    out[128 + lane] = s;
    __builtin_amdgcn_sched_barrier(0);
    t[3] = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 64; i++) __syncthreads();
    __builtin_amdgcn_sched_barrier(0);
    t[4] = __builtin_amdgcn_s_memtime();
    if (lane == 0)
        for (int i = 0; i < 4; i++) cyc[blockIdx.x * 4 + i] = t[i + 1] - t[i];
}

int main()
{
    double *in, *out;
    unsigned long long *cyc;
    hipMalloc(&in, 64 * sizeof(double)); hipMalloc(&out, 256 * sizeof(double));
    hipMalloc(&cyc, 1024 * 4 * sizeof(unsigned long long));
    double h[64];
    for (int i = 0; i < 64; i++) h[i] = 1.0 + 1e-3 * i;
    hipMemcpy(in, h, sizeof h, hipMemcpyHostToDevice);
    for (int grid : {1, 1024}) {
        kern<<<grid, 64>>>(in, out, cyc);
        kern<<<grid, 64>>>(in, out, cyc);
        hipDeviceSynchronize();
        unsigned long long hc[4096];
        hipMemcpy(hc, cyc, grid * 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
        double m[4] = {0, 0, 0, 0};
        for (int g = 0; g < grid; g++)
            for (int i = 0; i < 4; i++) m[i] += hc[4 * g + i] / (double)grid;
        // s_memtime counts at the 100 MHz reference clock on gfx950? report raw and per-op
        printf("grid %4d (s_memtime ticks / 64 ops): dependent MFMA %.1f, 4 chains %.1f, LDS load chain %.1f, barrier %.1f\n",
               grid, m[0] / 64, m[1] / 64, m[2] / 64, m[3] / 64);
    }
    return 0;
}
