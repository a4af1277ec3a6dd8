// Diagnostic (not product code): cost of an LDS store when many lanes of a wave write the SAME address
// (the SRB-12 factor's unconditional "sink" stores) against distinct addresses.  One wave, 4096 stores
// of 8 B per lane per pattern, s_memtime around each loop.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench/lds_same_addr tools/ubench/lds_same_addr.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void __launch_bounds__(64) lds_stores(unsigned long long *out, double v)
{
    __shared__ double buf[2048];
    const int lane = threadIdx.x;
    const int addr[4] = {lane,                                   // distinct
                         0,                                      // all lanes one address
                         (lane >= 12 && lane < 37) ? lane : 1000, // 39 lanes one address (the sink pattern)
                         1000 + (lane & 15)};                    // 16 addresses, 4 lanes each
    for (int p = 0; p < 4; p++) {
        volatile double *b = buf + addr[p];
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll 16
        for (int i = 0; i < 4096; i++) b[0] = v + i;
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) out[p] = t1 - t0;
    }
}

int main()
{
    unsigned long long *d, h[4];
    hipMalloc(&d, sizeof h);
    for (int rep = 0; rep < 3; rep++) {
        lds_stores<<<1, 64>>>(d, 1.0 + rep);
        hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    }
    printf("cycles per store instruction: distinct %.1f, one address %.1f, sink pattern (39 lanes) %.1f, 16 addresses x4 %.1f\n",
           h[0] / 4096.0, h[1] / 4096.0, h[2] / 4096.0, h[3] / 4096.0);
    hipFree(d);
    return 0;
}
