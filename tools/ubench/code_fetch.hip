// Diagnostic (not product code): HBM fetch of a kernel's machine code per dispatch (VERDICT r04 item 5:
// the configs[2] solve kernel fetches 0.72 MB per launch beyond its 0.76 MB of code x 8 XCDs, its inputs and
// its table lines).  code_big executes ~4096 distinct FMAs with distinct constants once per workgroup
// (~100 KB of straight-line code), code_small 16 of them; both at 1024 and 4096 workgroups under
// rocprofv3 --pmc FETCH_SIZE.  The fixed part of code_big minus code_small against its code size tells
// how many times per dispatch each XCD fetches the code.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench/code_fetch tools/ubench/code_fetch.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)
#define F1 s = fma(s, 1.0 + (double)(__COUNTER__) * 1.0e-7, t);
#define F4 F1 F1 F1 F1
#define F16 F4 F4 F4 F4
#define F64 F16 F16 F16 F16
#define F256 F64 F64 F64 F64
#define F1024 F256 F256 F256 F256
#define F4096 F1024 F1024 F1024 F1024

__global__ void __launch_bounds__(64) code_big(const double *__restrict__ in, double *__restrict__ out)
{
    double s = in[threadIdx.x], t = in[64 + threadIdx.x];
    F4096
    out[blockIdx.x * 64 + threadIdx.x] = s;
}

__global__ void __launch_bounds__(64) code_small(const double *__restrict__ in, double *__restrict__ out)
{
    double s = in[threadIdx.x], t = in[64 + threadIdx.x];
    F16
    out[blockIdx.x * 64 + threadIdx.x] = s;
}

int main()
{
    double *in = nullptr, *out = nullptr;
    CHK(hipMalloc(&in, 128 * sizeof(double)));
    CHK(hipMalloc(&out, (size_t)4096 * 64 * sizeof(double)));
    CHK(hipMemset(in, 0, 128 * sizeof(double)));
    CHK(hipDeviceSynchronize());
    const int grids[2] = {1024, 4096};
    for (int g : grids)
        for (int rep = 0; rep < 3; rep++) {
            code_big<<<g, 64>>>(in, out);
            code_small<<<g, 64>>>(in, out);
            CHK(hipGetLastError());
            CHK(hipDeviceSynchronize());
        }
    printf("{\"grids\": [1024, 4096], \"reps\": 3}\n");
    CHK(hipFree(in));
    CHK(hipFree(out));
    return 0;
}
