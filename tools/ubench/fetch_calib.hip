// Diagnostic (not product code): calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for the
// access widths the solve kernels use (MI355X_MICROARCH.md, HBM section: only 16-B/lane
// streaming reads and stores are calibrated on gfx950; "calibrate on a known byte count in your
// own access pattern").  Three kernels over a 1 GiB buffer (4x the 256 MiB Infinity Cache, so
// every line comes from HBM), each touching every byte exactly once:
//   calib_read8    8-B/lane coalesced loads (the solve kernels' fp64 loads)
//   calib_read16   16-B/lane coalesced loads (the guide's calibrated pattern)
//   calib_write8   8-B/lane coalesced stores (the solve kernels' fp64 stores)
// Each read kernel writes one double per workgroup (negligible next to 1 GiB).  The expected
// byte count is printed; tools/pmc_traffic.py calib divides the counters by it.
//   hipcc --offload-arch=gfx950 -O3 -o fetch_calib tools/ubench/fetch_calib.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void calib_read8(const double *__restrict__ a, size_t n, double *__restrict__ out)
{
    double s = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
    __shared__ double red[256];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[blockIdx.x] = red[0];
}

__global__ void calib_read16(const double2 *__restrict__ a, size_t n2, double *__restrict__ out)
{
    double s = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x) {
        const double2 v = a[i];
        s += v.x + v.y;
    }
    __shared__ double red[256];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[blockIdx.x] = red[0];
}

__global__ void calib_write8(double *__restrict__ a, size_t n, double v)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = v + (double)(i & 7);
}

int main()
{
    const size_t bytes = (size_t)1 << 30, n = bytes / 8;
    const int blocks = 8192, threads = 256;
    double *a = nullptr, *out = nullptr;
    CHK(hipMalloc(&a, bytes));
    CHK(hipMalloc(&out, blocks * sizeof(double)));
    CHK(hipMemset(a, 0, bytes));
    CHK(hipDeviceSynchronize());
    for (int rep = 0; rep < 2; rep++) {
        calib_write8<<<blocks, threads>>>(a, n, 1.0 + rep);
        CHK(hipGetLastError());
        calib_read8<<<blocks, threads>>>(a, n, out);
        CHK(hipGetLastError());
        calib_read16<<<blocks, threads>>>((const double2 *)a, n / 2, out);
        CHK(hipGetLastError());
        CHK(hipDeviceSynchronize());
    }
    double h[4];
    CHK(hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost));
    printf("{\"bytes_per_dispatch\": %zu, \"check\": %.1f}\n", bytes, h[0]);
    CHK(hipFree(a));
    CHK(hipFree(out));
    return 0;
}
