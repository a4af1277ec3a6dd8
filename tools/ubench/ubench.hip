// Microbenchmark of single-wave latencies on gfx950 (diagnostic, not product code).
// Each test runs REP dependent repetitions of one pattern in one 64-lane wave and
// reports s_memtime cycles per repetition.
#include <hip/hip_runtime.h>
#include <cstdio>
#define REP 256
__device__ __forceinline__ double rdl(double v, int lane) {
  long long b = __double_as_longlong(v);
  int lo = __builtin_amdgcn_readlane((int)b, lane), hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
template <int CTRL> __device__ __forceinline__ double dppd(double v) {
  long long b = __double_as_longlong(v);
  int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xf, 0xf, false);
  int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__global__ void k(unsigned long long *out, double *sink, double seed) {
  __shared__ double lds[1024];
  const int t = threadIdx.x;
  double x = seed + t, y = 1.0 + 1e-9 * t;
  lds[t] = x; lds[t + 64] = y;
  __syncthreads();
  unsigned long long t0, t1; int slot = 0;
#define TIME(BODY) { __builtin_amdgcn_sched_barrier(0); t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); \
    for (int r = 0; r < REP; r++) { BODY; } __builtin_amdgcn_sched_barrier(0); t1 = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0); if (t == 0) out[slot] = t1 - t0; slot++; }
  // 0 empty loop
  TIME(asm volatile("" : "+v"(x)));
  // 1 dependent f64 fma
  TIME(x = fma(x, y, 1e-12); asm volatile("" : "+v"(x)));
  // 2 four independent fma chains (per rep: 4 fmas)
  double a = x, b = y, c = x + 1, d = y + 1;
  TIME(a = fma(a, y, 1e-12); b = fma(b, y, 1e-12); c = fma(c, y, 1e-12); d = fma(d, y, 1e-12); asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d)));
  x += a + b + c + d;
  // 3 LDS write -> read (other lane) round trip, dependent
  TIME(lds[t] = x; __builtin_amdgcn_wave_barrier(); x = lds[(t + 1) & 63] * y; asm volatile("" : "+v"(x)));
  // 4 readlane -> fma dependent
  TIME(x = fma(rdl(x, r & 63), y, 1e-12); asm volatile("" : "+v"(x)));
  // 5 rsq + 2 Newton, dependent
  TIME({ double q = __builtin_amdgcn_rsq(x); q = fma(0.5 * q, fma(-x * q, q, 1.0), q); q = fma(0.5 * q, fma(-x * q, q, 1.0), q); x = x * 0.5 + q; } asm volatile("" : "+v"(x)));
  // 6 DPP wave sum (4 dpp + 2 permlane swaps), dependent
  TIME({ double v = x; v += dppd<0xB1>(v); v += dppd<0x4E>(v); v += dppd<0x141>(v); v += dppd<0x140>(v);
         long long bb = __double_as_longlong(v); auto lo = __builtin_amdgcn_permlane32_swap((unsigned)bb, (unsigned)bb, false, false);
         auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(bb >> 32), (unsigned)(bb >> 32), false, false);
         v = __longlong_as_double(((long long)hi[0] << 32) | lo[0]) + __longlong_as_double(((long long)hi[1] << 32) | lo[1]);
         x = v * 1e-3; } asm volatile("" : "+v"(x)));
  // 7 uniform branch on a VALU compare of a readlane value
  TIME({ double p = rdl(x, 3); if (p > 1e300) { x = x + 1; } x = fma(x, y, 1e-12); } asm volatile("" : "+v"(x)));
  // 8 LDS load (independent address) -> use, dependent through address
  int idx = t;
  TIME(idx = ((int)lds[idx & 127] + idx + 1) & 127; asm volatile("" : "+v"(idx)));
  // 9 __shfl_xor (ds_bpermute) dependent
  TIME(x = __shfl_xor(x, 1, 64) * y; asm volatile("" : "+v"(x)));
  // 10 f64 division (IEEE sequence), dependent
  TIME(x = 1.0 / (x + 2.0); asm volatile("" : "+v"(x)));
  // 11 ds_write + ds_read with s_waitcnt, 8 reads of 8 addresses (broadcast), dependent
  TIME(lds[t] = x; __builtin_amdgcn_wave_barrier(); x = (lds[0] + lds[1] + lds[2] + lds[3] + lds[4] + lds[5] + lds[6] + lds[7]) * 1e-3; asm volatile("" : "+v"(x)));
  // 12 v_mfma_f64_16x16x4 dependent chain
  typedef double d4 __attribute__((ext_vector_type(4)));
  d4 acc = {x, y, x, y};
  TIME(acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc, 0, 0, 0); asm volatile("" : "+v"(acc)));
  x += acc[0] + acc[1] + acc[2] + acc[3];
  // 13 4 independent mfma chains
  d4 a0 = acc, a1 = acc, a2 = acc, a3 = acc;
  TIME(a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a0, 0, 0, 0); a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a1, 0, 0, 0);
       a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a2, 0, 0, 0); a3 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a3, 0, 0, 0);
       asm volatile("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3)));
  x += a0[0] + a1[1] + a2[2] + a3[3];
  // 14 v_readlane_b32 pair alone (to SGPR), dependent via scalar add
  int si = 0;
  TIME({ int q = __builtin_amdgcn_readlane((int)idx + si, r & 63); si = q & 7; } asm volatile("" : "+s"(si)));
  // 15 16 independent readlane pairs -> 16 independent fma (per rep)
  double rr[16];
  for (int i = 0; i < 16; i++) rr[i] = x + i;
  TIME({
#pragma unroll
    for (int i = 0; i < 16; i++) rr[i] = fma(rdl(rr[(i + 1) & 15], i), y, rr[i]);
  } asm volatile("" : "+v"(rr[0]), "+v"(rr[5]), "+v"(rr[9]), "+v"(rr[15])));
  for (int i = 0; i < 16; i++) x += rr[i];
  // 16 v_rcp_f64 + 2 NR dependent
  TIME({ double q = __builtin_amdgcn_rcp(x); q = fma(q, fma(-x, q, 1.0), q); q = fma(q, fma(-x, q, 1.0), q); x = q + 1.0; } asm volatile("" : "+v"(x)));
  // 17 16 independent fma (per rep)
  TIME({
#pragma unroll
    for (int i = 0; i < 16; i++) rr[i] = fma(rr[i], y, 1e-12);
  } asm volatile("" : "+v"(rr[0]), "+v"(rr[5]), "+v"(rr[9]), "+v"(rr[15])));
  for (int i = 0; i < 16; i++) x += rr[i];
  // 18 __syncthreads (single-wave workgroup) with one LDS write before
  TIME({ lds[t] = x; __syncthreads(); x = lds[t ^ 1] * y; } asm volatile("" : "+v"(x)));
  // 19 16 ds_read_b64 of independent lane-varying addresses then sum (per rep)
  TIME({ double acc2 = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) acc2 += lds[(t * 17 + i * 3 + (idx & 1)) & 1023];
    x = acc2 * 1e-3; } asm volatile("" : "+v"(x)));
  // 20 v_cndmask-heavy select chain 16 (per rep)
  TIME({
#pragma unroll
    for (int i = 0; i < 16; i++) rr[i] = (t == i) ? rr[i] * y : rr[i];
  } asm volatile("" : "+v"(rr[0]), "+v"(rr[5]), "+v"(rr[9]), "+v"(rr[15])));
  for (int i = 0; i < 16; i++) x += rr[i];
  sink[t] = x + idx + si;
}
int main() {
  unsigned long long *o; double *s;
  hipMalloc(&o, 64 * 8); hipMalloc(&s, 64 * 8);
  const char *names[] = {"empty loop", "dep f64 fma", "4 indep fma chains (per rep)", "LDS write->read rt", "readlane->fma",
                         "rsq+2NR", "DPP wave sum", "readlane+uniform branch+fma", "LDS load dep via addr", "shfl_xor f64",
                         "f64 div", "LDS write + 8 bcast reads", "mfma f64 dep", "4 indep mfma (per rep)", "readlane->salu",
                         "16 indep readlane+fma (per rep)", "rcp+2NR dep", "16 indep fma (per rep)", "LDS wr+syncthreads+rd", "16 ds_read_b64 lane-var (per rep)", "16 cndmask-mul (per rep)"};
  for (int pass = 0; pass < 2; pass++) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o, s, 1.5);
    hipDeviceSynchronize();
  }
  unsigned long long h[64]; hipMemcpy(h, o, 21 * 8, hipMemcpyDeviceToHost);
  for (int i = 0; i < 21; i++) printf("%-32s %8.1f cycles/rep\n", names[i], (double)h[i] / REP);
  return 0;
}
