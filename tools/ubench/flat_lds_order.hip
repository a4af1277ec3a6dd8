// Diagnostic (not product code): are FLAT (generic-address) accesses that land in LDS
// ordered with the DS instructions of the same wavefront when nothing waits in between?  The NW = 1 SYNC()
// of the solve kernel is a wavefront fence that emits no s_waitcnt: it relies on a wave's LDS operations
// being performed in issue order.  Each pattern issues the two accesses back to back in inline assembly
// (one s_waitcnt after both), over many iterations, waves and workgroups, and counts the lanes that saw the
// other order:
//   0  flat_store X       -> ds_read X          (read-after-write: stale value?)
//   1  ds_write X         -> flat_load X        (read-after-write)
//   2  flat_load X        -> ds_write X         (write-after-read: the load returns the NEW value?)
//   3  flat_store X       -> ds_write X         (write-after-write: the flat store lands last?)
//   4  ds_write X         -> ds_read X          (control: DS only)
//   5  flat_store X       -> ds_read Y          (Y: the next lane's word, written by that lane's flat store)
//   6  ds_write X         -> flat_load Y        (Y: the next lane's word)
// Patterns 7..10 repeat 0, 1, 5 and 6 with a VMEM global load issued first (a flat access then queues
// behind it in the vector-memory path while the DS instruction does not).
//   11  flat_load X, s_waitcnt vmcnt(0) lgkmcnt(0), ds_write X   (does the wait cover the flat LDS read?)
//   12  flat_load r <- X, s_waitcnt vmcnt(0) lgkmcnt(0), r overwritten by a VALU move, read back
//       after 64 s_nop: does the load's data land in r after the wait?
//   13  the same as 11 with a global_load of global memory (control)
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench/flat_lds_order tools/ubench/flat_lds_order.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define LDSA(p) ((uint32_t)(uintptr_t)(__attribute__((address_space(3))) void *)(p))

__global__ void __launch_bounds__(256) order_test(int mode, int iters, const double *__restrict__ gsrc, unsigned long long *count)
{
    __shared__ double buf[256 * 4];
    const int tid = threadIdx.x, lane = tid & 63, wbase = tid - lane;
    double *mine = buf + 4 * tid;
    double *next = buf + 4 * (wbase + ((lane + 1) & 63));
    const uint64_t gmine = (uint64_t)(uintptr_t)mine, gnext = (uint64_t)(uintptr_t)next;
    const uint32_t lmine = LDSA(mine), lnext = LDSA(next);
    const bool pre = mode >= 7 && mode <= 10;
    const int m = pre ? (mode == 7 ? 0 : mode == 8 ? 1 : mode == 9 ? 5 : 6) : mode;
    unsigned long long bad = 0;
    mine[0] = (double)tid;                  // = vold of iteration 1
    __syncthreads();
    for (int it = 1; it <= iters; it++) {
        const double v = (double)it * 256.0 + tid, vold = (double)(it - 1) * 256.0 + tid;
        const double vnext = (double)it * 256.0 + (wbase + ((lane + 1) & 63));
        double r = 0.0, g = 0.0;
        if (pre) asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(g) : "v"(gsrc + (it & 1023)) : "memory");
        switch (m) {
        case 0:
            asm volatile("flat_store_dwordx2 %1, %2\n\tds_read_b64 %0, %3\n\ts_waitcnt vmcnt(0) lgkmcnt(0)"
                         : "=v"(r) : "v"(gmine), "v"(v), "v"(lmine) : "memory");
            bad += r != v;
            break;
        case 1:
            asm volatile("ds_write_b64 %3, %2\n\tflat_load_dwordx2 %0, %1\n\ts_waitcnt vmcnt(0) lgkmcnt(0)"
                         : "=v"(r) : "v"(gmine), "v"(v), "v"(lmine) : "memory");
            bad += r != v;
            break;
        case 2:
            asm volatile("flat_load_dwordx2 %0, %1\n\tds_write_b64 %3, %2\n\ts_waitcnt vmcnt(0) lgkmcnt(0)"
                         : "=v"(r) : "v"(gmine), "v"(v), "v"(lmine) : "memory");
            bad += r != vold;
            break;
        case 3:
            asm volatile("flat_store_dwordx2 %0, %1\n\tds_write_b64 %2, %3\n\ts_waitcnt vmcnt(0) lgkmcnt(0)"
                         :: "v"(gmine), "v"(-v), "v"(lmine), "v"(v) : "memory");
            asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(lmine) : "memory");
            bad += r != v;
            break;
        case 4:
            asm volatile("ds_write_b64 %1, %2\n\tds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                         : "=v"(r) : "v"(lmine), "v"(v) : "memory");
            bad += r != v;
            break;
        case 5:
            asm volatile("flat_store_dwordx2 %1, %2\n\tds_read_b64 %0, %3\n\ts_waitcnt vmcnt(0) lgkmcnt(0)"
                         : "=v"(r) : "v"(gmine), "v"(v), "v"(lnext) : "memory");
            bad += r != vnext;
            break;
        case 6:
            asm volatile("ds_write_b64 %2, %1\n\tflat_load_dwordx2 %0, %3\n\ts_waitcnt vmcnt(0) lgkmcnt(0)"
                         : "=v"(r) : "v"(v), "v"(lmine), "v"(gnext) : "memory");
            bad += r != vnext;
            break;
        case 11:
            asm volatile("flat_load_dwordx2 %0, %1\n\ts_waitcnt vmcnt(0) lgkmcnt(0)\n\tds_write_b64 %3, %2\n\ts_waitcnt lgkmcnt(0)"
                         : "=&v"(r) : "v"(gmine), "v"(v), "v"(lmine) : "memory");
            bad += r != vold;
            break;
        case 12: {
            const double sentinel = -1.0 - it;
            asm volatile("flat_load_dwordx2 %0, %1\n\ts_waitcnt vmcnt(0) lgkmcnt(0)\n\t"
                         "v_mov_b64 %0, %2\n\t"
                         "s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7"
                         : "=&v"(r) : "v"(gmine), "v"(sentinel) : "memory");
            bad += r != sentinel;
            asm volatile("ds_write_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" :: "v"(lmine), "v"(v) : "memory");
            break;
        }
        default: {            // 13: global memory control for 11
            double *gw = (double *)gsrc + 1024 + blockIdx.x * 256 + tid;
            asm volatile("global_load_dwordx2 %0, %1, off\n\ts_waitcnt vmcnt(0)\n\tglobal_store_dwordx2 %1, %2, off\n\ts_waitcnt vmcnt(0)"
                         : "=&v"(r) : "v"(gw), "v"(v) : "memory");
            bad += (it > 1) && r != vold;
            break;
        }
        }
        if (pre) asm volatile("s_waitcnt vmcnt(0)" :: "v"(g) : "memory");
        __syncthreads();            // every lane's word holds this iteration's value before the next one
    }
    if (bad) atomicAdd(count + mode, bad);
}

int main()
{
    const int modes = 14, iters = 4096, blocks = 1024;
    const char *name[modes] = {"flat_store -> ds_read (same word)", "ds_write -> flat_load (same word)",
                               "flat_load -> ds_write (WAR)", "flat_store -> ds_write (WAW)", "ds_write -> ds_read (control)",
                               "flat_store -> ds_read (next lane's word)", "ds_write -> flat_load (next lane's word)",
                               "global load, flat_store -> ds_read", "global load, ds_write -> flat_load",
                               "global load, flat_store -> ds_read (next lane)", "global load, ds_write -> flat_load (next lane)",
                               "flat_load, waitcnt(0), ds_write (WAR)", "flat_load, waitcnt(0), register overwritten",
                               "global_load, waitcnt, global_store (control)"};
    unsigned long long *d, h[modes];
    double *g;
    hipMalloc(&d, sizeof h);
    const size_t gn = 1024 + (size_t)blocks * 256;
    hipMalloc(&g, gn * sizeof(double));
    hipMemset(g, 0, gn * sizeof(double));
    hipMemset(d, 0, sizeof h);
    for (int mo = 0; mo < modes; mo++) order_test<<<blocks, 256>>>(mo, iters, g, d);
    if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    const double total = (double)iters * blocks * 256;
    for (int mo = 0; mo < modes; mo++)
        printf("%-48s other order seen %12llu of %.0f lane-iterations (%.3g)\n", name[mo], h[mo], total, h[mo] / total);
    hipFree(d);
    hipFree(g);
    return 0;
}
