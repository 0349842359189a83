// xcd_local_copy.hip -- measurement tool (not product): can an XCD-local
// working set be streamed faster than HBM?  The question behind an MSD-first
// sort whose ~1 M-key buckets (4 MiB) would be finished by ONE XCD in
// ping-pong passes between two buffers.
//
// A persistent grid (2 blocks per CU, every block resident) learns each
// block's XCD (HW_REG_XCC_ID); XCD x owns buffers A_x, B_x of S bytes and its
// blocks copy A_x -> B_x -> A_x ... ITER times, with an XCD-local barrier
// (one counter per XCD, all blocks resident) between copies.  Reported:
// aggregate bytes moved (read + write) / time, for S from 1 to 64 MiB per
// buffer, next to the same copies on buffers of 1 GiB (HBM-bound).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));          \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

typedef unsigned u4 __attribute__((ext_vector_type(4)));

// ctl: [0..7] per-XCD registration counters, [8] grid registration,
// [16..23] per-XCD barrier counters
__global__ __launch_bounds__(256) void xcd_copy(u4 *buf, size_t words_per_buf, int iters, unsigned *ctl,
                                                unsigned *err) {
  __shared__ unsigned s_xcd, s_rank, s_cnt;
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  xcc &= 7;
  if (threadIdx.x == 0) {
    s_xcd = xcc;
    s_rank = atomicAdd(ctl + xcc, 1u);
    atomicAdd(ctl + 8, 1u);
    // grid-wide registration: every block of the (resident) grid
    unsigned spins = 0;
    while (__hip_atomic_load(ctl + 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gridDim.x) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1u << 24)) {
        atomicExch(err, 1u);
        break;
      }
    }
    s_cnt = __hip_atomic_load(ctl + xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const unsigned x = s_xcd, rank = s_rank, cnt = s_cnt;
  u4 *a = buf + (size_t)x * 2 * words_per_buf, *b = a + words_per_buf;
  for (int it = 0; it < iters; it++) {
    const u4 *src = (it & 1) ? b : a;
    u4 *dst = (it & 1) ? a : b;
    for (size_t i = (size_t)rank * 256 + threadIdx.x; i < words_per_buf; i += (size_t)cnt * 256) dst[i] = src[i];
    // XCD-local barrier: cnt blocks arrive, iteration it+1 waits for all
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      // same-XCD hand-off: the stores have reached this XCD's L2 (no L2
      // write-back: the readers share the L2), then the arrival
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      atomicAdd(ctl + 16 + x, 1u);
      const unsigned target = cnt * (unsigned)(it + 1);
      unsigned spins = 0;
      while (__hip_atomic_load(ctl + 16 + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 24)) {
          atomicExch(err, 2u);
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent"); // this CU's L1 invalidated, L2 kept
    }
    __syncthreads();
  }
}

int main() {
  int dev = 0, cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const unsigned grid = (unsigned)cus * 2;
  const size_t max_bytes = size_t(1) << 30; // per buffer, 8 XCDs x 2 buffers = 16 GiB
  u4 *buf;
  unsigned *ctl, *err;
  CK(hipMalloc(&buf, max_bytes * 16));
  CK(hipMemset(buf, 1, max_bytes * 16));
  CK(hipMalloc(&ctl, 256));
  CK(hipMalloc(&err, 4));
  CK(hipMemset(err, 0, 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (size_t mib : {1, 2, 4, 8, 16, 32, 64, 1024}) {
    const size_t bytes = mib << 20;
    const int iters = mib >= 1024 ? 2 : 32;
    float best = 1e30f;
    for (int r = 0; r < 4; r++) {
      CK(hipMemset(ctl, 0, 256));
      CK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(xcd_copy, dim3(grid), dim3(256), 0, 0, buf, bytes / 16, iters, ctl, err);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r) best = ms < best ? ms : best;
    }
    unsigned herr = 0;
    CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
    const double moved = 8.0 * 2.0 * (double)bytes * iters; // 8 XCDs, read + write
    printf("{\"MiB_per_buffer\": %zu, \"iters\": %d, \"ms\": %.4f, \"TBps_read_plus_write\": %.2f, \"err\": %u}\n", mib,
           iters, best, moved / (best * 1e-3) / 1e12, herr);
    fflush(stdout);
  }
  CK(hipFree(buf));
  return 0;
}
