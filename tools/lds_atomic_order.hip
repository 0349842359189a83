// lds_atomic_order.hip -- measurement tool (not product): do the lanes of ONE
// ds_add_rtn_u32 wave-instruction that hit the same LDS address get their
// old values in ascending lane order?  (If so, an LDS atomic counter gives a
// stable within-wave rank for radix sorting.)  Counts violations over many
// random digit patterns and distributions.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void probe(const unsigned *digits, int slots, unsigned *viol, unsigned *checked) {
  __shared__ unsigned cnt[4][257];
  __shared__ unsigned got[4][64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = tid; i < 4 * 257; i += blockDim.x) (&cnt[0][0])[i] = 0;
  __syncthreads();
  unsigned bad = 0, chk = 0;
  for (int r = 0; r < slots; r++) {
    const unsigned d = digits[((size_t)blockIdx.x * slots + r) * 256 + tid];
    const unsigned old = atomicAdd(&cnt[w][d], 1u);
    got[w][lane] = old;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    // lane compares itself with every lower lane holding the same digit
    for (int j = 0; j < lane; j++) {
      const unsigned dj = digits[((size_t)blockIdx.x * slots + r) * 256 + w * 64 + j];
      if (dj == d) {
        chk++;
        if (!(got[w][j] < old)) bad++;
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  atomicAdd(viol, bad);
  atomicAdd(checked, chk);
}

int main() {
  const int blocks = 2048, slots = 32;
  const size_t n = (size_t)blocks * slots * 256;
  std::vector<unsigned> h(n);
  unsigned *dd, *dv, *dc;
  hipMalloc(&dd, n * 4);
  hipMalloc(&dv, 4);
  hipMalloc(&dc, 4);
  const int ranges[] = {256, 16, 4, 2, 1};
  for (int range : ranges) {
    srand(range);
    for (auto &x : h) x = (unsigned)(rand() % range);
    hipMemcpy(dd, h.data(), n * 4, hipMemcpyHostToDevice);
    hipMemset(dv, 0, 4);
    hipMemset(dc, 0, 4);
    hipLaunchKernelGGL(probe, dim3(blocks), dim3(256), 0, 0, dd, slots, dv, dc);
    unsigned v = 0, c = 0;
    hipMemcpy(&v, dv, 4, hipMemcpyDeviceToHost);
    hipMemcpy(&c, dc, 4, hipMemcpyDeviceToHost);
    printf("digits in [0,%3d): %u same-address lane pairs checked, %u out of lane order\n", range, c, v);
  }
  return 0;
}
