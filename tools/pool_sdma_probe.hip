// Round-5 probe: does memory from the stream-ordered pool keep what a copy
// engine writes into it?  Mirrors the allocation / fill / copy pattern of
// tests/cpp/shp_tests.cpp noncommutative_case (three vectors per case,
// n = 1 ... 2000003 elements of 8 / 12 / 16 bytes, zero-filled by a kernel,
// the input copied in from pinned memory and read back) without libdrhip.
//   pool_sdma_probe <pool|hipmalloc> [rounds]
// Prints the number of cases whose read-back differs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                             \
      std::exit(2);                                                                            \
    }                                                                                          \
  } while (0)

__global__ void fill_zero(unsigned *p, size_t nw) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nw; i += (size_t)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(0u, p + i);
}

static bool g_pool = true;
static hipStream_t g_st;
static void *alloc(size_t b) {
  void *p = nullptr;
  if (g_pool) {
    CK(hipMallocAsync(&p, b, g_st));
    CK(hipStreamSynchronize(g_st));
  } else {
    CK(hipMalloc(&p, b));
  }
  unsigned nw = 0;
  (void)nw;
  fill_zero<<<2048, 256, 0, g_st>>>((unsigned *)p, b / 4);
  CK(hipGetLastError());
  CK(hipStreamSynchronize(g_st));
  return p;
}
static void release(void *p) {
  if (g_pool) CK(hipFreeAsync(p, g_st));
  else {
    CK(hipStreamSynchronize(g_st));
    CK(hipFree(p));
  }
}

int main(int argc, char **argv) {
  g_pool = argc < 2 || std::strcmp(argv[1], "hipmalloc") != 0;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 20;
  CK(hipStreamCreateWithFlags(&g_st, hipStreamNonBlocking));
  hipMemPool_t pool;
  CK(hipDeviceGetDefaultMemPool(&pool, 0));
  uint64_t keep = UINT64_MAX;
  CK(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep));
  const size_t maxb = 2000003ull * 16 * 2;
  unsigned char *src = nullptr, *back = nullptr;
  CK(hipHostMalloc((void **)&src, maxb, hipHostMallocPortable));
  CK(hipHostMalloc((void **)&back, maxb, hipHostMallocPortable));
  int bad = 0, cases = 0;
  unsigned seed = 1;
  for (int r = 0; r < rounds; r++)
    for (size_t n : {size_t(1), size_t(1000), size_t(300007), size_t(2000003)})
      for (size_t es : {size_t(8), size_t(12), size_t(16)}) {
        const size_t b = n * es;
        void *v = alloc(b), *o = alloc(b), *o2 = alloc(2 * b);
        for (size_t i = 0; i < b; i++) src[i] = (unsigned char)((seed = seed * 1103515245u + 12345u) >> 16);
        CK(hipMemcpyAsync(v, src, b, hipMemcpyHostToDevice, g_st));
        CK(hipStreamSynchronize(g_st));
        CK(hipMemcpyAsync(back, v, b, hipMemcpyDeviceToHost, g_st));
        CK(hipStreamSynchronize(g_st));
        cases++;
        if (std::memcmp(src, back, b) != 0) {
          size_t f = 0;
          while (f < b && src[f] == back[f]) f++;
          if (bad < 5)
            std::printf("round %d n %zu elem %zu: read-back differs from byte %zu (address %p)\n", r, n, es, f,
                        (void *)((char *)v + f));
          bad++;
        }
        // the scans' outputs: o and o2 written by the device
        CK(hipMemcpyAsync(o, v, b, hipMemcpyDeviceToDevice, g_st));
        CK(hipMemcpyAsync(o2, v, b, hipMemcpyDeviceToDevice, g_st));
        CK(hipStreamSynchronize(g_st));
        release(v);
        release(o);
        release(o2);
        CK(hipStreamSynchronize(g_st));
      }
  std::printf("{\"alloc\": \"%s\", \"cases\": %d, \"bad\": %d}\n", g_pool ? "pool" : "hipmalloc", cases, bad);
  return 0;
}
