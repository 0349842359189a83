// scan_sweep.hip -- measurement tool (not product): times scan_kernel
// variants (vectors per thread U, fp32 final combine, nontemporal stores,
// look-back removed) against a copy kernel of the same tile shape on a
// 2^30-element f32 vector.  Build: make -C tools scan_sweep.
#include "../distributed-ranges_amd/csrc/scan_kernel.hpp"

#include <cstring>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_reduce.hpp>

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace drhip;

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

template <int U>
__global__ __launch_bounds__(256) void copy_tile(const float4 *in, float4 *out, size_t nvec) {
  const size_t base = (size_t)blockIdx.x * 256 * U;
  float4 r[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    size_t i = base + u * 256 + threadIdx.x;
    if (i < nvec) r[u] = in[i];
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    size_t i = base + u * 256 + threadIdx.x;
    if (i < nvec) out[i] = r[u];
  }
}

__global__ void fill_rand(float *x, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    x[i] = (h >> 8) * (1.0f / 16777216.0f);
  }
}

static float elapsed(hipEvent_t a, hipEvent_t b) {
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

struct Ctx {
  float *in, *out;
  size_t n;
  char *ws;
  unsigned *err;
  hipStream_t st;
};

template <int U, int FLAGS, int MINW = 1> static double run_scan(Ctx &c, int reps, double *last) {
  constexpr size_t TILE = 256 * U * 4;
  const size_t ntiles = (c.n + TILE - 1) / TILE;
  const size_t gran_b = (ntiles * 16 + 255) & ~size_t(255);
  Granules<double> gr;
  gr.base = c.ws + 256;
  gr.bytes = (int)gran_b;
  ScanArgs<double> a{};
  a.err = c.err;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f, sum = 0;
  for (int r = -2; r < reps; r++) {
    CK(hipMemsetAsync(c.ws, 0, 256 + gran_b, c.st));
    CK(hipEventRecord(e0, c.st));
    hipLaunchKernelGGL((scan_kernel<DRHIP_PLUS, float, true, U, FLAGS, MINW>), dim3((unsigned)ntiles), dim3(256), 0,
                       c.st, c.in, c.out, c.n, (unsigned *)c.ws, gr, 0, 0.0f, a);
    CK(hipEventRecord(e1, c.st));
    CK(hipStreamSynchronize(c.st));
    if (r >= 0) {
      float ms = elapsed(e0, e1);
      sum += ms;
      best = ms < best ? ms : best;
    }
  }
  float l;
  CK(hipMemcpy(&l, c.out + c.n - 1, 4, hipMemcpyDeviceToHost));
  *last = l;
  return sum / reps;
}

template <int U, int FLAGS, int MINW = 1> static void run_diag(Ctx &c) {
  constexpr size_t TILE = 256 * U * 4;
  const size_t ntiles = (c.n + TILE - 1) / TILE;
  const size_t gran_b = (ntiles * 16 + 255) & ~size_t(255);
  Granules<double> gr;
  gr.base = c.ws + 256;
  gr.bytes = (int)gran_b;
  ScanArgs<double> a{};
  a.err = c.err;
  CK(hipMalloc(&a.diag, ntiles * 64));
  for (int r = 0; r < 3; r++) {
    CK(hipMemsetAsync(c.ws, 0, 256 + gran_b, c.st));
    CK(hipMemsetAsync(a.diag, 0, ntiles * 64, c.st));
    hipLaunchKernelGGL((scan_kernel<DRHIP_PLUS, float, true, U, FLAGS | SCAN_DIAG, MINW>), dim3((unsigned)ntiles), dim3(256),
                       0, c.st, c.in, c.out, c.n, (unsigned *)c.ws, gr, 0, 0.0f, a);
    CK(hipStreamSynchronize(c.st));
  }
  std::vector<unsigned long long> d(ntiles * 8);
  CK(hipMemcpy(d.data(), a.diag, ntiles * 64, hipMemcpyDeviceToHost));
  unsigned long long t0 = ~0ull, tend = 0;
  double s_load = 0, s_lb = 0, s_store = 0, s_steps = 0, s_spins = 0;
  unsigned max_steps = 0;
  size_t hist[8] = {0};
  for (size_t t = 1; t < ntiles; t++) {
    unsigned long long *x = &d[t * 8];
    t0 = x[0] < t0 ? x[0] : t0;
    tend = x[3] > tend ? x[3] : tend;
    s_load += x[1] - x[0];
    s_lb += x[2] - x[1];
    s_store += x[3] - x[2];
    s_steps += x[4];
    s_spins += x[5];
    max_steps = x[4] > max_steps ? x[4] : max_steps;
    hist[x[4] < 7 ? x[4] : 7]++;
  }
  // resident tiles over time ~ sum(durations) / wall
  const double wall = (double)(tend - t0);
  double sum_dur = 0;
  for (size_t t = 1; t < ntiles; t++) sum_dur += d[t * 8 + 3] - d[t * 8];
  const double m = (double)(ntiles - 1);
  printf("diag U=%d flags=%d: per tile (10 ns ticks) load+agg %.1f  lookback %.1f  combine+store %.1f ;"
         " steps avg %.2f max %u spins avg %.2f ; wall %.3f ms, avg resident tiles %.0f\n",
         U, FLAGS, s_load / m, s_lb / m, s_store / m, s_steps / m, max_steps, s_spins / m, wall * 1e-5,
         sum_dur / wall);
  printf("  steps histogram:");
  for (int i = 0; i < 8; i++) printf(" %d:%zu", i, hist[i]);
  printf("\n");
  CK(hipFree(a.diag));
}

template <int U> static double run_copy(Ctx &c, int reps) {
  const size_t nvec = c.n / 4;
  const size_t blocks = (nvec + 256 * U - 1) / (256 * U);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float sum = 0;
  for (int r = -2; r < reps; r++) {
    CK(hipEventRecord(e0, c.st));
    hipLaunchKernelGGL((copy_tile<U>), dim3((unsigned)blocks), dim3(256), 0, c.st, (const float4 *)c.in,
                       (float4 *)c.out, nvec);
    CK(hipEventRecord(e1, c.st));
    CK(hipStreamSynchronize(c.st));
    if (r >= 0) sum += elapsed(e0, e1);
  }
  return sum / reps;
}

#define SCANW(U, F, W, name)                                                                       \
  do {                                                                                             \
    double last;                                                                                   \
    double ms = run_scan<U, F, W>(c, reps, &last);                                                 \
    printf("scan U=%-2d minw=%d %-16s %8.3f ms", U, W, name, ms);                                  \
    printf(" %7.1f GB/s  last=%.6e rel=%.2e\n", bytes / ms / 1e6, last, (last - ref) / ref);       \
  } while (0)
#define SCAN(U, F, name)                                                                           \
  do {                                                                                             \
    double last;                                                                                   \
    double ms = run_scan<U, F>(c, reps, &last);                                                    \
    printf("scan U=%-2d %-22s %8.3f ms %7.1f GB/s  last=%.6e rel=%.2e\n", U, name, ms,            \
           bytes / ms / 1e6, last, (last - ref) / ref);                                             \
  } while (0)

int main(int argc, char **argv) {
  int log2n = argc > 1 ? atoi(argv[1]) : 30;
  int reps = argc > 2 ? atoi(argv[2]) : 10;
  Ctx c;
  c.n = size_t(1) << log2n;
  CK(hipStreamCreateWithFlags(&c.st, hipStreamNonBlocking));
  CK(hipMalloc(&c.in, c.n * 4));
  CK(hipMalloc(&c.out, c.n * 4));
  CK(hipMalloc(&c.ws, 64 << 20));
  CK(hipHostMalloc(&c.err, 256, hipHostMallocMapped));
  *c.err = 0;
  hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, c.st, c.in, c.n);
  CK(hipStreamSynchronize(c.st));
  std::vector<float> h(c.n);
  CK(hipMemcpy(h.data(), c.in, c.n * 4, hipMemcpyDeviceToHost));
  double ref = 0;
  for (size_t i = 0; i < c.n; i++) ref += h[i];
  const double bytes = 8.0 * c.n;
  printf("n = 2^%d f32, %d reps, fp64 total %.9e\n", log2n, reps, ref);
  printf("copy U=4  %8.3f ms %7.1f GB/s\n", run_copy<4>(c, reps), bytes / run_copy<4>(c, reps) / 1e6);
  printf("copy U=8  %8.3f ms %7.1f GB/s\n", run_copy<8>(c, reps), bytes / run_copy<8>(c, reps) / 1e6);
  printf("copy U=16 %8.3f ms %7.1f GB/s\n", run_copy<16>(c, reps), bytes / run_copy<16>(c, reps) / 1e6);
  SCANW(16, SCAN_NT_STORE, 1, "nt-store (product)");
  SCANW(16, SCAN_NT_STORE | SCAN_NT_LOAD, 1, "nt-load+store");
  SCANW(16, SCAN_NT_LOAD, 1, "nt-load");
  SCANW(12, SCAN_NT_STORE | SCAN_NT_LOAD, 1, "nt-load+store");
  SCANW(16, SCAN_NT_STORE | SCAN_NT_LOAD | SCAN_NO_LOOKBACK, 1, "nt nolb(timing)");
  {
    size_t tb = 0;
    CK(rocprim::inclusive_scan(nullptr, tb, c.in, c.out, c.n, rocprim::plus<float>(), c.st));
    void *tmp;
    CK(hipMalloc(&tmp, tb));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float tot = 0;
    for (int r = -2; r < reps; r++) {
      CK(hipEventRecord(e0, c.st));
      CK(rocprim::inclusive_scan(tmp, tb, c.in, c.out, c.n, rocprim::plus<float>(), c.st));
      CK(hipEventRecord(e1, c.st));
      CK(hipStreamSynchronize(c.st));
      if (r >= 0) tot += elapsed(e0, e1);
    }
    printf("rocprim inclusive_scan (yardstick) %8.3f ms %7.1f GB/s\n", tot / reps, bytes / (tot / reps) / 1e6);
    float *res;
    CK(hipMalloc(&res, 4));
    tb = 0;
    CK(rocprim::reduce(nullptr, tb, c.in, res, 0.0f, c.n, rocprim::plus<float>(), c.st));
    void *tmp2;
    CK(hipMalloc(&tmp2, tb));
    tot = 0;
    for (int r = -2; r < reps; r++) {
      CK(hipEventRecord(e0, c.st));
      CK(rocprim::reduce(tmp2, tb, c.in, res, 0.0f, c.n, rocprim::plus<float>(), c.st));
      CK(hipEventRecord(e1, c.st));
      CK(hipStreamSynchronize(c.st));
      if (r >= 0) tot += elapsed(e0, e1);
    }
    printf("rocprim reduce (yardstick)         %8.3f ms %7.1f GB/s\n", tot / reps, bytes / 2 / (tot / reps) / 1e6);
  }
  printf("err word %u\n", *c.err);
  return 0;
}
