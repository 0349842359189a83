// sort_stamps.hip -- measurement tool (not product): runs drhip_sort on 2^N
// uint32 keys with a libdrhip.so built with -DDRHIP_SORT_STAMPS
// (tools/sort_stamps.sh) and prints where one onesweep pass spends its time
// per tile: claim, key loads, ranking, digit offsets, publish + look-back +
// LDS reorder, barrier, write-out, and the look-back round trips.
#include <hip/hip_runtime.h>
#include <dlfcn.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../include/drhip.h"

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void gen(uint32_t *x, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t h = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
    h ^= h >> 31;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 29;
    x[i] = (uint32_t)h;
  }
}

static double pct(std::vector<double> v, double p) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, (size_t)(p * v.size()))];
}

int main(int argc, char **argv) {
  const int log2n = argc > 1 ? atoi(argv[1]) : 28;
  const size_t n = size_t(1) << log2n;
  typedef int (*stamps_fn)(void *, size_t);
  auto fn = (stamps_fn)dlsym(RTLD_DEFAULT, "drhip_dbg_sort_stamps");
  if (!fn) {
    fprintf(stderr, "libdrhip.so was not built with -DDRHIP_SORT_STAMPS\n");
    return 2;
  }
  int dev = 0;
  if (drhip_init(&dev, 1)) return 1;
  hipStream_t st;
  drhip_stream(0, (void **)&st);
  uint32_t *keys, *src;
  CK(hipMalloc(&keys, n * 4));
  CK(hipMalloc(&src, n * 4));
  hipLaunchKernelGGL(gen, dim3(4096), dim3(256), 0, st, src, n, 12345u);
  size_t wsb = 0;
  drhip_sort_workspace(0, DRHIP_U32, n, &wsb);
  void *ws;
  CK(hipMalloc(&ws, wsb));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float ms = 0;
  for (int r = 0; r < 3; r++) {
    CK(hipMemcpyAsync(keys, src, n * 4, hipMemcpyDeviceToDevice, st));
    CK(hipEventRecord(e0, st));
    if (drhip_sort(0, DRHIP_U32, keys, n, ws, wsb)) return 1;
    CK(hipEventRecord(e1, st));
    CK(hipStreamSynchronize(st));
    CK(hipEventElapsedTime(&ms, e0, e1));
  }
  const int slots = 10;
  const size_t tiles = n / 8192;
  std::vector<unsigned long long> s(tiles * slots);
  fn(s.data(), s.size() * 8);
  printf("sort 2^%d: %.3f ms (stamped build), %zu tiles in the stamped pass\n", log2n, ms, tiles);
  const char *names[] = {"claim", "load", "rank", "offsets", "lookback+reorder", "barrier"};
  std::vector<double> ph[6], tot, trips, waits, t0;
  unsigned long long rt_min = ~0ull, rt_max = 0;
  for (size_t t = 0; t < tiles; t++) {
    const unsigned long long *v = &s[t * slots];
    if (!v[0]) continue;
    for (int k = 0; k < 6; k++) ph[k].push_back((double)(v[k + 2] - v[k + 1]));
    tot.push_back((v[8] - v[0]) * 10.0); // 100 MHz real-time clock -> ns
    trips.push_back((double)(v[9] & 0xFFFFFFFFull));
    waits.push_back((double)((v[9] >> 32) & 0x7FFFFFFFull));
    t0.push_back((double)v[0]);
    rt_min = std::min(rt_min, v[0]);
    rt_max = std::max(rt_max, v[8]);
  }
  printf("pass span %.1f us over %zu stamped tiles\n", (rt_max - rt_min) * 0.01, tot.size());
  printf("%-18s %10s %10s %10s %10s  (shader cycles)\n", "phase", "p10", "p50", "p90", "mean");
  for (int k = 0; k < 6; k++) {
    double m = 0;
    for (double x : ph[k]) m += x;
    m /= std::max<size_t>(1, ph[k].size());
    printf("%-18s %10.0f %10.0f %10.0f %10.0f\n", names[k], pct(ph[k], .1), pct(ph[k], .5), pct(ph[k], .9), m);
  }
  double m = 0, mt = 0;
  for (double x : tot) m += x;
  for (double x : trips) mt += x;
  printf("%-18s %10.0f %10.0f %10.0f %10.0f  (ns, block start -> end)\n", "tile total", pct(tot, .1), pct(tot, .5),
         pct(tot, .9), m / std::max<size_t>(1, tot.size()));
  printf("%-18s %10.0f %10.0f %10.0f %10.2f  (digit 0's look-back round trips)\n", "trips", pct(trips, .1),
         pct(trips, .5), pct(trips, .9), mt / std::max<size_t>(1, trips.size()));
  double mw = 0;
  for (double x : waits) mw += x;
  printf("%-18s %10.0f %10.0f %10.0f %10.2f  (of them: an unpublished predecessor, polled again)\n", "waits",
         pct(waits, .1), pct(waits, .5), pct(waits, .9), mw / std::max<size_t>(1, waits.size()));
  drhip_finalize();
  return 0;
}
