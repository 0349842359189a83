// copy_sweep.hip -- measurement tool (not product): the read-one/write-one
// streaming ceiling that bounds every 1-in-1-out kernel (transform, stencils,
// scan).  Variants: vectors per thread per iteration U, nontemporal loads /
// stores, contiguous per-block ranges vs grid-stride chunks, grid size; plus
// hipMemcpyDtoD as the yardstick.  2^30 f32 in, 2^30 f32 out.
// Build: make -C tools copy_sweep.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

template <int U, bool CONTIG, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void cp(const f4 *__restrict__ x, f4 *__restrict__ y, size_t nv) {
  if (CONTIG) {
    const size_t per = (nv + gridDim.x - 1) / gridDim.x;
    const size_t lo = blockIdx.x * per, hi = lo + per < nv ? lo + per : nv;
    size_t i = lo + threadIdx.x;
    for (; i + (U - 1) * 256 < hi; i += U * 256) {
      f4 v[U];
#pragma unroll
      for (int u = 0; u < U; u++) v[u] = NTL ? __builtin_nontemporal_load(x + i + u * 256) : x[i + u * 256];
#pragma unroll
      for (int u = 0; u < U; u++) {
        f4 w = v[u] * 2.0f;
        if (NTS)
          __builtin_nontemporal_store(w, y + i + u * 256);
        else
          y[i + u * 256] = w;
      }
    }
    for (; i < hi; i += 256) y[i] = x[i] * 2.0f;
  } else {
    const size_t chunk = (size_t)U * 256;
    const size_t nfull = nv / chunk;
    for (size_t c = blockIdx.x; c < nfull; c += gridDim.x) {
      f4 v[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const f4 *p = x + c * chunk + u * 256 + threadIdx.x;
        v[u] = NTL ? __builtin_nontemporal_load(p) : *p;
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        f4 w = v[u] * 2.0f;
        f4 *q = y + c * chunk + u * 256 + threadIdx.x;
        if (NTS)
          __builtin_nontemporal_store(w, q);
        else
          *q = w;
      }
    }
  }
}

__global__ void fill(float *x, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    x[i] = (float)((i * 2654435761u) >> 8 & 0xFFFF) / 65536.0f;
}

static const size_t N = size_t(1) << 30;

template <typename F> void timeit(F f, hipStream_t st, const char *name, int U, int grid) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float tot = 0;
  const int reps = 10;
  for (int r = -2; r < reps; r++) {
    CK(hipEventRecord(e0, st));
    f();
    CK(hipEventRecord(e1, st));
    CK(hipStreamSynchronize(st));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 0) tot += ms;
  }
  const double ms = tot / reps;
  printf("%-26s U=%-2d grid %7d  %7.3f ms  %7.1f GB/s (r+w)\n", name, U, grid, ms, 8.0 * N / ms / 1e6);
}

template <int U, bool CONTIG, bool NTL, bool NTS>
void run(const float *x, float *y, int grid, hipStream_t st, const char *name) {
  timeit([&] { hipLaunchKernelGGL((cp<U, CONTIG, NTL, NTS>), dim3(grid), dim3(256), 0, st, (const f4 *)x, (f4 *)y, N / 4); },
         st, name, U, grid);
}

int main() {
  float *x, *y;
  CK(hipMalloc(&x, N * 4));
  CK(hipMalloc(&y, N * 4));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, st, x, N);
  CK(hipStreamSynchronize(st));
  timeit([&] { CK(hipMemcpyDtoDAsync(y, x, N * 4, st)); }, st, "hipMemcpyDtoD", 0, 0);
  for (int grid : {2048, 4096, 16384}) {
    run<1, false, false, false>(x, y, grid, st, "stride");
    run<4, false, false, false>(x, y, grid, st, "stride");
    run<4, false, true, true>(x, y, grid, st, "stride ntl nts");
    run<4, false, true, false>(x, y, grid, st, "stride ntl");
    run<4, false, false, true>(x, y, grid, st, "stride nts");
    run<4, true, false, false>(x, y, grid, st, "contig");
    run<4, true, true, true>(x, y, grid, st, "contig ntl nts");
    run<8, true, true, true>(x, y, grid, st, "contig ntl nts");
    run<8, true, true, false>(x, y, grid, st, "contig ntl");
    run<2, true, true, true>(x, y, grid, st, "contig ntl nts");
  }
  // one vector per thread, one-shot grid (no loop): the classic elementwise launch
  run<1, false, false, false>(x, y, (int)(N / 4 / 256), st, "oneshot");
  run<1, false, true, true>(x, y, (int)(N / 4 / 256), st, "oneshot ntl nts");
  run<1, false, true, false>(x, y, (int)(N / 4 / 256), st, "oneshot ntl");
  run<2, false, true, true>(x, y, (int)(N / 4 / 512), st, "oneshot ntl nts");
  run<4, false, true, true>(x, y, (int)(N / 4 / 1024), st, "oneshot ntl nts");
  run<8, false, true, true>(x, y, (int)(N / 4 / 2048), st, "oneshot ntl nts");
  run<4, false, true, true>(x, y, (int)(N / 4 / 2048), st, "half-shot ntl nts");
  run<1, false, true, true>(x, y, 131072, st, "stride ntl nts");
  run<1, false, true, true>(x, y, 65536, st, "stride ntl nts");
  return 0;
}
