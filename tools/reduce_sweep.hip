// reduce_sweep.hip -- measurement tool (not product): f32 sum-reduction
// stage-1 variants on 2^30 elements (loads per thread per iteration U,
// interleaved grid-stride vs contiguous block ranges, nontemporal loads,
// grid size) to pick the drhip_reduce design.  Build: make -C tools.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double block_sum(double v) {
  __shared__ double sm[4];
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = v;
  __syncthreads();
  return sm[0] + sm[1] + sm[2] + sm[3];
}

// INTERLEAVED: chunk c of U*256 vectors, blocks stride by gridDim
// CONTIG: block b owns vectors [b*per, (b+1)*per)
template <int U, bool CONTIG, bool NT>
__global__ __launch_bounds__(256) void red(const f4 *x, size_t nv, double *part) {
  double acc = 0;
  if (CONTIG) {
    const size_t per = (nv + gridDim.x - 1) / gridDim.x;
    const size_t lo = blockIdx.x * per, hi = lo + per < nv ? lo + per : nv;
    size_t i = lo + threadIdx.x;
    for (; i + (U - 1) * 256 < hi; i += U * 256) {
      f4 v[U];
#pragma unroll
      for (int u = 0; u < U; u++) v[u] = NT ? __builtin_nontemporal_load(x + i + u * 256) : x[i + u * 256];
      float s = 0;
#pragma unroll
      for (int u = 0; u < U; u++) s += (v[u].x + v[u].y) + (v[u].z + v[u].w);
      acc += s;
    }
    for (; i < hi; i += 256) {
      f4 v = x[i];
      acc += (v.x + v.y) + (v.z + v.w);
    }
  } else {
    const size_t chunk = (size_t)U * 256;
    size_t c = blockIdx.x;
    const size_t nfull = nv / chunk;
    for (; c < nfull; c += gridDim.x) {
      f4 v[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const f4 *p = x + c * chunk + u * 256 + threadIdx.x;
        v[u] = NT ? __builtin_nontemporal_load(p) : *p;
      }
      float s = 0;
#pragma unroll
      for (int u = 0; u < U; u++) s += (v[u].x + v[u].y) + (v[u].z + v[u].w);
      acc += s;
    }
  }
  double t = block_sum(acc);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

__global__ void fill(float *x, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    x[i] = (float)((i * 2654435761u) >> 8 & 0xFFFF) / 65536.0f;
}

template <int U, bool CONTIG, bool NT> void run(const float *x, size_t n, double *part, int grid, hipStream_t st,
                                                const char *name) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float tot = 0;
  const int reps = 10;
  for (int r = -2; r < reps; r++) {
    CK(hipEventRecord(e0, st));
    hipLaunchKernelGGL((red<U, CONTIG, NT>), dim3(grid), dim3(256), 0, st, (const f4 *)x, n / 4, part);
    CK(hipEventRecord(e1, st));
    CK(hipStreamSynchronize(st));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 0) tot += ms;
  }
  const double ms = tot / reps;
  printf("%-28s U=%-2d grid %5d  %7.3f ms  %7.1f GB/s\n", name, U, grid, ms, 4.0 * n / ms / 1e6);
}

int main() {
  const size_t n = size_t(1) << 30;
  float *x;
  double *part;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&part, 65536 * 8));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, st, x, n);
  CK(hipStreamSynchronize(st));
  for (int grid : {1024, 2048, 4096}) {
    run<4, false, false>(x, n, part, grid, st, "interleaved");
    run<8, false, false>(x, n, part, grid, st, "interleaved");
    run<8, false, true>(x, n, part, grid, st, "interleaved nt");
    run<4, true, false>(x, n, part, grid, st, "contiguous");
    run<8, true, false>(x, n, part, grid, st, "contiguous");
    run<16, true, false>(x, n, part, grid, st, "contiguous");
    run<8, true, true>(x, n, part, grid, st, "contiguous nt");
  }
  return 0;
}
