// pmc_calib.hip -- measurement tool (not product): kernels with KNOWN HBM byte
// counts, to calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE per access pattern
// on gfx950 (MI355X_MICROARCH.md: FETCH_SIZE reads 1/2 of a 16-B/lane
// streaming read; other widths uncalibrated).  Run each counter in its own
// pass:  rocprofv3 --pmc FETCH_SIZE -- ./pmc_calib ;  --pmc WRITE_SIZE -- ...
//
// Kernels (table = 4 GiB of fp32, far past the 256 MiB Infinity Cache):
//   cal_read16     every lane one 16-B load, 2 GiB streamed        (2 GiB)
//   cal_read4      every lane one 4-B load, 2 GiB streamed         (2 GiB)
//   cal_gather128  2^25 4-B loads, each on its own 128-B line, in a
//                  scattered (odd-multiplier permutation) order    (2^25 lines)
//   cal_gather64   2^26 4-B loads, each on its own 64-B half line  (2^26 halves)
//   cal_scatter128 2^25 4-B stores, each on its own 128-B line     (2^25 lines)
//   cal_write16    every lane one 16-B store, 2 GiB                (2 GiB)
// Prints per kernel: launches, avg ms, and the "known" count to divide by.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                      \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                    \
      exit(1);                                                                                     \
    }                                                                                              \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void cal_read16(const f4 *__restrict__ p, size_t n4, float *out) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  float s = 0.f;
  if (i < n4) {
    f4 v = __builtin_nontemporal_load(p + i);
    s = v.x + v.y + v.z + v.w;
  }
  if (s == 12345.678f) out[0] = s; // never true for U[0,1) data: keeps the load
}
__global__ void cal_read4(const float *__restrict__ p, size_t n, float *out) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  float s = i < n ? p[i] : 0.f;
  if (s == 12345.678f) out[0] = s;
}
// line index l = (i * odd) mod 2^bits: a bijection, so every gather is on a
// distinct line, visited in scattered order
template <int FLOATS_PER_LINE>
__global__ void cal_gather(const float *__restrict__ p, unsigned bits, size_t count, float *out) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const size_t l = (i * 0x9E3779B1ull) & ((size_t(1) << bits) - 1);
  float s = p[l * FLOATS_PER_LINE];
  if (s == 12345.678f) out[0] = s;
}
__global__ void cal_scatter128(float *__restrict__ p, unsigned bits, size_t count) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const size_t l = (i * 0x9E3779B1ull) & ((size_t(1) << bits) - 1);
  p[l * 32] = (float)i;
}
__global__ void cal_write16(f4 *__restrict__ p, size_t n4) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n4) __builtin_nontemporal_store(f4{1.f, 2.f, 3.f, (float)i}, p + i);
}
__global__ void init_k(float *p, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = (float)((i * 2654435761u) & 0xFFFF) * (1.0f / 65536.0f);
}

int main() {
  const size_t table = size_t(1) << 30; // floats = 4 GiB
  float *t, *out;
  CK(hipMalloc(&t, table * 4));
  CK(hipMalloc(&out, 64));
  hipLaunchKernelGGL(init_k, dim3((unsigned)(table / 256)), dim3(256), 0, 0, t, table);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 5;
  auto run = [&](const char *name, double known, const char *unit, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; r++) launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-16s launches %d avg_ms %.4f known %.6g %s\n", name, reps + 1, ms / reps, known, unit);
  };
  const size_t half = table / 2; // 2 GiB of floats
  run("cal_read16", (double)half * 4, "bytes", [&] {
    hipLaunchKernelGGL(cal_read16, dim3((unsigned)(half / 4 / 256)), dim3(256), 0, 0, (const f4 *)t, half / 4, out);
  });
  run("cal_read4", (double)half * 4, "bytes", [&] {
    hipLaunchKernelGGL(cal_read4, dim3((unsigned)(half / 256)), dim3(256), 0, 0, t, half, out);
  });
  run("cal_gather128", (double)(size_t(1) << 25), "loads (distinct 128-B lines)", [&] {
    hipLaunchKernelGGL(cal_gather<32>, dim3((1u << 25) / 256), dim3(256), 0, 0, t, 25u, size_t(1) << 25, out);
  });
  run("cal_gather64", (double)(size_t(1) << 26), "loads (distinct 64-B halves)", [&] {
    hipLaunchKernelGGL(cal_gather<16>, dim3((1u << 26) / 256), dim3(256), 0, 0, t, 26u, size_t(1) << 26, out);
  });
  run("cal_scatter128", (double)(size_t(1) << 25), "stores (distinct 128-B lines)", [&] {
    hipLaunchKernelGGL(cal_scatter128, dim3((1u << 25) / 256), dim3(256), 0, 0, t, 25u, size_t(1) << 25);
  });
  run("cal_write16", (double)half * 4, "bytes", [&] {
    hipLaunchKernelGGL(cal_write16, dim3((unsigned)(half / 4 / 256)), dim3(256), 0, 0, (f4 *)t, half / 4);
  });
  CK(hipFree(t));
  CK(hipFree(out));
  return 0;
}
