// scan_sweep.hip -- measurement tool (not product): times scan_kernel
// variants (vectors per thread U, fp32 final combine, nontemporal stores,
// look-back removed) against a copy kernel of the same tile shape on a
// 2^30-element f32 vector.  Build: make -C tools scan_sweep.
#include "../distributed-ranges_amd/csrc/scan_kernel.hpp"

#include <cstring>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_reduce.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

// Rejected design kept for the record: 1.86-2.0 ms vs 1.62 ms
// for the look-back kernel at 2^30 f32.

namespace drhip {

// ---------------------------------------------------------------------------
// Chunked scan through the Infinity Cache (prototype, tools/scan_sweep.hip).
// The range is cut into chunks small enough that a chunk read once stays in
// the 256 MiB Infinity Cache until it is read again.  Launch i runs two block
// roles: blocks [0, nscan) scan chunk i tile by tile, each tile's prefix being
// carry[i] + the fp64 sum of the chunk's earlier tile aggregates (computed by
// launch i-1, so no in-launch waiting at all); blocks [nscan, nscan+nred)
// read chunk i+1 once (default cache policy: it lands in the Infinity Cache)
// and write its tile aggregates.  HBM traffic stays 4 B read + 4 B written
// per element; the second read of each element is an Infinity Cache hit.
template <typename A> struct ChunkArgs {
  const A *agg;      // tile aggregates of the chunk scanned here
  A *next_agg;       // tile aggregates of the next chunk (reduce role)
  const A *carry_in; // carry[i]
  A *carry_out;      // carry[i+1] (written by the last scan tile)
  unsigned nscan, nred;
  const void *next_in;
  size_t next_n;
};

template <int OP, typename T, int U>
__global__ __launch_bounds__(kScanThreads) void scan_chunk_kernel(const T *in, T *out, size_t n,
                                                                 ChunkArgs<scan_acc_t<OP, T>> ca) {
  using C = scan_c_t<OP, T>;
  using A = scan_acc_t<OP, T>;
  using OpC = Op<OP, C>;
  using OpA = Op<OP, A>;
  constexpr int V = Vec16<T>::N;
  constexpr size_t TILE = (size_t)kScanThreads * U * V;
  __shared__ C s_wt[U][kScanWaves];
  __shared__ C s_pre[U][kScanWaves];
  __shared__ A s_excl;
  __shared__ A s_red[kScanWaves];
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;

  if (blockIdx.x >= ca.nscan) {
    // ---- reduce role: one tile of the next chunk, default-policy loads
    const size_t t = blockIdx.x - ca.nscan;
    const T *nin = static_cast<const T *>(ca.next_in);
    const size_t base = t * TILE;
    C s = OpC::identity();
    if (base + TILE <= ca.next_n) {
      const Vec16<T> *src = reinterpret_cast<const Vec16<T> *>(nin + base);
#pragma unroll
      for (int u = 0; u < U; u++) {
        const Vec16<T> r = src[u * kScanThreads + tid];
#pragma unroll
        for (int j = 0; j < V; j++) s = OpC::apply(s, (C)r.v[j]);
      }
    } else {
      for (size_t g = base + tid; g < ca.next_n; g += kScanThreads) s = OpC::apply(s, (C)nin[g]);
    }
    A sa = wave_reduce<OP>((A)s);
    if (lane == 0) s_red[wid] = sa;
    __syncthreads();
    if (tid == 0) {
      A r = s_red[0];
#pragma unroll
      for (int w = 1; w < kScanWaves; w++) r = OpA::apply(r, s_red[w]);
      ca.next_agg[t] = r;
    }
    return;
  }

  // ---- scan role
  const size_t tile = blockIdx.x;
  const size_t base = tile * TILE;
  const bool full = base + TILE <= n;
  C v[U][V];
  if (full) {
    const Vec16<T> *src = reinterpret_cast<const Vec16<T> *>(in + base);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const Vec16<T> r = load_nt(src + u * kScanThreads + tid);
#pragma unroll
      for (int j = 0; j < V; j++) v[u][j] = (C)r.v[j];
    }
  } else {
    const T *src = in + base;
    const unsigned rem = (unsigned)(n - base);
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int j = 0; j < V; j++) {
        const unsigned li = ((unsigned)u * kScanThreads + tid) * V + j;
        v[u][j] = li < rem ? (C)src[li] : OpC::identity();
        __builtin_amdgcn_sched_barrier(0);
      }
  }
#pragma unroll
  for (int u = 0; u < U; u++)
#pragma unroll
    for (int j = 1; j < V; j++) v[u][j] = OpC::apply(v[u][j - 1], v[u][j]);
  C w[U];
#pragma unroll
  for (int u = 0; u < U; u++) w[u] = wave_inclusive_scan<OP>(v[u][V - 1]);
  if (lane == kWave - 1) {
#pragma unroll
    for (int u = 0; u < U; u++) s_wt[u][wid] = w[u];
  }
#pragma unroll
  for (int u = 0; u < U; u++) w[u] = wave_shift_up1(w[u], OpC::identity());
  __syncthreads();
  if (wid == 0) {
    constexpr int NP = U * kScanWaves;
    const C pt = lane < NP ? (&s_wt[0][0])[lane] : OpC::identity();
    const C incl = wave_inclusive_scan<OP>(pt);
    const C pre = wave_shift_up1(incl, OpC::identity());
    if (lane < NP) (&s_pre[0][0])[lane] = pre;
    const C agg = shfl_idx(incl, kWave - 1);
    // prefix of this tile: carry + aggregates of the chunk's earlier tiles
    A e = OpA::identity();
    for (size_t t = lane; t < tile; t += kWave) e = OpA::apply(e, ca.agg[t]);
    e = wave_reduce<OP>(e);
    const A excl = OpA::apply(*ca.carry_in, e);
    if (lane == 0) {
      s_excl = excl;
      if (tile == ca.nscan - 1) *ca.carry_out = OpA::apply(excl, (A)agg);
    }
  }
  __syncthreads();
  const A excl = s_excl;
#pragma unroll
  for (int u = 0; u < U; u++) {
    const C pw = OpC::apply(s_pre[u][wid], w[u]);
#pragma unroll
    for (int j = 0; j < V; j++) v[u][j] = OpC::apply(pw, v[u][j]);
  }
  if (full) {
    Vec16<T> *dst = reinterpret_cast<Vec16<T> *>(out + base);
#pragma unroll
    for (int u = 0; u < U; u++) {
      Vec16<T> r;
#pragma unroll
      for (int j = 0; j < V; j++) r.v[j] = (T)OpA::apply(excl, (A)v[u][j]);
      store_nt(dst + u * kScanThreads + tid, r);
    }
  } else {
    T *dst = out + base;
    const unsigned rem = (unsigned)(n - base);
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int j = 0; j < V; j++) {
        const unsigned li = ((unsigned)u * kScanThreads + tid) * V + j;
        if (li < rem) dst[li] = (T)OpA::apply(excl, (A)v[u][j]);
        __builtin_amdgcn_sched_barrier(0);
      }
  }
}

} // namespace drhip

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

// (rejected design, kept here as a measured variant)
// Persistent variant: the grid is the resident capacity; each block loops
// over tiles claimed one ahead (scan_tile's NEXT).  Forward progress: the
// smallest unfinished claimed tile is either some block's current tile (all
// its predecessors are finished) or some block's next claim, whose current
// tile -- claimed earlier, hence smaller -- is then finished.
template <int OP, typename T, bool ALIGNED, int U, int FLAGS, int MINW>
__global__ __launch_bounds__(kScanThreads, MINW) void scan_kernel_persist(const T *in, T *out, size_t n,
                                                                         unsigned *counter,
                                                                         granules_t<OP, T> gr,
                                                                         int has_init, scan_c_t<OP, T> init,
                                                                         ScanArgs<scan_acc_t<OP, T>> a) {
  constexpr size_t TILE = (size_t)kScanThreads * U * Vec16<T>::N;
  const size_t ntiles = (n + TILE - 1) / TILE;
  __shared__ ScanSmem<OP, T, U> sm;
  if (threadIdx.x == 0) sm.s_tile = atomicAdd(counter, 1u);
  __syncthreads();
  size_t tile = sm.s_tile;
  while (tile < ntiles) {
    scan_tile<OP, T, ALIGNED, U, FLAGS>(in, out, n, tile, counter, gr, has_init, init, a, sm);
    tile = sm.s_next; // written before scan_tile's second barrier
    __syncthreads();  // everyone has read s_next / s_pre before the next tile reuses them
  }
}

struct Ctx {
  float *in, *out;
  size_t n;
  char *ws;
  unsigned *err;
  hipStream_t st;
  int persist_mult = 0;
};

template <int U, int FLAGS, int MINW = 1, int NT = 256> static double run_scan(Ctx &c, int reps, double *last) {
  constexpr size_t TILE = NT * U * 4;
  const size_t ntiles = (c.n + TILE - 1) / TILE;
  const size_t gran_b = (ntiles * 32 + 1023) & ~size_t(1023);
  granules_t<DRHIP_PLUS, float> gr;
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
    if (FLAGS & SCAN_PERSIST) {
      static int per_cu = 0, cus = 0;
      if (!per_cu) {
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per_cu, scan_kernel_persist<DRHIP_PLUS, float, true, U, FLAGS, MINW>, 256, 0));
        hipDeviceProp_t p;
        CK(hipGetDeviceProperties(&p, 0));
        cus = p.multiProcessorCount;
        printf("  persistent: %d blocks/CU x %d CUs\n", per_cu, cus);
      }
      const size_t grid = std::min<size_t>(ntiles, (size_t)per_cu * cus * (c.persist_mult ? c.persist_mult : 1));
      hipLaunchKernelGGL((scan_kernel_persist<DRHIP_PLUS, float, true, U, FLAGS, MINW>), dim3((unsigned)grid), dim3(256),
                         0, c.st, c.in, c.out, c.n, (unsigned *)c.ws, gr, 0, 0.0f, a);
    } else {
      hipLaunchKernelGGL((scan_kernel<DRHIP_PLUS, float, true, U, FLAGS, MINW, NT>), dim3((unsigned)ntiles), dim3(NT),
                         0, c.st, c.in, c.out, c.n, (unsigned *)c.ws, gr, 0, 0.0f, a);
    }
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

// chunked scan through the Infinity Cache: chunk = CHE elements
template <int U> static double run_chunked(Ctx &c, size_t che, int reps, double *last) {
  constexpr size_t TILE = 256 * U * 4;
  const size_t nch = (c.n + che - 1) / che;
  const size_t tpc = (che + TILE - 1) / TILE;
  double *agg = (double *)(c.ws + 256);          // [2][tpc]
  double *carry = agg + 2 * tpc + 64;            // [nch + 1]
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float sum = 0;
  for (int r = -2; r < reps; r++) {
    CK(hipMemsetAsync(carry, 0, 8, c.st));
    CK(hipEventRecord(e0, c.st));
    for (size_t i = 0; i <= nch; i++) {
      ChunkArgs<double> a{};
      const size_t n_i = i < nch ? std::min(che, c.n - i * che) : 0;
      const size_t n_next = i + 1 < nch ? std::min(che, c.n - (i + 1) * che) : 0;
      a.nscan = (unsigned)((n_i + TILE - 1) / TILE);
      a.nred = (unsigned)((n_next + TILE - 1) / TILE);
      if (i == 0) { // prologue: reduce chunk 0 only
        a.nscan = 0;
        a.nred = (unsigned)((std::min(che, c.n) + TILE - 1) / TILE);
        a.next_in = c.in;
        a.next_n = std::min(che, c.n);
        a.next_agg = agg;
        hipLaunchKernelGGL((scan_chunk_kernel<DRHIP_PLUS, float, U>), dim3(a.nred), dim3(256), 0, c.st, c.in, c.out,
                           0, a);
        continue;
      }
      const size_t ci = i - 1; // chunk scanned in this launch
      const size_t nci = std::min(che, c.n - ci * che);
      a.nscan = (unsigned)((nci + TILE - 1) / TILE);
      const size_t nn = ci + 1 < nch ? std::min(che, c.n - (ci + 1) * che) : 0;
      a.nred = (unsigned)((nn + TILE - 1) / TILE);
      a.agg = agg + (ci & 1) * tpc;
      a.next_agg = agg + ((ci + 1) & 1) * tpc;
      a.carry_in = carry + ci;
      a.carry_out = carry + ci + 1;
      a.next_in = c.in + (ci + 1) * che;
      a.next_n = nn;
      hipLaunchKernelGGL((scan_chunk_kernel<DRHIP_PLUS, float, U>), dim3(a.nscan + a.nred), dim3(256), 0, c.st,
                         c.in + ci * che, c.out + ci * che, nci, a);
    }
    CK(hipEventRecord(e1, c.st));
    CK(hipStreamSynchronize(c.st));
    if (r >= 0) sum += elapsed(e0, e1);
  }
  float l;
  CK(hipMemcpy(&l, c.out + c.n - 1, 4, hipMemcpyDeviceToHost));
  *last = l;
  return sum / reps;
}

#define CHUNKED(U, LOG2CHE)                                                                       \
  do {                                                                                             \
    double last;                                                                                   \
    double ms = run_chunked<U>(c, size_t(1) << LOG2CHE, reps, &last);                              \
    printf("chunked U=%-2d chunk 2^%d        %8.3f ms %7.1f GB/s  last=%.6e rel=%.2e\n", U, LOG2CHE, ms,   \
           bytes / ms / 1e6, last, (last - ref) / ref);                                             \
  } while (0)

template <int U, int FLAGS, int MINW = 1> static void run_diag(Ctx &c) {
  constexpr size_t TILE = 256 * U * 4;
  const size_t ntiles = (c.n + TILE - 1) / TILE;
  const size_t gran_b = (ntiles * 32 + 1023) & ~size_t(1023);
  granules_t<DRHIP_PLUS, float> gr;
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
  if (argc > 3 && atoi(argv[3]) == 6) {
    // fp32 final combine (SCAN_F32_COMBINE) A/B
    for (int k = 0; k < 3; k++) {
      SCANW(32, kScanFlags, 1, "U32 f64 combine");
      SCANW(32, kScanFlags | SCAN_F32_COMBINE, 1, "U32 f32 combine");
    }
    return 0;
  }
  if (argc > 3 && atoi(argv[3]) == 5) {
    // early look-back (SCAN_EARLY_LB) A/B on top of the early aggregate
    for (int k = 0; k < 3; k++) {
      SCANW(32, kScanFlags | SCAN_EARLY_AGG, 1, "U32 early agg");
      SCANW(32, kScanFlags | SCAN_EARLY_AGG | SCAN_EARLY_LB, 1, "U32 early lb");
    }
    SCANW(16, kScanFlags | SCAN_EARLY_AGG, 1, "U16 early agg");
    SCANW(16, kScanFlags | SCAN_EARLY_AGG | SCAN_EARLY_LB, 1, "U16 early lb");
    run_diag<32, kScanFlags | SCAN_EARLY_AGG>(c);
    run_diag<32, kScanFlags | SCAN_EARLY_AGG | SCAN_EARLY_LB>(c);
    return 0;
  }
  if (argc > 3 && atoi(argv[3]) == 4) {
    // early tile aggregate (SCAN_EARLY_AGG) A/B, interleaved
    for (int k = 0; k < 3; k++) {
      SCANW(32, kScanFlags & ~SCAN_EARLY_AGG, 1, "U32 late agg");
      SCANW(32, kScanFlags | SCAN_EARLY_AGG, 1, "U32 early agg");
    }
    run_diag<32, kScanFlags & ~SCAN_EARLY_AGG>(c);
    run_diag<32, kScanFlags | SCAN_EARLY_AGG>(c);
    return 0;
  }
  SCANW(16, kScanFlags, 1, "product U16");
  SCANW(32, kScanFlags, 1, "product U32");
  SCANW(16, kScanFlags | SCAN_NO_LOOKBACK, 1, "no look-back");
  SCANW(32, kScanFlags | SCAN_NO_LOOKBACK, 1, "no look-back");
  {
    double last;
    double ms = run_scan<32, kScanFlags, 1, 512>(c, reps, &last);
    printf("scan U=32 512 thr  %8.3f ms %7.1f GB/s rel=%.2e\n", ms, bytes / ms / 1e6, (last - ref) / ref);
    ms = run_scan<16, kScanFlags, 1, 512>(c, reps, &last);
    printf("scan U=16 512 thr  %8.3f ms %7.1f GB/s rel=%.2e\n", ms, bytes / ms / 1e6, (last - ref) / ref);
    ms = run_scan<24, kScanFlags, 1, 512>(c, reps, &last);
    printf("scan U=24 512 thr  %8.3f ms %7.1f GB/s rel=%.2e\n", ms, bytes / ms / 1e6, (last - ref) / ref);
    ms = run_scan<32, kScanFlags, 1, 1024>(c, reps, &last);
    printf("scan U=32 1024 thr %8.3f ms %7.1f GB/s rel=%.2e\n", ms, bytes / ms / 1e6, (last - ref) / ref);
  }
  if (argc > 3 && atoi(argv[3]) == 3) {
    SCANW(16, SCAN_NT_STORE, 1, "global ld/st");
    SCANW(32, SCAN_NT_STORE | SCAN_BUFFER, 1, "buffer, cached ld");
    SCANW(40, kScanFlags, 1, "");
    SCANW(48, kScanFlags, 1, "");
  }
  if (argc > 3 && atoi(argv[3]) == 2) {
    SCANW(16, kScanFlags | SCAN_PERSIST, 1, "persistent");
    SCANW(8, kScanFlags, 1, "");
  }
  run_diag<16, kScanFlags>(c);
  run_diag<32, kScanFlags>(c);
  if (argc > 3 && atoi(argv[3]) == 1) {
    CHUNKED(16, 22);
    CHUNKED(16, 24);
  }
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
