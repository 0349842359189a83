// sort_digit_probe.hip -- measurement tool (not product): does an LSD radix
// pass with 11-bit digits (2048 bins) move keys fast enough for a 3-pass
// 11/11/10 sort to beat the shipped 4 x 8-bit onesweep?
//
// One pass WITHOUT look-back, in the shape of the shipped pass 0 (csrc/sort.hip:
// tile histogram -> every tile's digit bases, then rank / reorder in LDS /
// write-out of digit runs), for B = 8 and B = 11 bits, 16 K-key tiles of 256
// threads x 64 keys, 2^28 random uint32 keys:
//   hist_tiles   per-tile digit counts  (reads 4 B/key, writes NB words/tile)
//   bases (4 small kernels)  every (tile, digit)'s output base
//   scatter      load the tile, rank each key with one LDS ds_add_rtn,
//                exclusive scan of the counts, reorder the tile by digit in
//                LDS, write every digit run to its base (4 + 4 B/key)
// with tiles taken in dispatch order or in groups of 64 consecutive tiles
// per XCD (the shipped sort's grouping, which merges the partial 128-B lines
// at digit-run ends in one L2).  The shipped passes 1-3 add a look-back of NB
// status words per tile on top: 256 words at 8 bits, 2048 at 11 bits -- not
// modelled here, which favours B = 11.  Output is checked: digits
// non-decreasing over all 2^28 keys, key sum preserved.
// Prints one JSON line per (B, grouping): kernel ms (HIP events, median of 5).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
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

constexpr int NT = 256, KPT = 64, TILE = NT * KPT, NCH = 64;
typedef unsigned u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned hash32(unsigned x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

__global__ void gen(unsigned *k, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) k[i] = hash32((unsigned)i * 2654435761u + 12345u);
}

__device__ unsigned g_nxt[64 * 256];

template <int B> __device__ __forceinline__ unsigned digit(unsigned k) { return k & ((1u << B) - 1); }

// tile -> the tile a block takes: dispatch order, or groups of G consecutive
// tiles per XCD (block b runs on XCD b % 8 under round-robin dispatch)
template <bool GROUPED> __device__ __forceinline__ unsigned tile_of(unsigned b) {
  if (!GROUPED) return b;
  constexpr unsigned G = 64;
  const unsigned xcd = b % 8, j = b / 8;
  return ((j / G) * 8 + xcd) * G + j % G;
}

template <int B> __global__ __launch_bounds__(NT) void hist_tiles(const unsigned *keys, unsigned *hist) {
  constexpr int NB = 1 << B;
  __shared__ unsigned cnt[NB];
  for (int d = threadIdx.x; d < NB; d += NT) cnt[d] = 0;
  __syncthreads();
  const u4 *src = reinterpret_cast<const u4 *>(keys + (size_t)blockIdx.x * TILE);
#pragma unroll
  for (int j = 0; j < KPT / 4; j++) {
    const u4 v = __builtin_nontemporal_load(src + j * NT + threadIdx.x);
    atomicAdd(&cnt[digit<B>(v.x)], 1u);
    atomicAdd(&cnt[digit<B>(v.y)], 1u);
    atomicAdd(&cnt[digit<B>(v.z)], 1u);
    atomicAdd(&cnt[digit<B>(v.w)], 1u);
  }
  __syncthreads();
  for (int d = threadIdx.x; d < NB; d += NT) hist[(size_t)blockIdx.x * NB + d] = cnt[d];
}

// per (digit group of 64, chunk of tiles): the chunk's count per digit
template <int B> __global__ void chunk_sums(const unsigned *hist, unsigned ntiles, unsigned *csum) {
  constexpr int NB = 1 << B;
  const unsigned d = blockIdx.x * 64 + threadIdx.x, c = blockIdx.y, ct = ntiles / NCH;
  unsigned s = 0;
  for (unsigned t = c * ct; t < (c + 1) * ct; t++) s += hist[(size_t)t * NB + d];
  csum[c * NB + d] = s;
}

template <int B> __global__ void chunk_scan(const unsigned *csum, unsigned *cbase, unsigned *total) {
  constexpr int NB = 1 << B;
  const unsigned d = blockIdx.x * 64 + threadIdx.x;
  unsigned run = 0;
  for (int c = 0; c < NCH; c++) {
    cbase[c * NB + d] = run;
    run += csum[c * NB + d];
  }
  total[d] = run;
}

template <int B> __global__ void digit_start(const unsigned *total, unsigned *dstart) {
  constexpr int NB = 1 << B;
  if (threadIdx.x == 0) {
    unsigned run = 0;
    for (int d = 0; d < NB; d++) {
      dstart[d] = run;
      run += total[d];
    }
  }
}

template <int B>
__global__ void tile_bases(const unsigned *hist, const unsigned *cbase, const unsigned *dstart, unsigned ntiles,
                           unsigned *base) {
  constexpr int NB = 1 << B;
  const unsigned d = blockIdx.x * 64 + threadIdx.x, c = blockIdx.y, ct = ntiles / NCH;
  unsigned run = dstart[d] + cbase[c * NB + d];
  for (unsigned t = c * ct; t < (c + 1) * ct; t++) {
    base[(size_t)t * NB + d] = run;
    run += hist[(size_t)t * NB + d];
  }
}

// L4: 4-byte loads in the shipped kernel's layout (wave w owns keys
// [w*KPW, (w+1)*KPW), key r of lane l at w*KPW + r*64 + l: the layout its
// stable lane-ordered ranking needs) instead of 16-byte loads; NXT: count the
// next digit during the write-out (LDS atomics, as the shipped passes do)
template <int B, bool GROUPED, bool L4 = false, bool NXT = false>
__global__ __launch_bounds__(NT, 2) void scatter(const unsigned *keys, unsigned *out, const unsigned *base) {
  constexpr int NB = 1 << B;
  constexpr int PER = NB / NT; // counts per thread in the scan
  __shared__ unsigned cnt[NB];  // counts, then exclusive prefixes
  __shared__ unsigned sbase[NB]; // output base - prefix, per digit
  __shared__ unsigned buf[TILE]; // the reordered tile; its first words carry the wave sums of the scan
  unsigned *wsum = buf;          // (2 blocks per CU at B = 11 need <= 80 KiB of LDS)
  const unsigned tile = tile_of<GROUPED>(blockIdx.x);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int d = tid; d < NB; d += NT) cnt[d] = 0;
  __syncthreads();
  unsigned k[KPT];
  if constexpr (L4) {
    const unsigned *src = keys + (size_t)tile * TILE + wid * (TILE / (NT / 64)) + lane;
#pragma unroll
    for (int j = 0; j < KPT; j++) k[j] = __builtin_nontemporal_load(src + j * 64);
  } else {
    const u4 *src = reinterpret_cast<const u4 *>(keys + (size_t)tile * TILE);
#pragma unroll
    for (int j = 0; j < KPT / 4; j++) {
      const u4 v = __builtin_nontemporal_load(src + j * NT + tid);
      k[4 * j] = v.x;
      k[4 * j + 1] = v.y;
      k[4 * j + 2] = v.z;
      k[4 * j + 3] = v.w;
    }
  }
  unsigned short r[KPT];
#pragma unroll
  for (int j = 0; j < KPT; j++) r[j] = (unsigned short)atomicAdd(&cnt[digit<B>(k[j])], 1u);
  __syncthreads();
  // exclusive scan of cnt[0..NB): thread t owns [t*PER, (t+1)*PER)
  unsigned loc[PER > 0 ? PER : 1], s = 0;
  if constexpr (PER >= 1) {
#pragma unroll
    for (int q = 0; q < PER; q++) {
      loc[q] = s;
      s += cnt[tid * PER + q];
    }
  }
  unsigned incl = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) wsum[wid] = incl;
  __syncthreads();
  unsigned pre = incl - s;
  for (int w = 0; w < wid; w++) pre += wsum[w];
  if constexpr (PER >= 1) {
#pragma unroll
    for (int q = 0; q < PER; q++) {
      const int d = tid * PER + q;
      const unsigned p = pre + loc[q];
      cnt[d] = p;
      sbase[d] = base[(size_t)tile * NB + d] - p;
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < KPT; j++) buf[cnt[digit<B>(k[j])] + r[j]] = k[j];
  __syncthreads();
  __shared__ unsigned s_nxt[NXT ? NT / 64 : 1][NXT ? 256 : 1];
  if constexpr (NXT) {
    for (int i = tid; i < 4 * 256; i += NT) (&s_nxt[0][0])[i] = 0;
    __syncthreads();
  }
#pragma unroll 8
  for (int i = tid; i < TILE; i += NT) {
    const unsigned key = buf[i];
    out[sbase[digit<B>(key)] + i] = key;
    if constexpr (NXT) atomicAdd(&s_nxt[wid][(key >> B) & 255], 1u);
  }
  if constexpr (NXT) {
    __syncthreads();
    unsigned c = 0;
    for (int w = 0; w < NT / 64; w++) c += s_nxt[w][tid];
    if (c) atomicAdd(g_nxt + (tile % 64) * 256 + tid, c); // partitioned global counts, as the shipped pass
  }
}

static float med(std::vector<float> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

template <int B, bool GROUPED, bool L4 = false, bool NXT = false>
static void run(unsigned *keys, unsigned *out, size_t n, uint64_t keysum) {
  constexpr int NB = 1 << B;
  const unsigned ntiles = (unsigned)(n / TILE);
  unsigned *hist, *base, *csum, *cbase, *total, *dstart;
  CK(hipMalloc(&hist, (size_t)ntiles * NB * 4));
  CK(hipMalloc(&base, (size_t)ntiles * NB * 4));
  CK(hipMalloc(&csum, (size_t)NCH * NB * 4));
  CK(hipMalloc(&cbase, (size_t)NCH * NB * 4));
  CK(hipMalloc(&total, NB * 4));
  CK(hipMalloc(&dstart, NB * 4));
  hipEvent_t e[6];
  for (auto &x : e) CK(hipEventCreate(&x));
  std::vector<float> th, tb, ts;
  for (int rep = 0; rep < 6; rep++) {
    CK(hipEventRecord(e[0]));
    hipLaunchKernelGGL(hist_tiles<B>, dim3(ntiles), dim3(NT), 0, 0, keys, hist);
    CK(hipEventRecord(e[1]));
    hipLaunchKernelGGL(chunk_sums<B>, dim3(NB / 64, NCH), dim3(64), 0, 0, hist, ntiles, csum);
    hipLaunchKernelGGL(chunk_scan<B>, dim3(NB / 64), dim3(64), 0, 0, csum, cbase, total);
    hipLaunchKernelGGL(digit_start<B>, dim3(1), dim3(64), 0, 0, total, dstart);
    hipLaunchKernelGGL(tile_bases<B>, dim3(NB / 64, NCH), dim3(64), 0, 0, hist, cbase, dstart, ntiles, base);
    CK(hipEventRecord(e[2]));
    hipLaunchKernelGGL((scatter<B, GROUPED, L4, NXT>), dim3(ntiles), dim3(NT), 0, 0, keys, out, base);
    CK(hipEventRecord(e[3]));
    CK(hipGetLastError());
    CK(hipEventSynchronize(e[3]));
    float a, b, c;
    CK(hipEventElapsedTime(&a, e[0], e[1]));
    CK(hipEventElapsedTime(&b, e[1], e[2]));
    CK(hipEventElapsedTime(&c, e[2], e[3]));
    if (rep) { // rep 0 warms up
      th.push_back(a);
      tb.push_back(b);
      ts.push_back(c);
    }
  }
  // check: digits non-decreasing, key sum preserved
  std::vector<unsigned> h(n);
  CK(hipMemcpy(h.data(), out, n * 4, hipMemcpyDeviceToHost));
  size_t bad = 0;
  uint64_t sum = 0;
  for (size_t i = 0; i < n; i++) {
    sum += h[i];
    if (i && (h[i] & (NB - 1)) < (h[i - 1] & (NB - 1))) bad++;
  }
  const double sms = med(ts);
  printf("{\"bits\": %d, \"grouped\": %d, \"load4\": %d, \"next_count\": %d, \"keys\": %zu, \"hist_ms\": %.4f, \"bases_ms\": %.4f, \"scatter_ms\": %.4f, "
         "\"scatter_TBps\": %.3f, \"pass_ms\": %.4f, \"ok\": %s}\n",
         B, (int)GROUPED, (int)L4, (int)NXT, n, med(th), med(tb), sms, 8.0 * n / (sms * 1e-3) / 1e12, med(th) + med(tb) + sms,
         (bad == 0 && sum == keysum) ? "true" : "false");
  fflush(stdout);
  for (auto &x : e) CK(hipEventDestroy(x));
  CK(hipFree(hist));
  CK(hipFree(base));
  CK(hipFree(csum));
  CK(hipFree(cbase));
  CK(hipFree(total));
  CK(hipFree(dstart));
}

int main(int argc, char **argv) {
  const int log2n = argc > 1 ? atoi(argv[1]) : 28;
  const size_t n = size_t(1) << log2n;
  if (n % ((size_t)TILE * 8 * 64) != 0) {
    fprintf(stderr, "n must be a multiple of %d\n", TILE * 8 * 64);
    return 1;
  }
  unsigned *keys, *out;
  CK(hipMalloc(&keys, n * 4));
  CK(hipMalloc(&out, n * 4));
  hipLaunchKernelGGL(gen, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, keys, n);
  CK(hipDeviceSynchronize());
  std::vector<unsigned> h(n);
  CK(hipMemcpy(h.data(), keys, n * 4, hipMemcpyDeviceToHost));
  uint64_t keysum = 0;
  for (unsigned v : h) keysum += v;
  std::vector<unsigned>().swap(h);
  for (int round = 0; round < 2; round++) {
    run<8, false>(keys, out, n, keysum);
    run<8, true>(keys, out, n, keysum);
    run<11, false>(keys, out, n, keysum);
    run<11, true>(keys, out, n, keysum);
    run<8, true, true, false>(keys, out, n, keysum);
    run<8, true, true, true>(keys, out, n, keysum);
  }
  CK(hipFree(keys));
  CK(hipFree(out));
  return 0;
}
