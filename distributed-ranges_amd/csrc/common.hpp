// common.hpp -- shared device/host helpers for libdrhip (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <limits>
#include <type_traits>
#include <utility>
#include <vector>

#include "../../include/drhip.h"

namespace drhip {

// ---------------------------------------------------------------- runtime

// the range a segment's tile prefixes describe (drhip_reduce_tiles; the
// following drhip_inclusive_scan_tiles must scan that same range)
struct TilesRange {
  const void *x = nullptr;
  size_t n = 0;
  int dtype = -1, op = -1;
  unsigned per = 1;
};

struct Segment {
  int device = 0;
  hipStream_t stream = nullptr;
  int num_cus = 256;
  // Workspace: scan tile status, reduce block partials, sort scratch
  // descriptors.  Grown on demand (outside any timed region) and reused.
  void *ws = nullptr;
  size_t ws_bytes = 0;
  // Error word written by bounded in-kernel spins (pinned host memory).
  unsigned *err = nullptr;
  // Device words zeroed at drhip_init for kernels that count their finished
  // blocks and reset the count themselves (the last block folds and writes
  // 0 back), so a launch needs no memset node and replays in a HIP graph:
  // from word kSyncReduce the single-pass reduce's counters, from kSyncDot
  // the dot's (a top counter + up to 128 group counters, one 128-B line
  // each: reduce.hip last_block_fold).
  unsigned *dsync = nullptr;
  // drhip_reduce_tiles' per-tile prefixes and the range they describe (the
  // following drhip_inclusive_scan_tiles must scan that same range)
  void *tiles = nullptr;
  size_t tiles_bytes = 0;
  TilesRange tr;
  // HIP graphs (drhip_graph_*): captured graphs hold raw pointers to ws and
  // tiles, so neither may be reallocated while a graph of this segment is
  // alive (live_graphs) or being captured; the tile range a capture's
  // drhip_reduce_tiles describes takes effect when the graph is LAUNCHED
  // (tr is restored at drhip_graph_end to its value before the capture)
  // DRHIP_CHECK_TILES=1 (read at drhip_init): a 64-bit hash of the range at
  // drhip_reduce_tiles, recomputed and compared by drhip_inclusive_scan_tiles
  // (a changed input sets the error word) -- thash[0] at the reduce, [1] now
  bool check_tiles = false;
  unsigned long long *thash = nullptr;
  int live_graphs = 0;
  bool capturing = false, cap_tiles = false;
  TilesRange tr_before, tr_captured;
  // RCCL communicator (ncclComm_t) of this segment, or null (comm.hip).
  void *comm = nullptr;
  // Recorded on `stream` by drhip_free of another segment's memory, so the
  // free is ordered after the work every segment has queued (no host sync).
  hipEvent_t fence = nullptr;
  hipEvent_t null_fence = nullptr; // recorded on the device's NULL stream by drhip_free
  // drhip_malloc source: plain hipMalloc/hipFree (default) or the
  // stream-ordered pool (DRHIP_ALLOC=pool at drhip_init)
  bool pool = false;
  // DRHIP_ALLOC=pool with DRHIP_POOL=private: a pool of this segment's own
  // (hipMemPoolCreate) instead of the device's default pool
  hipMemPool_t own_pool = nullptr;
  // drhip_malloc source DRHIP_ALLOC=cache: this segment's freed hipMalloc
  // blocks, whole, by size class, each with the fences recorded at its free
  // (one per segment stream + the device's NULL stream): reused once every
  // fence has completed (csrc/runtime.hip cache_take)
  bool cache = false;
  struct Cached {
    void *base = nullptr;
    size_t cls = 0;
    std::vector<std::pair<int, hipEvent_t>> fences; // (device, event)
  };
  std::vector<Cached> cached;
  size_t cached_bytes = 0;
  // DRHIP_COPY=staged: pageable copies chunked through this pinned buffer
  void *stage = nullptr;
  size_t stage_bytes = 0;
};
enum : int { kSyncReduce = 0, kSyncDot = 8192, kSyncTiles = 16384, kSyncWords = 24576 };
// Destroys seg's communicator if it has one (drhip_finalize).
void comm_release(Segment &s);

int num_segments();
Segment *segment(int seg);                  // nullptr if bad index / not initialised
int ensure_workspace(int seg, size_t bytes); // grows seg's workspace
int seg_realloc(Segment *s, void **p, size_t nb); // replaces ws / tiles by nb bytes
// DRHIP_OK if seg's ws / tiles buffers may be reallocated now (no graph of
// the segment alive or being captured), else an error naming `what`
int may_reallocate(Segment *s, const char *what);
int set_hip_error(hipError_t e, const char *what);
int set_error(int code, const char *what);
// Ordering lane for persistent kernels (grid = the device's resident
// capacity, blocks spinning on other blocks' progress: the XCD-grouped
// onesweep sort).  Two such kernels running at once on one device can each
// hold CUs the other needs, so when several segments share a device
// (duplicated devices) persistent_lane_begin makes s's stream wait for the
// previous persistent work queued on that device and persistent_lane_end
// records s's; no-ops when s owns its device alone.
int persistent_lane_begin(Segment *s);
int persistent_lane_end(Segment *s);
// Inclusive +-scan of uint32 on seg's stream (scan.hip); used by the sort.
int scan_inclusive_u32(Segment *s, int seg, const uint32_t *in, uint32_t *out, size_t n);

#define DRHIP_CHECK_HIP(expr)                                                 \
  do {                                                                        \
    hipError_t _e = (expr);                                                   \
    if (_e != hipSuccess) return ::drhip::set_hip_error(_e, #expr);           \
  } while (0)

#define DRHIP_GET_SEG(var, seg)                                               \
  ::drhip::Segment *var = ::drhip::segment(seg);                              \
  do {                                                                        \
    if (::drhip::num_segments() == 0)                                         \
      return ::drhip::set_error(DRHIP_ERR_NOT_INIT, "drhip_init not called"); \
    if (!var) return ::drhip::set_error(DRHIP_ERR_BAD_SEG, "bad segment");    \
  } while (0)

// Every kernel launch is followed by this: captures launch failures.
#define DRHIP_CHECK_LAUNCH() DRHIP_CHECK_HIP(hipGetLastError())

// -------------------------------------------------------------- typing

template <typename T> struct acc_of { using type = T; };
template <> struct acc_of<float> { using type = double; };
template <typename T> using acc_t = typename acc_of<T>::type;

// In-tile compute type: floats stay fp32 inside a tile, ints are unsigned so
// wrapping is defined; converted back on store.
template <typename T> struct ctype_of { using type = T; };
template <> struct ctype_of<int32_t> { using type = uint32_t; };
template <> struct ctype_of<int64_t> { using type = uint64_t; };

template <int OP, typename T> struct Op;

template <typename T> struct Op<DRHIP_PLUS, T> {
  __host__ __device__ static T identity() { return T(0); }
  __host__ __device__ static T apply(T a, T b) { return a + b; }
};
template <typename T> struct Op<DRHIP_MUL, T> {
  __host__ __device__ static T identity() { return T(1); }
  __host__ __device__ static T apply(T a, T b) { return a * b; }
};
template <typename T> struct Op<DRHIP_MIN, T> {
  __host__ __device__ static T identity() {
    return std::numeric_limits<T>::has_infinity ? std::numeric_limits<T>::infinity()
                                                : std::numeric_limits<T>::max();
  }
  __host__ __device__ static T apply(T a, T b) { return b < a ? b : a; }
};
template <typename T> struct Op<DRHIP_MAX, T> {
  __host__ __device__ static T identity() {
    return std::numeric_limits<T>::has_infinity ? -std::numeric_limits<T>::infinity()
                                                : std::numeric_limits<T>::lowest();
  }
  __host__ __device__ static T apply(T a, T b) { return a < b ? b : a; }
};

// min/max on signed ints must compare signed: use the element type itself
// for those ops (no wrapping issue), unsigned only for +/*.
template <int OP, typename T> struct compute_of {
  using type = typename ctype_of<T>::type;
};
template <typename T> struct compute_of<DRHIP_MIN, T> { using type = T; };
template <typename T> struct compute_of<DRHIP_MAX, T> { using type = T; };
template <> struct compute_of<DRHIP_MIN, float> { using type = float; };
template <> struct compute_of<DRHIP_MAX, float> { using type = float; };
// fp32 products are formed in fp64: the exact product of two fp32 values fits
// in a double, so an elementwise a*b rounds identically; a long product
// chain (reduce / scan) no longer drifts (fp32 drifts ~2e-5 over 4095
// factors near 1).
template <> struct compute_of<DRHIP_MUL, float> { using type = double; };

// ------------------------------------------------------- dtype dispatch

template <typename F> int dispatch_dtype(int dtype, F &&f) {
  switch (dtype) {
  case DRHIP_I32: return f(int32_t{});
  case DRHIP_U32: return f(uint32_t{});
  case DRHIP_I64: return f(int64_t{});
  case DRHIP_U64: return f(uint64_t{});
  case DRHIP_F32: return f(float{});
  case DRHIP_F64: return f(double{});
  default: return set_error(DRHIP_ERR_BAD_ARG, "unsupported dtype");
  }
}

template <typename F> int dispatch_op(int op, F &&f) {
  switch (op) {
  case DRHIP_PLUS: return f(std::integral_constant<int, DRHIP_PLUS>{});
  case DRHIP_MUL: return f(std::integral_constant<int, DRHIP_MUL>{});
  case DRHIP_MIN: return f(std::integral_constant<int, DRHIP_MIN>{});
  case DRHIP_MAX: return f(std::integral_constant<int, DRHIP_MAX>{});
  default: return set_error(DRHIP_ERR_BAD_ARG, "unsupported op");
  }
}

template <typename T> constexpr int dtype_code_of() {
  if constexpr (std::is_same_v<T, int32_t>) return DRHIP_I32;
  else if constexpr (std::is_same_v<T, uint32_t>) return DRHIP_U32;
  else if constexpr (std::is_same_v<T, int64_t>) return DRHIP_I64;
  else if constexpr (std::is_same_v<T, uint64_t>) return DRHIP_U64;
  else if constexpr (std::is_same_v<T, float>) return DRHIP_F32;
  else return DRHIP_F64;
}

inline size_t dtype_size(int dtype) {
  switch (dtype) {
  case DRHIP_I32: case DRHIP_U32: case DRHIP_F32: return 4;
  case DRHIP_I64: case DRHIP_U64: case DRHIP_F64: return 8;
  default: return 0;
  }
}

// --------------------------------------------------------- device bits

constexpr int kWave = 64;

// 16-byte vector of T (the coalescing sweet spot: 1 KiB per wave-instruction).
template <typename T> struct alignas(16) Vec16 {
  static constexpr int N = 16 / sizeof(T);
  T v[N];
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Nontemporal 16-byte load / store for data a kernel streams exactly once:
// keeps the Infinity Cache and L2 for re-read data (tools/reduce_sweep.hip:
// f32 sum of 2^30 elements 0.687 -> 0.608 ms, 6.25 -> 7.07 TB/s).
template <typename T> __device__ __forceinline__ Vec16<T> load_nt(const Vec16<T> *p) {
  const u32x4 w = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
  Vec16<T> r;
  __builtin_memcpy(&r, &w, 16);
  return r;
}
template <typename T> __device__ __forceinline__ void store_nt(Vec16<T> *p, const Vec16<T> &v) {
  u32x4 w;
  __builtin_memcpy(&w, &v, 16);
  __builtin_nontemporal_store(w, reinterpret_cast<u32x4 *>(p));
}

template <typename T> __device__ __forceinline__ T shfl_xor(T x, int m) {
  if constexpr (sizeof(T) == 8) {
    uint64_t u;
    __builtin_memcpy(&u, &x, 8);
    uint32_t lo = (uint32_t)u, hi = (uint32_t)(u >> 32);
    lo = __shfl_xor(lo, m, kWave);
    hi = __shfl_xor(hi, m, kWave);
    u = ((uint64_t)hi << 32) | lo;
    T r;
    __builtin_memcpy(&r, &u, 8);
    return r;
  } else {
    uint32_t u;
    __builtin_memcpy(&u, &x, 4);
    u = __shfl_xor(u, m, kWave);
    T r;
    __builtin_memcpy(&r, &u, 4);
    return r;
  }
}

template <typename T> __device__ __forceinline__ T shfl_up(T x, int d) {
  if constexpr (sizeof(T) == 8) {
    uint64_t u;
    __builtin_memcpy(&u, &x, 8);
    uint32_t lo = (uint32_t)u, hi = (uint32_t)(u >> 32);
    lo = __shfl_up(lo, d, kWave);
    hi = __shfl_up(hi, d, kWave);
    u = ((uint64_t)hi << 32) | lo;
    T r;
    __builtin_memcpy(&r, &u, 8);
    return r;
  } else {
    uint32_t u;
    __builtin_memcpy(&u, &x, 4);
    u = __shfl_up(u, d, kWave);
    T r;
    __builtin_memcpy(&r, &u, 4);
    return r;
  }
}

template <typename T> __device__ __forceinline__ T shfl_idx(T x, int src) {
  if constexpr (sizeof(T) == 8) {
    uint64_t u;
    __builtin_memcpy(&u, &x, 8);
    uint32_t lo = (uint32_t)u, hi = (uint32_t)(u >> 32);
    lo = __shfl(lo, src, kWave);
    hi = __shfl(hi, src, kWave);
    u = ((uint64_t)hi << 32) | lo;
    T r;
    __builtin_memcpy(&r, &u, 8);
    return r;
  } else {
    uint32_t u;
    __builtin_memcpy(&u, &x, 4);
    u = __shfl(u, src, kWave);
    T r;
    __builtin_memcpy(&r, &u, 4);
    return r;
  }
}

// Butterfly all-reduce across the 64-lane wave.
template <int OP, typename T> __device__ __forceinline__ T wave_reduce(T x) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) x = Op<OP, T>::apply(x, shfl_xor(x, m));
  return x;
}

// ---- DPP wave primitives (GFX9 row_shr / row_bcast / wave_shr): no LDS
// traffic, no address registers, one VALU op + one DPP move per step.
// `old` = identity is what a lane receives when its DPP source is outside
// the row / masked row, so apply(x, identity) leaves it unchanged.
enum : int {
  DPP_ROW_SHR1 = 0x111, DPP_ROW_SHR2 = 0x112, DPP_ROW_SHR4 = 0x114, DPP_ROW_SHR8 = 0x118,
  DPP_WAVE_SHL1 = 0x130, DPP_WAVE_SHR1 = 0x138, DPP_ROW_BCAST15 = 0x142, DPP_ROW_BCAST31 = 0x143
};

template <int CTRL, int ROW_MASK, typename T> __device__ __forceinline__ T dpp_move(T old, T x) {
  if constexpr (sizeof(T) == 8) {
    uint64_t uo, ux;
    __builtin_memcpy(&uo, &old, 8);
    __builtin_memcpy(&ux, &x, 8);
    const int lo = __builtin_amdgcn_update_dpp((int)(uint32_t)uo, (int)(uint32_t)ux, CTRL, ROW_MASK, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(uint32_t)(uo >> 32), (int)(uint32_t)(ux >> 32), CTRL,
                                               ROW_MASK, 0xf, false);
    const uint64_t r = ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
    T t;
    __builtin_memcpy(&t, &r, 8);
    return t;
  } else {
    int io, ix;
    __builtin_memcpy(&io, &old, 4);
    __builtin_memcpy(&ix, &x, 4);
    const int r = __builtin_amdgcn_update_dpp(io, ix, CTRL, ROW_MASK, 0xf, false);
    T t;
    __builtin_memcpy(&t, &r, 4);
    return t;
  }
}

// Inclusive scan across the 64-lane wave: within 16-lane rows by shifts
// 1, 2, 4, 8, then row 0/2 totals into rows 1/3 (row_bcast:15) and the
// rows 0-1 total into rows 2-3 (row_bcast:31).
template <int OP, typename T> __device__ __forceinline__ T wave_inclusive_scan(T x) {
  using O = Op<OP, T>;
  const T id = O::identity();
  x = O::apply(dpp_move<DPP_ROW_SHR1, 0xf>(id, x), x);
  x = O::apply(dpp_move<DPP_ROW_SHR2, 0xf>(id, x), x);
  x = O::apply(dpp_move<DPP_ROW_SHR4, 0xf>(id, x), x);
  x = O::apply(dpp_move<DPP_ROW_SHR8, 0xf>(id, x), x);
  x = O::apply(dpp_move<DPP_ROW_BCAST15, 0xa>(id, x), x);
  x = O::apply(dpp_move<DPP_ROW_BCAST31, 0xc>(id, x), x);
  return x;
}

// Lane i receives lane i-1's value; lane 0 receives `fill`.
template <typename T> __device__ __forceinline__ T wave_shift_up1(T x, T fill) {
  return dpp_move<DPP_WAVE_SHR1, 0xf>(fill, x);
}

// Lane i receives lane i+1's value; lane 63 receives `fill`.
template <typename T> __device__ __forceinline__ T wave_shift_down1(T x, T fill) {
  return dpp_move<DPP_WAVE_SHL1, 0xf>(fill, x);
}

template <typename T> __device__ __forceinline__ uint64_t to_bits64(T x) {
  if constexpr (sizeof(T) == 8) {
    uint64_t u;
    __builtin_memcpy(&u, &x, 8);
    return u;
  } else {
    uint32_t u;
    __builtin_memcpy(&u, &x, 4);
    return u;
  }
}
template <typename T> __device__ __forceinline__ T from_bits64(uint64_t u) {
  T r;
  if constexpr (sizeof(T) == 8) {
    __builtin_memcpy(&r, &u, 8);
  } else {
    uint32_t v = (uint32_t)u;
    __builtin_memcpy(&r, &v, 4);
  }
  return r;
}

inline unsigned grid_cap(const Segment *s, int blocks_per_cu) {
  return (unsigned)(s->num_cus * blocks_per_cu);
}

} // namespace drhip
