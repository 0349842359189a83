// runtime.hip -- device registry, streams, memory and error state.
//
// Replaces the reference's SYCL device layer: shp::init/devices/nprocs
// (include/dr/shp/init.hpp:16-52), the USM allocators
// (shp/allocators.hpp:13-72), shp::copy/copy_async/fill_async
// (shp/copy.hpp:19-173).  Where the reference creates a new sycl::queue per
// segment per algorithm call (e.g. reduce.hpp:63, for_each.hpp:106), every
// segment here owns ONE non-blocking HIP stream for its lifetime.
#include "common.hpp"


#include <cstdio>
#include <mutex>
#include <string>
#include <map>
#include <unordered_map>
#include <vector>

namespace drhip {

namespace {
std::vector<Segment> g_segs;
std::string g_err = "ok";
std::mutex g_mu;
// Live device blocks handed out by drhip_malloc (kind 'u') and the
// segments' internal buffers (workspace 'w', tile prefixes 't'), keyed by
// the base address of their reservation: every new block is checked against
// them (alloc_track), see drhip_free.
struct LiveRec {
  int seg = 0;
  char kind = 'u';
  size_t bytes = 0;      // the caller's size
  size_t total = 0;      // the reservation: bytes + 2 red zones in guard mode
  uintptr_t user = 0;    // the pointer the caller got (base + red zone)
  unsigned long long serial = 0;
};
static std::mutex g_live_mu;
static std::map<uintptr_t, LiveRec> g_live;
static unsigned long long g_serial = 0;
// DRHIP_ALLOC_TRACE=<path>: one line per allocation / free (tools/pool_replay.hip)
static FILE *g_trace = nullptr;
// DRHIP_ALLOC_GUARD=1: red zones of kGuard bytes on both sides of every
// drhip_malloc block, filled with kGuardWord and checked on drhip_free and
// drhip_sync -- an out-of-bounds store by a kernel, memset or copy of this
// library becomes a named failure with the block it hit.
static bool g_guard = false;
constexpr size_t kGuard = 4096;
constexpr unsigned kGuardWord = 0xA5C3E10Fu;
// live graph execs (drhip_graph_end .. drhip_graph_destroy): their segment
// and the tile range a captured drhip_reduce_tiles leaves when replayed
struct GraphRec {
  int seg = -1;
  bool has_tiles = false;
  TilesRange tiles;
};
std::unordered_map<void *, GraphRec> g_graphs;
} // namespace

int num_segments() { return (int)g_segs.size(); }

namespace {
// per device: the event closing the last persistent kernel sequence queued
// on it (persistent_lane_*), created when a device hosts > 1 segment
hipEvent_t g_lane[256];
bool g_lane_used[256];
bool device_shared(const Segment *s) {
  int k = 0;
  for (auto &o : g_segs) k += o.device == s->device;
  return k > 1;
}
} // namespace

int persistent_lane_begin(Segment *s) {
  const int d = s->device & 255;
  if (!device_shared(s)) return DRHIP_OK;
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  if (!g_lane[d]) DRHIP_CHECK_HIP(hipEventCreateWithFlags(&g_lane[d], hipEventDisableTiming));
  if (g_lane_used[d]) DRHIP_CHECK_HIP(hipStreamWaitEvent(s->stream, g_lane[d], 0));
  return DRHIP_OK;
}

int persistent_lane_end(Segment *s) {
  const int d = s->device & 255;
  if (!device_shared(s)) return DRHIP_OK;
  DRHIP_CHECK_HIP(hipEventRecord(g_lane[d], s->stream));
  g_lane_used[d] = true;
  return DRHIP_OK;
}

Segment *segment(int seg) {
  if (seg < 0 || seg >= (int)g_segs.size()) return nullptr;
  return &g_segs[seg];
}

int set_hip_error(hipError_t e, const char *what) {
  g_err = std::string(what) + ": " + hipGetErrorString(e);
  return DRHIP_ERR_HIP;
}

int set_error(int code, const char *what) {
  g_err = what;
  return code;
}

// Registers the reservation [base, base + total) as live.  A block that
// overlaps one already live -- the allocator handing out memory it has
// handed out before and that was not freed -- is refused with
// DRHIP_ERR_ALLOC and kept out of circulation (never freed: its pages are
// another block's), and both blocks are named on stderr.
int alloc_track(int seg, char kind, void *base, size_t total, size_t bytes, void *user) {
  std::lock_guard<std::mutex> lk(g_live_mu);
  const uintptr_t b = (uintptr_t)base, e = b + total;
  auto it = g_live.upper_bound(b);
  const LiveRec *hit = nullptr;
  uintptr_t hb = 0;
  if (it != g_live.begin()) {
    auto p = std::prev(it);
    if (p->first + p->second.total > b) hit = &p->second, hb = p->first;
  }
  if (!hit && it != g_live.end() && it->first < e) hit = &it->second, hb = it->first;
  const unsigned long long serial = ++g_serial;
  if (g_trace) {
    std::fprintf(g_trace, "M %llu %d %c 0x%llx %zu%s\n", serial, seg, kind, (unsigned long long)b, total,
                 hit ? " OVERLAP" : "");
    std::fflush(g_trace);
  }
  if (hit) {
    char msg[512];
    std::snprintf(msg, sizeof msg,
                  "the allocator returned [%p, %p) (segment %d, kind %c, %zu B, allocation #%llu) overlapping the live "
                  "block [%p, %p) (segment %d, kind %c, %zu B, allocation #%llu)",
                  base, (void *)e, seg, kind, total, serial, (void *)hb, (void *)(hb + hit->total), hit->seg, hit->kind,
                  hit->total, hit->serial);
    std::fprintf(stderr, "drhip: %s\n", msg);
    return set_error(DRHIP_ERR_ALLOC, msg);
  }
  LiveRec r;
  r.seg = seg;
  r.kind = kind;
  r.bytes = bytes;
  r.total = total;
  r.user = (uintptr_t)user;
  r.serial = serial;
  g_live[b] = r;
  return DRHIP_OK;
}

// The live record whose caller pointer is `user` (false if none): its base
// goes to *base.
static bool alloc_find(const void *user, uintptr_t *base, LiveRec *rec) {
  std::lock_guard<std::mutex> lk(g_live_mu);
  auto it = g_live.upper_bound((uintptr_t)user);
  if (it == g_live.begin()) return false;
  --it;
  if (it->second.user != (uintptr_t)user) return false;
  *base = it->first;
  *rec = it->second;
  return true;
}

static void alloc_untrack(uintptr_t base) {
  std::lock_guard<std::mutex> lk(g_live_mu);
  auto it = g_live.find(base);
  if (it == g_live.end()) return;
  if (g_trace) {
    std::fprintf(g_trace, "F %llu %d %c 0x%llx %zu\n", it->second.serial, it->second.seg, it->second.kind,
                 (unsigned long long)base, it->second.total);
    std::fflush(g_trace);
  }
  g_live.erase(it);
}

// ---- DRHIP_ALLOC=cache: a caching allocator over hipMalloc.  A freed
// block stays allocated -- its virtual-to-physical mapping never changes --
// and is handed out again, whole, for a request of the same size class once
// the fences recorded at its free (every segment stream, the NULL stream)
// have completed.  A container re-created in a loop gets its memory back
// without a driver call and without the device-wide synchronisation of
// hipFree.  Size classes: powers of two from 512 B below 1 MiB, multiples
// of 2 MiB above.  hipMalloc failing for lack of memory releases the cache
// (after draining the streams) and retries once.
static std::vector<hipEvent_t> g_evpool[256];
static size_t size_class(size_t b) {
  if (b >= (size_t(1) << 20)) return (b + (size_t(2) << 20) - 1) & ~((size_t(2) << 20) - 1);
  size_t c = 512;
  while (c < b) c <<= 1;
  return c;
}
static int ev_get(int dev, hipEvent_t *e) {
  auto &v = g_evpool[dev & 255];
  if (!v.empty()) {
    *e = v.back();
    v.pop_back();
    return DRHIP_OK;
  }
  DRHIP_CHECK_HIP(hipSetDevice(dev));
  DRHIP_CHECK_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
  return DRHIP_OK;
}
// a cached block of class cls whose fences have all completed (nullptr if
// none), the most recently freed first (its lines and translations are the
// likeliest still cached)
static void *cache_take(Segment *s, size_t cls) {
  for (size_t i = s->cached.size(); i-- > 0;) {
    auto &c = s->cached[i];
    if (c.cls != cls) continue;
    bool done = true;
    for (auto &f : c.fences)
      if (hipEventQuery(f.second) != hipSuccess) {
        (void)hipGetLastError();
        done = false;
        break;
      }
    if (!done) continue;
    void *p = c.base;
    for (auto &f : c.fences) g_evpool[f.first & 255].push_back(f.second);
    s->cached_bytes -= c.cls;
    s->cached.erase(s->cached.begin() + (std::ptrdiff_t)i);
    return p;
  }
  return nullptr;
}
// every cached block of every segment on `dev` (all < 0) back to the driver,
// after the streams that may still use them
static void cache_release(int dev) {
  for (auto &o : g_segs)
    if (o.stream) {
      (void)hipSetDevice(o.device);
      (void)hipStreamSynchronize(o.stream);
    }
  for (auto &o : g_segs) {
    if (dev >= 0 && o.device != dev) continue;
    (void)hipSetDevice(o.device);
    for (auto &c : o.cached) {
      (void)hipFree(c.base);
      for (auto &f : c.fences) g_evpool[f.first & 255].push_back(f.second);
    }
    o.cached.clear();
    o.cached_bytes = 0;
  }
}
static int cache_put(Segment *s, void *base, size_t cls) {
  Segment::Cached c;
  c.base = base;
  c.cls = cls;
  for (auto &o : g_segs) {
    hipEvent_t e;
    if (int rc = ev_get(o.device, &e)) return rc;
    DRHIP_CHECK_HIP(hipSetDevice(o.device));
    DRHIP_CHECK_HIP(hipEventRecord(e, o.stream));
    c.fences.push_back({o.device, e});
  }
  hipEvent_t e;
  if (int rc = ev_get(s->device, &e)) return rc;
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  DRHIP_CHECK_HIP(hipEventRecord(e, nullptr));
  c.fences.push_back({s->device, e});
  s->cached.push_back(std::move(c));
  s->cached_bytes += cls;
  return DRHIP_OK;
}

// Guard mode: both red zones of a drhip_malloc block still hold kGuardWord
// (read after the work queued on the segment's stream).
static int guard_check(Segment *s, uintptr_t base, const LiveRec &r, const char *when) {
  static thread_local std::vector<unsigned> h;
  h.resize(2 * kGuard / 4);
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  DRHIP_CHECK_HIP(hipMemcpyAsync(h.data(), (void *)base, kGuard, hipMemcpyDeviceToHost, s->stream));
  // the zone after the block starts at its size rounded up to 4 B
  const size_t tail = (r.bytes + 3) & ~size_t(3);
  DRHIP_CHECK_HIP(hipMemcpyAsync(h.data() + kGuard / 4, (void *)(r.user + tail), kGuard - (tail - r.bytes),
                                 hipMemcpyDeviceToHost, s->stream));
  for (size_t i = kGuard / 4 + (kGuard - (tail - r.bytes)) / 4; i < h.size(); i++) h[i] = kGuardWord;
  DRHIP_CHECK_HIP(hipStreamSynchronize(s->stream));
  for (size_t i = 0; i < h.size(); i++)
    if (h[i] != kGuardWord) {
      const bool front = i < kGuard / 4;
      const size_t off = front ? kGuard - 4 * i : 4 * (i - kGuard / 4);
      char msg[384];
      std::snprintf(msg, sizeof msg,
                    "guard: %s, red zone of block %p (%zu B, segment %d, allocation #%llu) overwritten %zu B %s it "
                    "(0x%08x)",
                    when, (void *)r.user, r.bytes, r.seg, r.serial, off, front ? "before" : "after", h[i]);
      std::fprintf(stderr, "drhip: %s\n", msg);
      return set_error(DRHIP_ERR_ALLOC, msg);
    }
  return DRHIP_OK;
}

int may_reallocate(Segment *s, const char *what) {
  if (s->capturing)
    return set_error(DRHIP_ERR_UNSUPPORTED, (std::string(what) + " must grow during a graph capture: make one eager "
                                             "call at the largest size before drhip_graph_begin").c_str());
  if (s->live_graphs > 0)
    return set_error(DRHIP_ERR_UNSUPPORTED, (std::string(what) + " must grow while a captured graph of this segment "
                                             "is alive (it holds the buffer): drhip_graph_destroy it first, or warm "
                                             "up at the largest size before capturing").c_str());
  return DRHIP_OK;
}

// Replace a segment-internal buffer (workspace, tile prefixes) by one of
// nb bytes: hipFreeAsync / hipMallocAsync on the segment's stream with the
// pool, otherwise a stream drain + hipFree / hipMalloc.
int seg_realloc(Segment *s, void **p, size_t nb) {
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  const int seg = (int)(s - g_segs.data());
  const char kind = p == &s->ws ? 'w' : 't';
  if (*p) {
    if (s->pool) DRHIP_CHECK_HIP(hipFreeAsync(*p, s->stream));
    else {
      DRHIP_CHECK_HIP(hipStreamSynchronize(s->stream));
      DRHIP_CHECK_HIP(hipFree(*p));
    }
    alloc_untrack((uintptr_t)*p);
  }
  *p = nullptr;
  void *q = nullptr;
  if (s->pool) DRHIP_CHECK_HIP(hipMallocAsync(&q, nb, s->stream));
  else DRHIP_CHECK_HIP(hipMalloc(&q, nb));
  if (int rc = alloc_track(seg, kind, q, nb, nb, q)) return rc; // q stays out of circulation
  *p = q;
  return DRHIP_OK;
}

int ensure_workspace(int seg, size_t bytes) {
  Segment *s = segment(seg);
  if (!s) return set_error(DRHIP_ERR_BAD_SEG, "bad segment");
  if (s->ws_bytes >= bytes) return DRHIP_OK;
  if (int rc = may_reallocate(s, "the segment workspace")) return rc;
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  // the old buffer goes after the kernels already queued on this stream
  // that use it (stream-ordered with the pool, a drained stream otherwise)
  size_t nb = bytes < (size_t(1) << 20) ? (size_t(1) << 20) : bytes;
  nb = (nb + 4095) & ~size_t(4095);
  if (int rc = seg_realloc(s, &s->ws, nb)) return rc;
  s->ws_bytes = nb;
  return DRHIP_OK;
}

} // namespace drhip

using namespace drhip;

extern "C" {

const char *drhip_last_error(void) { return g_err.c_str(); }
const char *drhip_version(void) { return "drhip 0.1 (gfx950)"; }

int drhip_device_count(int *count) {
  if (!count) return set_error(DRHIP_ERR_BAD_ARG, "null count");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    *count = 0;
    return set_hip_error(e, "hipGetDeviceCount");
  }
  *count = n;
  return DRHIP_OK;
}

int drhip_finalize(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  int rc = DRHIP_OK;
  // every segment stream drained first: a stream may still read another
  // segment's memory (peer copies, misaligned scan pieces)
  for (auto &s : g_segs)
    if (s.stream && (hipSetDevice(s.device) != hipSuccess || hipStreamSynchronize(s.stream) != hipSuccess))
      rc = DRHIP_ERR_HIP;
  // Blocks still live are released here (a container must not outlive
  // finalize / re-init: its later drhip_free is refused as not live).
  {
    std::lock_guard<std::mutex> lk2(g_live_mu);
    for (auto &kv : g_live) {
      Segment &s = g_segs[kv.second.seg];
      (void)hipSetDevice(s.device);
      (void)(s.pool ? hipFreeAsync((void *)kv.first, s.stream) : hipFree((void *)kv.first));
    }
    g_live.clear();
  }
  cache_release(-1);
  for (auto &v : g_evpool) {
    for (auto e : v) (void)hipEventDestroy(e);
    v.clear();
  }
  for (auto &s : g_segs) {
    if (hipSetDevice(s.device) != hipSuccess) rc = DRHIP_ERR_HIP;
    if (s.stream) {
      (void)hipStreamSynchronize(s.stream);
      (void)hipStreamDestroy(s.stream);
    }
    s.ws = s.tiles = nullptr;
    if (s.fence) (void)hipEventDestroy(s.fence);
    if (s.null_fence) (void)hipEventDestroy(s.null_fence);
    if (s.err) (void)hipHostFree(s.err);
    if (s.stage) (void)hipHostFree(s.stage);
    if (s.dsync) (void)hipFree(s.dsync);
    if (s.thash) (void)hipFree(s.thash);
    comm_release(s);
  }
  // private pools last: every block of theirs has been released above
  for (auto &s : g_segs)
    if (s.own_pool) {
      (void)hipSetDevice(s.device);
      (void)hipDeviceSynchronize();
      (void)hipMemPoolDestroy(s.own_pool);
    }
  for (int d = 0; d < 256; d++)
    if (g_lane[d]) {
      (void)hipEventDestroy(g_lane[d]);
      g_lane[d] = nullptr;
      g_lane_used[d] = false;
    }
  // hand the pools' cached blocks back to the driver
  for (auto &s : g_segs) {
    hipMemPool_t pool;
    if (hipSetDevice(s.device) == hipSuccess && hipDeviceGetDefaultMemPool(&pool, s.device) == hipSuccess)
      (void)hipMemPoolTrimTo(pool, 0);
  }
  g_segs.clear();
  g_graphs.clear();
  if (g_trace) {
    std::fclose(g_trace);
    g_trace = nullptr;
  }
  return rc;
}

static int init_locked(const int *dev_ids, int nsegs);

int drhip_init(const int *dev_ids, int nsegs) {
  if (!dev_ids || nsegs <= 0) return set_error(DRHIP_ERR_BAD_ARG, "drhip_init: empty device list");
  if (!g_segs.empty()) drhip_finalize();
  int ndev = 0;
  int rc = drhip_device_count(&ndev);
  if (rc != DRHIP_OK) return rc;
  if (ndev == 0) return set_error(DRHIP_ERR_NO_DEVICE, "no HIP device visible");
  for (int i = 0; i < nsegs; i++)
    if (dev_ids[i] < 0 || dev_ids[i] >= ndev)
      return set_error(DRHIP_ERR_BAD_ARG, "drhip_init: device id out of range");
  {
    std::lock_guard<std::mutex> lk(g_mu);
    rc = init_locked(dev_ids, nsegs);
  }
  if (rc != DRHIP_OK) {
    // no half-built registry: release what was created, keep the error text
    const std::string why = g_err;
    (void)drhip_finalize();
    g_err = why;
  }
  return rc;
}

static int init_locked(const int *dev_ids, int nsegs) {
  // How a blocking wait (drhip_sync, every blocking shp:: call) waits for
  // the GPU: DRHIP_SYNC=spin (default: the host thread polls, lowest
  // latency for the reference's blocking API), yield, blocking (interrupt),
  // auto (the runtime's heuristic).  A device whose flags cannot be changed
  // any more (another library initialised it first, e.g. torch) keeps its
  // own; the call's error is ignored.
  {
    const char *sm = getenv("DRHIP_SYNC");
    unsigned fl = hipDeviceScheduleSpin;
    if (sm && !strcmp(sm, "yield")) fl = hipDeviceScheduleYield;
    else if (sm && !strcmp(sm, "blocking")) fl = hipDeviceScheduleBlockingSync;
    else if (sm && !strcmp(sm, "auto")) fl = hipDeviceScheduleAuto;
    for (int i = 0; i < nsegs; i++) {
      if (hipSetDevice(dev_ids[i]) == hipSuccess) (void)hipSetDeviceFlags(fl);
      (void)hipGetLastError();
    }
  }
  g_segs.resize(nsegs);
  for (int i = 0; i < nsegs; i++) {
    Segment &s = g_segs[i];
    s.device = dev_ids[i];
    DRHIP_CHECK_HIP(hipSetDevice(s.device));
    DRHIP_CHECK_HIP(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
    DRHIP_CHECK_HIP(hipEventCreateWithFlags(&s.fence, hipEventDisableTiming));
    // Segment memory comes from the device's stream-ordered pool; freed
    // blocks stay cached in the pool (no release threshold), so a container
    // re-created in a loop reuses its HBM without a driver call.
    hipMemPool_t pool;
    DRHIP_CHECK_HIP(hipDeviceGetDefaultMemPool(&pool, s.device));
    uint64_t keep = UINT64_MAX;
    DRHIP_CHECK_HIP(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep));
    hipDeviceProp_t prop;
    DRHIP_CHECK_HIP(hipGetDeviceProperties(&prop, s.device));
    s.num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    // Segment memory (drhip_malloc): by default the caching allocator over
    // hipMalloc (DRHIP_ALLOC=cache, cache_take / cache_put above);
    // DRHIP_ALLOC=hipmalloc plain hipMalloc / hipFree; DRHIP_ALLOC=pool the
    // device's stream-ordered pool (hipMallocAsync), which round 6 showed
    // handing out blocks whose contents a kernel and a copy engine see
    // differently (profiles/r06_pool_diagnosis.txt, reproduced without this
    // library by tools/pool_tlb_repro.hip): diagnosis only.
    const char *alloc = getenv("DRHIP_ALLOC");
    if (i == 0) {
      const char *g = getenv("DRHIP_ALLOC_GUARD");
      g_guard = g && g[0] == '1';
      const char *tr = getenv("DRHIP_ALLOC_TRACE");
      if (tr && tr[0] && !g_trace) {
        g_trace = std::fopen(tr, "a");
        if (g_trace) std::fprintf(g_trace, "I %d %s\n", nsegs, alloc ? alloc : "hipmalloc");
      }
    }
    s.pool = alloc && !strcmp(alloc, "pool");
    if (s.pool && i == 0)
      std::fprintf(stderr, "drhip: WARNING: DRHIP_ALLOC=pool selects the stream-ordered pool, which hands out blocks "
                           "a kernel and a copy engine see differently on this runtime "
                           "(profiles/r06_pool_diagnosis.txt); for diagnosis only, do not use it for results\n");
    s.cache =!alloc || !alloc[0] || !strcmp(alloc, "cache"); // the default; DRHIP_ALLOC=hipmalloc: plain
    if (s.pool) {
      // pool variants, for the round-5 pool stress (profiles/r05_pool_stress.txt):
      // DRHIP_POOL=private -> a pool of the segment's own; =noreuse -> the
      // default pool without cross-stream / opportunistic reuse
      const char *pm = getenv("DRHIP_POOL");
      if (pm && !strcmp(pm, "private")) {
        hipMemPoolProps props = {};
        props.allocType = hipMemAllocationTypePinned;
        props.location.type = hipMemLocationTypeDevice;
        props.location.id = s.device;
        DRHIP_CHECK_HIP(hipMemPoolCreate(&s.own_pool, &props));
        DRHIP_CHECK_HIP(hipMemPoolSetAttribute(s.own_pool, hipMemPoolAttrReleaseThreshold, &keep));
      } else if (pm && !strcmp(pm, "noreuse")) {
        int off = 0;
        DRHIP_CHECK_HIP(hipMemPoolSetAttribute(pool, hipMemPoolReuseFollowEventDependencies, &off));
        DRHIP_CHECK_HIP(hipMemPoolSetAttribute(pool, hipMemPoolReuseAllowOpportunistic, &off));
        DRHIP_CHECK_HIP(hipMemPoolSetAttribute(pool, hipMemPoolReuseAllowInternalDependencies, &off));
      }
    }
    // Error word in pinned, device-mapped host memory: a timed-out in-kernel
    // spin stores to it, drhip_sync reads it with a plain host load.
    DRHIP_CHECK_HIP(hipHostMalloc((void **)&s.err, 256, hipHostMallocMapped | hipHostMallocPortable));
    memset(s.err, 0, 256);
    DRHIP_CHECK_HIP(hipMalloc((void **)&s.dsync, kSyncWords * sizeof(unsigned)));
    DRHIP_CHECK_HIP(hipMemsetAsync(s.dsync, 0, kSyncWords * sizeof(unsigned), s.stream));
    {
      const char *ct = getenv("DRHIP_CHECK_TILES");
      s.check_tiles = ct && ct[0] == '1';
      if (s.check_tiles) DRHIP_CHECK_HIP(hipMalloc((void **)&s.thash, 256));
    }
  }
  // Peer access between distinct devices (xGMI): cross-segment reads/writes
  // (misaligned zipped scan pieces, gemv x replication, halo copies).
  for (int i = 0; i < nsegs; i++)
    for (int j = 0; j < nsegs; j++) {
      int a = g_segs[i].device, b = g_segs[j].device;
      if (a == b) continue;
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, a, b) == hipSuccess && can) {
        (void)hipSetDevice(a);
        hipError_t e = hipDeviceEnablePeerAccess(b, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
          return set_hip_error(e, "hipDeviceEnablePeerAccess");
        }
        (void)hipGetLastError();
        // pool allocations are not covered by peer access: device a may
        // read and write b's pool memory too
        hipMemPool_t pool_b;
        DRHIP_CHECK_HIP(hipDeviceGetDefaultMemPool(&pool_b, b));
        hipMemAccessDesc acc = {};
        acc.location.type = hipMemLocationTypeDevice;
        acc.location.id = a;
        acc.flags = hipMemAccessFlagsProtReadWrite;
        DRHIP_CHECK_HIP(hipMemPoolSetAccess(pool_b, &acc, 1));
      }
    }
  for (auto &s : g_segs) {
    DRHIP_CHECK_HIP(hipSetDevice(s.device));
    DRHIP_CHECK_HIP(hipStreamSynchronize(s.stream));
  }
  g_err = "ok";
  return DRHIP_OK;
}

int drhip_nprocs(int *nsegs) {
  if (!nsegs) return set_error(DRHIP_ERR_BAD_ARG, "null");
  *nsegs = (int)g_segs.size();
  return DRHIP_OK;
}

int drhip_device_of(int seg, int *dev_id) {
  DRHIP_GET_SEG(s, seg);
  if (!dev_id) return set_error(DRHIP_ERR_BAD_ARG, "null");
  *dev_id = s->device;
  return DRHIP_OK;
}

int drhip_stream(int seg, void **hip_stream) {
  DRHIP_GET_SEG(s, seg);
  if (!hip_stream) return set_error(DRHIP_ERR_BAD_ARG, "null");
  *hip_stream = (void *)s->stream;
  return DRHIP_OK;
}

int drhip_sync(int seg) {
  DRHIP_GET_SEG(s, seg);
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  DRHIP_CHECK_HIP(hipStreamSynchronize(s->stream));
  if (g_guard) {
    std::vector<std::pair<uintptr_t, LiveRec>> mine;
    {
      std::lock_guard<std::mutex> lk(g_live_mu);
      for (auto &kv : g_live)
        if (kv.second.seg == seg && kv.second.kind == 'u') mine.push_back(kv);
    }
    for (auto &kv : mine)
      if (int rc = guard_check(s, kv.first, kv.second, "at drhip_sync")) return rc;
  }
  unsigned err = __atomic_load_n(s->err, __ATOMIC_ACQUIRE);
  if (err) {
    __atomic_store_n(s->err, 0u, __ATOMIC_RELEASE);
    if (err == 4)
      return set_error(DRHIP_ERR_BAD_ARG, "drhip_inclusive_scan_tiles: the range changed since its drhip_reduce_tiles "
                                          "(DRHIP_CHECK_TILES)");
    return set_error(DRHIP_ERR_TIMEOUT, "an in-kernel bounded spin timed out");
  }
  return DRHIP_OK;
}

int drhip_graph_begin(int seg) {
  DRHIP_GET_SEG(s, seg);
  if (s->capturing) return set_error(DRHIP_ERR_BAD_ARG, "drhip_graph_begin: a capture is already open on seg");
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  // thread-local: other host threads' unrelated HIP calls do not break it
  DRHIP_CHECK_HIP(hipStreamBeginCapture(s->stream, hipStreamCaptureModeThreadLocal));
  s->capturing = true;
  s->cap_tiles = false;
  s->tr_before = s->tr;
  return DRHIP_OK;
}

int drhip_graph_end(int seg, void **graph_exec) {
  DRHIP_GET_SEG(s, seg);
  if (!graph_exec) return set_error(DRHIP_ERR_BAD_ARG, "drhip_graph_end: null");
  *graph_exec = nullptr;
  if (!s->capturing) return set_error(DRHIP_ERR_BAD_ARG, "drhip_graph_end: no capture open on seg");
  s->capturing = false;
  // nothing captured has run: the prefixes in the buffer are still those of
  // the range before the capture
  s->tr = s->tr_before;
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  hipGraph_t g = nullptr;
  DRHIP_CHECK_HIP(hipStreamEndCapture(s->stream, &g));
  hipGraphExec_t ex = nullptr;
  const hipError_t e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (e != hipSuccess) return set_hip_error(e, "hipGraphInstantiate");
  {
    std::lock_guard<std::mutex> lk(g_mu);
    g_graphs[(void *)ex] = GraphRec{seg, s->cap_tiles, s->tr_captured};
  }
  s->live_graphs++;
  *graph_exec = (void *)ex;
  return DRHIP_OK;
}

int drhip_graph_launch(int seg, void *graph_exec) {
  DRHIP_GET_SEG(s, seg);
  if (!graph_exec) return set_error(DRHIP_ERR_BAD_ARG, "drhip_graph_launch: null");
  GraphRec rec;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_graphs.find(graph_exec);
    if (it == g_graphs.end()) return set_error(DRHIP_ERR_BAD_ARG, "drhip_graph_launch: not a live drhip graph");
    rec = it->second;
  }
  if (rec.seg != seg) return set_error(DRHIP_ERR_BAD_ARG, "drhip_graph_launch: graph captured on another segment");
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  DRHIP_CHECK_HIP(hipGraphLaunch((hipGraphExec_t)graph_exec, s->stream));
  // a replayed drhip_reduce_tiles leaves the prefixes of its captured range
  if (rec.has_tiles) s->tr = rec.tiles;
  return DRHIP_OK;
}

int drhip_graph_destroy(void *graph_exec) {
  if (!graph_exec) return DRHIP_OK;
  int seg = -1;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_graphs.find(graph_exec);
    if (it != g_graphs.end()) {
      seg = it->second.seg;
      g_graphs.erase(it);
    }
  }
  // the registry entry is gone either way: the segment's buffers may grow
  // again even if the runtime refuses the destroy below
  if (Segment *s = segment(seg))
    if (s->live_graphs > 0) s->live_graphs--;
  DRHIP_CHECK_HIP(hipGraphExecDestroy((hipGraphExec_t)graph_exec));
  return DRHIP_OK;
}

int drhip_sync_all(void) {
  int rc = DRHIP_OK;
  for (int i = 0; i < (int)g_segs.size(); i++) {
    int r = drhip_sync(i);
    if (r != DRHIP_OK) rc = r;
  }
  return rc;
}

// drhip_free of a pointer that is not a live drhip_malloc block (a double
// free, or a pointer from elsewhere) is refused with DRHIP_ERR_BAD_ARG
// instead of reaching the allocator, where it could release a block that
// another container has been handed since.

int drhip_malloc(int seg, size_t bytes, void **ptr) {
  DRHIP_GET_SEG(s, seg);
  if (!ptr) return set_error(DRHIP_ERR_BAD_ARG, "null");
  *ptr = nullptr;
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  if (bytes == 0) bytes = 16;
  const size_t total = g_guard ? bytes + 2 * kGuard : bytes;
  void *base = nullptr;
  size_t reserved = total;
  if (s->cache) {
    reserved = size_class(total);
    base = cache_take(s, reserved);
    if (!base) {
      hipError_t e = hipMalloc(&base, reserved);
      if (e == hipErrorOutOfMemory) {
        (void)hipGetLastError();
        cache_release(s->device);
        DRHIP_CHECK_HIP(hipSetDevice(s->device));
        e = hipMalloc(&base, reserved);
      }
      if (e != hipSuccess) return set_hip_error(e, "hipMalloc");
    }
  } else if (!s->pool) {
    DRHIP_CHECK_HIP(hipMalloc(&base, total));
  } else {
    // Stream-ordered pool allocation on the segment's stream (the north
    // star's hipMallocAsync-backed segment allocator; a block freed earlier
    // is reused without a driver call).  Returned like the reference's
    // blocking USM allocation (allocators.hpp:45-57): the stream is drained,
    // so the block is valid for every stream and peer device.
    if (s->own_pool) DRHIP_CHECK_HIP(hipMallocFromPoolAsync(&base, total, s->own_pool, s->stream));
    else DRHIP_CHECK_HIP(hipMallocAsync(&base, total, s->stream));
  }
  void *user = g_guard ? static_cast<char *>(base) + kGuard : base;
  if (g_guard) {
    const size_t tail = (bytes + 3) & ~size_t(3); // the zone after the block starts at a 4-B boundary
    DRHIP_CHECK_HIP(hipMemsetD32Async((hipDeviceptr_t)base, kGuardWord, kGuard / 4, s->stream));
    DRHIP_CHECK_HIP(hipMemsetD32Async((hipDeviceptr_t)(static_cast<char *>(user) + tail), kGuardWord,
                                      (kGuard - (tail - bytes)) / 4, s->stream));
  }
  if (s->pool || g_guard) DRHIP_CHECK_HIP(hipStreamSynchronize(s->stream));
  if (int rc = alloc_track(seg, 'u', base, reserved, bytes, user)) return rc; // base stays out of circulation
  *ptr = user;
  return DRHIP_OK;
}

int drhip_free(int seg, void *ptr) {
  DRHIP_GET_SEG(s0, seg);
  if (!ptr) return DRHIP_OK;
  uintptr_t base = 0;
  LiveRec rec;
  if (!alloc_find(ptr, &base, &rec) || rec.kind != 'u') {
    std::fprintf(stderr, "drhip_free: %p is not a live drhip_malloc block (double free?)\n", ptr);
    return set_error(DRHIP_ERR_BAD_ARG, "drhip_free: not a live drhip_malloc block (double free?)");
  }
  // the block goes back through the segment that allocated it (its stream,
  // its pool), whichever segment the caller named
  Segment *s = segment(rec.seg);
  (void)s0;
  if (g_guard)
    if (int rc = guard_check(s, base, rec, "at drhip_free")) return rc;
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  if (s->cache) {
    // into the segment's cache behind fences on every stream: no host sync
    if (int rc = cache_put(s, (void *)base, rec.total)) return rc;
    alloc_untrack(base);
    return DRHIP_OK;
  }
  if (!s->pool) {
    // after the work queued on EVERY segment stream (peer reads of this
    // memory included): hipFree alone waits for this device only
    for (auto &o : g_segs) {
      DRHIP_CHECK_HIP(hipSetDevice(o.device));
      DRHIP_CHECK_HIP(hipStreamSynchronize(o.stream));
    }
    DRHIP_CHECK_HIP(hipSetDevice(s->device));
    DRHIP_CHECK_HIP(hipFree((void *)base)); // synchronises the device
    alloc_untrack(base);
    return DRHIP_OK;
  }
  // The block returns to the pool after the work already queued on EVERY
  // segment's stream (peer reads of this memory included) and on the
  // device's NULL stream: seg's stream waits on a fence recorded on each of
  // them, then frees in order.  No host synchronisation.  Work the caller
  // queued on OTHER streams of its own (e.g. a torch side stream) is not
  // fenced: drain those before freeing memory they use, or select
  // the default allocator (hipFree synchronises the device).
  for (auto &o : g_segs) {
    if (&o == s) continue;
    DRHIP_CHECK_HIP(hipSetDevice(o.device));
    DRHIP_CHECK_HIP(hipEventRecord(o.fence, o.stream));
    DRHIP_CHECK_HIP(hipSetDevice(s->device));
    DRHIP_CHECK_HIP(hipStreamWaitEvent(s->stream, o.fence, 0));
  }
  if (!s->null_fence) DRHIP_CHECK_HIP(hipEventCreateWithFlags(&s->null_fence, hipEventDisableTiming));
  DRHIP_CHECK_HIP(hipEventRecord(s->null_fence, nullptr));
  DRHIP_CHECK_HIP(hipStreamWaitEvent(s->stream, s->null_fence, 0));
  DRHIP_CHECK_HIP(hipFreeAsync((void *)base, s->stream));
  alloc_untrack(base);
  return DRHIP_OK;
}

int drhip_host_alloc(size_t bytes, void **ptr) {
  if (!ptr) return set_error(DRHIP_ERR_BAD_ARG, "null");
  DRHIP_CHECK_HIP(hipHostMalloc(ptr, bytes ? bytes : 16, hipHostMallocPortable | hipHostMallocMapped));
  return DRHIP_OK;
}

int drhip_host_free(void *ptr) {
  if (!ptr) return DRHIP_OK;
  DRHIP_CHECK_HIP(hipHostFree(ptr));
  return DRHIP_OK;
}

// True for host memory the HIP runtime does not know (plain malloc/new,
// numpy buffers): pageable, so an "async" copy cannot be stream-ordered.
static bool is_pageable(const void *p) {
  hipPointerAttribute_t attr;
  hipError_t e = hipPointerGetAttributes(&attr, p);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return true;
  }
  return attr.type == hipMemoryTypeUnregistered;
}

// DRHIP_COPY=staged (diagnosis, round 5): a pageable copy chunked through
// the segment's pinned 64 MiB buffer, each chunk an async copy on the
// segment's stream; the strongest amplifier of the pool's zero pages
// (profiles/r05_pool_stress.txt), 0 failures on hipMalloc'd memory.
static int copy_staged(Segment *s, void *dst, const void *src, size_t bytes, hipMemcpyKind kind) {
  constexpr size_t kChunk = size_t(64) << 20;
  if (!s->stage) {
    DRHIP_CHECK_HIP(hipHostMalloc(&s->stage, kChunk, hipHostMallocPortable));
    s->stage_bytes = kChunk;
  }
  for (size_t off = 0; off < bytes; off += kChunk) {
    const size_t len = bytes - off < kChunk ? bytes - off : kChunk;
    DRHIP_CHECK_HIP(hipStreamSynchronize(s->stream)); // the stage is free
    if (kind == hipMemcpyHostToDevice) {
      memcpy(s->stage, static_cast<const char *>(src) + off, len);
      DRHIP_CHECK_HIP(hipMemcpyAsync(static_cast<char *>(dst) + off, s->stage, len, kind, s->stream));
    } else {
      DRHIP_CHECK_HIP(hipMemcpyAsync(s->stage, static_cast<const char *>(src) + off, len, kind, s->stream));
      DRHIP_CHECK_HIP(hipStreamSynchronize(s->stream));
      memcpy(static_cast<char *>(dst) + off, s->stage, len);
    }
  }
  DRHIP_CHECK_HIP(hipStreamSynchronize(s->stream));
  return DRHIP_OK;
}

static int copy_async(int seg, void *dst, const void *src, size_t bytes, hipMemcpyKind kind) {
  DRHIP_GET_SEG(s, seg);
  if (bytes == 0) return DRHIP_OK;
  if (!dst || !src) return set_error(DRHIP_ERR_BAD_ARG, "null pointer");
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  const void *host = kind == hipMemcpyHostToDevice ? src : kind == hipMemcpyDeviceToHost ? dst : nullptr;
  if (host && is_pageable(host)) {
    // Pageable host buffer (the std::vector side of shp::copy,
    // copy.hpp:19-60): the copy goes on the segment's stream, ordered after
    // every kernel already queued there (the runtime stages it), and the
    // call blocks until it has landed, like copy().
    static const bool staged = [] {
      const char *e = getenv("DRHIP_COPY");
      return e && !strcmp(e, "staged");
    }();
    if (staged) return copy_staged(s, dst, src, bytes, kind);
    DRHIP_CHECK_HIP(hipMemcpyAsync(dst, src, bytes, kind, s->stream));
    DRHIP_CHECK_HIP(hipStreamSynchronize(s->stream));
    return DRHIP_OK;
  }
  DRHIP_CHECK_HIP(hipMemcpyAsync(dst, src, bytes, kind, s->stream));
  return DRHIP_OK;
}

int drhip_memcpy_h2d(int seg, void *dst, const void *src, size_t bytes) {
  return copy_async(seg, dst, src, bytes, hipMemcpyHostToDevice);
}
int drhip_memcpy_d2h(int seg, void *dst, const void *src, size_t bytes) {
  return copy_async(seg, dst, src, bytes, hipMemcpyDeviceToHost);
}
int drhip_memcpy_d2d(int seg, void *dst, const void *src, size_t bytes) {
  // hipMemcpyDefault: unified addressing resolves same-device vs peer (xGMI).
  return copy_async(seg, dst, src, bytes, hipMemcpyDefault);
}

} // extern "C"
