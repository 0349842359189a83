// pool_replay.hip -- standalone replay of a libdrhip allocation trace
// (DRHIP_ALLOC_TRACE, csrc/runtime.hip alloc_track) on the device's
// stream-ordered pool, WITHOUT libdrhip: the same hipMallocAsync /
// hipFreeAsync sequence, sizes and per-segment streams, with every new block
// checked against the blocks still live.  If the pool hands out a block that
// overlaps a live one here, the overlap is the runtime's, not this library's.
//
//   hipcc -O2 --offload-arch=gfx950 tools/pool_replay.hip -o tools/pool_replay
//   tools/pool_replay TRACE [--touch] [--spin-us N] [--reps R]
//
// --touch: memset every new block (the library writes what it allocates);
// --spin-us N: a spinning kernel of ~N us on the stream before every free,
// so frees are still pending when the next allocation comes (as behind the
// library's kernels); --reps: replay the trace R times in one process.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                \
    }                                                                              \
  } while (0)

__global__ void spin_kernel(long long cycles) {
  const long long t0 = clock64();
  while (clock64() - t0 < cycles) {
  }
}

struct Op {
  char what;  // 'M' or 'F'
  unsigned long long serial;
  int seg;
  char kind;
  size_t total;
};

int main(int argc, char **argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s TRACE [--touch] [--spin-us N] [--reps R]\n", argv[0]);
    return 2;
  }
  bool touch = false;
  long spin_us = 0;
  int reps = 1;
  for (int i = 2; i < argc; i++) {
    if (!strcmp(argv[i], "--touch")) touch = true;
    else if (!strcmp(argv[i], "--spin-us") && i + 1 < argc) spin_us = atol(argv[++i]);
    else if (!strcmp(argv[i], "--reps") && i + 1 < argc) reps = atoi(argv[++i]);
  }
  FILE *f = std::fopen(argv[1], "r");
  if (!f) {
    std::perror(argv[1]);
    return 2;
  }
  std::vector<Op> ops;
  int nsegs = 1;
  char line[512];
  while (std::fgets(line, sizeof line, f)) {
    Op o{};
    unsigned long long base;
    if (line[0] == 'I') {
      if (!ops.empty()) break; // the first process's trace only
      std::sscanf(line + 2, "%d", &nsegs);
      continue;
    }
    if ((line[0] == 'M' || line[0] == 'F') &&
        std::sscanf(line + 2, "%llu %d %c %llx %zu", &o.serial, &o.seg, &o.kind, &base, &o.total) == 5) {
      o.what = line[0];
      ops.push_back(o);
    }
  }
  std::fclose(f);
  std::printf("trace: %zu operations over %d segments\n", ops.size(), nsegs);
  CK(hipSetDevice(0));
  hipMemPool_t pool;
  CK(hipDeviceGetDefaultMemPool(&pool, 0));
  uint64_t keep = UINT64_MAX;
  CK(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep));
  std::vector<hipStream_t> st(nsegs);
  for (auto &s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int clock_khz = 0;
  CK(hipDeviceGetAttribute(&clock_khz, hipDeviceAttributeClockRate, 0));
  const long long spin_cycles = (long long)spin_us * clock_khz / 1000;
  long overlaps = 0;
  for (int rep = 0; rep < reps; rep++) {
    std::unordered_map<unsigned long long, std::pair<uintptr_t, size_t>> bySerial;
    std::map<uintptr_t, std::pair<size_t, unsigned long long>> live;
    for (const Op &o : ops) {
      hipStream_t s = st[o.seg % nsegs];
      if (o.what == 'M') {
        void *p = nullptr;
        CK(hipMallocAsync(&p, o.total, s));
        if (touch) CK(hipMemsetAsync(p, 0x5a, o.total, s));
        if (o.kind == 'u') CK(hipStreamSynchronize(s)); // drhip_malloc drains its stream
        const uintptr_t b = (uintptr_t)p, e = b + o.total;
        auto it = live.upper_bound(b);
        bool hit = false;
        uintptr_t hb = 0;
        size_t ht = 0;
        unsigned long long hs = 0;
        if (it != live.begin()) {
          auto q = std::prev(it);
          if (q->first + q->second.first > b) hit = true, hb = q->first, ht = q->second.first, hs = q->second.second;
        }
        if (!hit && it != live.end() && it->first < e)
          hit = true, hb = it->first, ht = it->second.first, hs = it->second.second;
        if (hit) {
          overlaps++;
          if (overlaps <= 10)
            std::printf("rep %d: OVERLAP: allocation #%llu [%p, %p) %zu B overlaps live #%llu [%p, %p) %zu B\n", rep,
                        o.serial, p, (void *)e, o.total, hs, (void *)hb, (void *)(hb + ht), ht);
          // keep it out of the live map (it is a second claim on those pages)
          bySerial[o.serial] = {0, 0};
          continue;
        }
        live[b] = {o.total, o.serial};
        bySerial[o.serial] = {b, o.total};
      } else {
        auto it = bySerial.find(o.serial);
        if (it == bySerial.end() || it->second.first == 0) continue;
        if (spin_cycles) hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, s, spin_cycles);
        CK(hipFreeAsync((void *)it->second.first, s));
        live.erase(it->second.first);
        bySerial.erase(it);
      }
    }
    for (auto &kv : live) CK(hipFreeAsync((void *)kv.first, st[0]));
    CK(hipDeviceSynchronize());
  }
  std::printf("replay: %d rep(s), %ld overlapping allocation(s)\n", reps, overlaps);
  return overlaps ? 1 : 0;
}
