// pool_tlb_repro.hip -- standalone reproducer (no libdrhip) of the round-5/6
// stream-ordered pool failure: after a pool block is filled by a
// host-to-device COPY, a KERNEL reading the same addresses sees other bytes
// (profiles/r06_pool_diagnosis.txt).
//
// Replays an allocation trace written by libdrhip (DRHIP_ALLOC_TRACE) with
// the same hipMallocAsync / hipFreeAsync sequence on one stream, and gives
// every block of >= 4 KiB the library's treatment of a distributed_vector
// filled from a std::vector (shp::copy with DRHIP_COPY=staged):
//   1. fill: the block's pattern (word i of allocation s = mix(s, i)) copied
//      in 64 MiB chunks through a pinned staging buffer (hipMemcpyAsync
//      host-to-device on the stream, drained per chunk);
//   2. kernel view: a kernel hashes the block (order-free sum of w_i (2i+1));
//   3. copy view: the block copied back (device-to-host) and compared;
//   4. before the block's free, the kernel view again.
// A block whose kernel view differs from its pattern while the copy view
// matches (or the reverse) has two engines translating one virtual address
// to different memory.
//
//   hipcc -O2 --offload-arch=gfx950 tools/pool_tlb_repro.hip -o tools/pool_tlb_repro
//   tools/pool_tlb_repro TRACE [--alloc pool|hipmalloc] [--reps R] [--fill copy|kernel]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unordered_map>
#include <vector>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
      std::exit(2);                                                                            \
    }                                                                                          \
  } while (0)

__host__ __device__ inline unsigned mix(unsigned long long s, unsigned long long i) {
  unsigned long long z = s * 0x9E3779B97F4A7C15ull + i + 0x632BE59BD9B4E019ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return (unsigned)((z ^ (z >> 31)) >> 16) | 1u; // never 0: a zero page shows
}

// the fill by a KERNEL instead of the copy engine (--fill kernel)
__global__ void fill_kernel(unsigned *p, size_t nw, unsigned long long s) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nw; i += (size_t)gridDim.x * blockDim.x)
    p[i] = mix(s, i);
}

__global__ void hash_kernel(const unsigned *p, size_t nw, unsigned long long *out) {
  unsigned long long acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nw; i += (size_t)gridDim.x * blockDim.x)
    acc += (unsigned long long)p[i] * (2ull * i + 1ull);
  atomicAdd(out, acc);
}

struct Op {
  char what;
  unsigned long long serial;
  char kind;
  size_t total;
};

int main(int argc, char **argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s TRACE [--alloc pool|hipmalloc] [--reps R]\n", argv[0]);
    return 2;
  }
  bool pool = true, kfill = false;
  int reps = 1;
  for (int i = 2; i + 1 < argc; i++) {
    if (!strcmp(argv[i], "--alloc")) pool = strcmp(argv[++i], "hipmalloc") != 0;
    else if (!strcmp(argv[i], "--reps")) reps = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--fill")) kfill = !strcmp(argv[++i], "kernel");
  }
  FILE *f = std::fopen(argv[1], "r");
  if (!f) {
    std::perror(argv[1]);
    return 2;
  }
  std::vector<Op> ops;
  char line[512];
  while (std::fgets(line, sizeof line, f)) {
    if (line[0] == 'I') {
      if (!ops.empty()) break;
      continue;
    }
    Op o{};
    int seg;
    unsigned long long base;
    if ((line[0] == 'M' || line[0] == 'F') &&
        std::sscanf(line + 2, "%llu %d %c %llx %zu", &o.serial, &seg, &o.kind, &base, &o.total) == 5) {
      o.what = line[0];
      ops.push_back(o);
    }
  }
  std::fclose(f);
  CK(hipSetDevice(0));
  hipMemPool_t mp;
  CK(hipDeviceGetDefaultMemPool(&mp, 0));
  uint64_t keep = UINT64_MAX;
  CK(hipMemPoolSetAttribute(mp, hipMemPoolAttrReleaseThreshold, &keep));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t null_fence;
  CK(hipEventCreateWithFlags(&null_fence, hipEventDisableTiming));
  constexpr size_t kChunk = size_t(64) << 20;
  void *stage = nullptr;
  CK(hipHostMalloc(&stage, kChunk, hipHostMallocPortable));
  unsigned long long *dhash = nullptr;
  CK(hipMalloc(&dhash, 8));
  std::vector<unsigned> host;
  long kernel_bad = 0, copy_bad = 0, checked = 0, later_bad = 0;
  auto kernel_hash = [&](const void *p, size_t bytes) {
    CK(hipMemsetAsync(dhash, 0, 8, st));
    hipLaunchKernelGGL(hash_kernel, dim3(1024), dim3(256), 0, st, (const unsigned *)p, bytes / 4, dhash);
    unsigned long long h = 0;
    CK(hipMemcpyAsync(&h, dhash, 8, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    return h;
  };
  for (int rep = 0; rep < reps; rep++) {
    std::unordered_map<unsigned long long, std::pair<void *, size_t>> live;
    std::unordered_map<unsigned long long, unsigned long long> want_hash;
    for (const Op &o : ops) {
      if (o.what == 'M') {
        void *p = nullptr;
        if (pool) CK(hipMallocAsync(&p, o.total, st));
        else CK(hipMalloc(&p, o.total));
        if (o.kind == 'u') CK(hipStreamSynchronize(st));
        live[o.serial] = {p, o.total};
        if (o.kind != 'u' || o.total < 4096) continue;
        const size_t nw = o.total / 4;
        host.resize(nw);
        unsigned long long hh = 0;
        for (size_t i = 0; i < nw; i++) {
          host[i] = mix(o.serial + 1000003ull * rep, i);
          hh += (unsigned long long)host[i] * (2ull * i + 1ull);
        }
        want_hash[o.serial] = hh;
        // 1. staged fill (host -> pinned -> device, chunk by chunk), or the
        //    same pattern written by a kernel (--fill kernel)
        if (kfill) {
          hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, st, (unsigned *)p, nw, o.serial + 1000003ull * rep);
        } else {
          for (size_t off = 0; off < nw * 4; off += kChunk) {
            const size_t len = nw * 4 - off < kChunk ? nw * 4 - off : kChunk;
            CK(hipStreamSynchronize(st));
            memcpy(stage, (const char *)host.data() + off, len);
            CK(hipMemcpyAsync((char *)p + off, stage, len, hipMemcpyHostToDevice, st));
          }
        }
        CK(hipStreamSynchronize(st));
        // 2. kernel view, 3. copy view
        const bool kok = kernel_hash(p, nw * 4) == hh;
        bool cok = true;
        for (size_t off = 0; off < nw * 4 && cok; off += kChunk) {
          const size_t len = nw * 4 - off < kChunk ? nw * 4 - off : kChunk;
          CK(hipMemcpyAsync(stage, (char *)p + off, len, hipMemcpyDeviceToHost, st));
          CK(hipStreamSynchronize(st));
          cok = memcmp(stage, (const char *)host.data() + off, len) == 0;
        }
        checked++;
        kernel_bad += !kok;
        copy_bad += !cok;
        if ((!kok || !cok) && kernel_bad + copy_bad <= 10)
          std::printf("rep %d allocation #%llu [%p, +%zu): kernel view %s, copy view %s\n", rep, o.serial, p, o.total,
                      kok ? "intact" : "WRONG", cok ? "intact" : "WRONG");
      } else {
        auto it = live.find(o.serial);
        if (it == live.end()) continue;
        auto wh = want_hash.find(o.serial);
        if (wh != want_hash.end()) {
          // 4. the kernel view just before the free
          if (kernel_hash(it->second.first, it->second.second / 4 * 4) != wh->second) {
            later_bad++;
            if (later_bad <= 10)
              std::printf("rep %d allocation #%llu: kernel view WRONG before its free\n", rep, o.serial);
          }
          want_hash.erase(wh);
        }
        if (pool) {
          CK(hipEventRecord(null_fence, nullptr));
          CK(hipStreamWaitEvent(st, null_fence, 0));
          CK(hipFreeAsync(it->second.first, st));
        } else {
          CK(hipStreamSynchronize(st));
          CK(hipFree(it->second.first));
        }
        live.erase(it);
      }
    }
    for (auto &kv : live) {
      if (pool) CK(hipFreeAsync(kv.second.first, st));
      else CK(hipFree(kv.second.first));
    }
    CK(hipDeviceSynchronize());
  }
  std::printf("%s, %s fill: %d rep(s), %ld filled blocks checked: kernel view wrong %ld, copy view wrong %ld, kernel view "
              "wrong before free %ld\n",
              pool ? "pool" : "hipMalloc", kfill ? "kernel" : "copy", reps, checked, kernel_bad, copy_bad, later_bad);
  return kernel_bad + copy_bad + later_bad ? 1 : 0;
}
