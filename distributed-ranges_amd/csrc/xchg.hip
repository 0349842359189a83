// xchg.hip -- all-gather of one 8-byte value per segment through flag slots
// in device memory: the combine of a strong-scaled reduce + inclusive_scan
// step ("RCCL all_gather or P2P stores into a slot plus a
// flag, whichever measures faster") without a collective.
//
// Replaces, for that step, the reference's gather of the segment results
// (reduce.hpp:81-83 folds them in segment order on the host;
// inclusive_scan.hpp:108-116 scans the piece totals on device 0) -- here
// every rank ends with all w values in segment order in device memory and
// the scan kernel folds them itself (drhip_inclusive_scan_tiles partials).
//
// Slot array of one rank (fine-grained device memory, so stores from peer
// GPUs are seen by this GPU's polls): a 128-B header line holding the
// rank's exchange count, then for every source rank s two 128-B lines, one
// per epoch parity, each {value, epoch}.  One exchange (one 1-block kernel
// on the segment's stream):
//   e = ++header (device-side: graph replays advance it too);
//   for every rank j: store value into slot (rank, e & 1) of j's array, then
//     store e there with release semantics at system scope;
//   wait until every slot (s, e & 1) of this rank's array holds epoch e
//     (acquire), copy the w values to gathered[] in rank order.
// Two parities: a rank can post exchange e + 1 only after every rank posted
// e, so its store lands on the other parity while a slower rank may still
// read parity e & 1.  A wait that does not finish within the spin bound
// sets the segment's error word (drhip_sync returns DRHIP_ERR_TIMEOUT).
#include "common.hpp"

#include <cstring>

namespace drhip {

constexpr int kXchgMaxRanks = 64;
constexpr size_t kXchgLine = 128;
constexpr unsigned kXchgSpinLimit = 1u << 20; // ~1-2 s of polls

struct XchgPeers {
  unsigned long long *p[kXchgMaxRanks]; // every rank's slot array, as mapped in this process
};

size_t xchg_bytes(int w) { return kXchgLine * (1 + 2 * (size_t)w); }

__global__ __launch_bounds__(64) void xchg_allgather_kernel(unsigned long long *local, XchgPeers peers, int w,
                                                            int rank, const void *value, int vbytes,
                                                            void *gathered, unsigned *err) {
  constexpr size_t L = kXchgLine / 8; // 64-bit words per line
  const int lane = threadIdx.x;
  __shared__ unsigned long long s_e;
  if (lane == 0) {
    const unsigned long long e = __hip_atomic_load(local, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    __hip_atomic_store(local, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_e = e;
  }
  __syncthreads();
  const unsigned long long e = s_e;
  const unsigned long long v = vbytes == 8 ? *(const unsigned long long *)value : *(const unsigned *)value;
  const size_t par = (size_t)(e & 1);
  // post: lane j stores into rank j's array (slot `rank`, parity e & 1)
  for (int j = lane; j < w; j += 64) {
    unsigned long long *slot = peers.p[j] + L * (1 + 2 * (size_t)rank + par);
    __hip_atomic_store(slot, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(slot + 1, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // wait: lane s polls slot s of this rank's array
  bool timed_out = false;
  for (int s = lane; s < w; s += 64) {
    const unsigned long long *slot = local + L * (1 + 2 * (size_t)s + par);
    unsigned spins = 0;
    while (__hip_atomic_load(slot + 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != e) {
      if (++spins > kXchgSpinLimit) {
        timed_out = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    const unsigned long long g = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (vbytes == 8) ((unsigned long long *)gathered)[s] = g;
    else ((unsigned *)gathered)[s] = (unsigned)g;
  }
  if (timed_out) __hip_atomic_store(err, 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

} // namespace drhip

using namespace drhip;

extern "C" int drhip_xchg_bytes(int w, size_t *bytes) {
  if (!bytes || w < 1 || w > kXchgMaxRanks) return set_error(DRHIP_ERR_BAD_ARG, "drhip_xchg_bytes: 1 <= w <= 64");
  *bytes = xchg_bytes(w);
  return DRHIP_OK;
}

extern "C" int drhip_xchg_alloc(int seg, int w, void **slots) {
  DRHIP_GET_SEG(s, seg);
  if (!slots || w < 1 || w > kXchgMaxRanks) return set_error(DRHIP_ERR_BAD_ARG, "drhip_xchg_alloc: 1 <= w <= 64");
  *slots = nullptr;
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  void *p = nullptr;
  DRHIP_CHECK_HIP(hipExtMallocWithFlags(&p, xchg_bytes(w), hipDeviceMallocFinegrained));
  const hipError_t e = hipMemset(p, 0, xchg_bytes(w));
  if (e != hipSuccess) {
    (void)hipFree(p);
    return set_hip_error(e, "hipMemset(xchg slots)");
  }
  *slots = p;
  return DRHIP_OK;
}

extern "C" int drhip_xchg_free(int seg, void *slots) {
  DRHIP_GET_SEG(s, seg);
  if (!slots) return DRHIP_OK;
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  DRHIP_CHECK_HIP(hipStreamSynchronize(s->stream));
  DRHIP_CHECK_HIP(hipFree(slots));
  return DRHIP_OK;
}

extern "C" int drhip_ipc_handle(const void *dev_ptr, void *handle) {
  if (!dev_ptr || !handle) return set_error(DRHIP_ERR_BAD_ARG, "drhip_ipc_handle: null");
  static_assert(sizeof(hipIpcMemHandle_t) <= DRHIP_IPC_HANDLE_BYTES, "handle size");
  hipIpcMemHandle_t h;
  DRHIP_CHECK_HIP(hipIpcGetMemHandle(&h, const_cast<void *>(dev_ptr)));
  memset(handle, 0, DRHIP_IPC_HANDLE_BYTES);
  memcpy(handle, &h, sizeof h);
  return DRHIP_OK;
}

extern "C" int drhip_ipc_open(int seg, const void *handle, void **dev_ptr) {
  DRHIP_GET_SEG(s, seg);
  if (!handle || !dev_ptr) return set_error(DRHIP_ERR_BAD_ARG, "drhip_ipc_open: null");
  *dev_ptr = nullptr;
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof h);
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  DRHIP_CHECK_HIP(hipIpcOpenMemHandle(dev_ptr, h, hipIpcMemLazyEnablePeerAccess));
  return DRHIP_OK;
}

extern "C" int drhip_ipc_close(int seg, void *dev_ptr) {
  DRHIP_GET_SEG(s, seg);
  if (!dev_ptr) return DRHIP_OK;
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  DRHIP_CHECK_HIP(hipStreamSynchronize(s->stream));
  DRHIP_CHECK_HIP(hipIpcCloseMemHandle(dev_ptr));
  return DRHIP_OK;
}

extern "C" int drhip_xchg_allgather(int seg, void *local_slots, void *const *peer_slots, int w, int rank,
                                    const void *value, int value_bytes, void *gathered) {
  DRHIP_GET_SEG(s, seg);
  if (!local_slots || !peer_slots || !value || !gathered || w < 1 || w > kXchgMaxRanks || rank < 0 || rank >= w)
    return set_error(DRHIP_ERR_BAD_ARG, "drhip_xchg_allgather: slots / value / gathered, 1 <= w <= 64, rank < w");
  if (value_bytes != 4 && value_bytes != 8) return set_error(DRHIP_ERR_BAD_ARG, "drhip_xchg_allgather: 4- or 8-byte values");
  XchgPeers peers{};
  for (int j = 0; j < w; j++) {
    if (!peer_slots[j]) return set_error(DRHIP_ERR_BAD_ARG, "drhip_xchg_allgather: null peer slot array");
    peers.p[j] = (unsigned long long *)peer_slots[j];
  }
  if (peers.p[rank] != (unsigned long long *)local_slots)
    return set_error(DRHIP_ERR_BAD_ARG, "drhip_xchg_allgather: peer_slots[rank] must be local_slots");
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  hipLaunchKernelGGL(xchg_allgather_kernel, dim3(1), dim3(64), 0, s->stream, (unsigned long long *)local_slots, peers,
                     w, rank, value, value_bytes, gathered, s->err);
  DRHIP_CHECK_LAUNCH();
  return DRHIP_OK;
}
