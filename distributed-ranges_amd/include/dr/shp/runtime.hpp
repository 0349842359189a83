// dr/shp/runtime.hpp -- device registry and execution policy of the shp
// drop-in layer, over the libdrhip C-ABI (include/drhip.h).
//
// Mirrors include/dr/shp/init.hpp:16-52 (init / finalize / devices /
// nprocs / context / par_unseq), algorithms/execution_policy.hpp:13-32
// (device_policy) and util.hpp:77-136 (get_numa_devices,
// get_duplicated_devices).  A "device" is a HIP device ordinal instead of a
// sycl::device; the list index is the segment rank, and an ordinal may
// repeat (the reference test harness's --devicesCount duplication,
// test/gtest/shp/shp-tests.cpp:34-39).  Every segment owns one HIP stream
// (created by drhip_init); algorithms enqueue on those streams and block
// before returning, like the reference.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <memory>
#include <utility>
#include <ranges>
#include <span>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../../include/drhip.h"

namespace shp {

namespace detail {

inline std::vector<int> &device_list() {
  static std::vector<int> d;
  return d;
}

// Throws on a non-zero C-ABI status (the reference propagates SYCL
// exceptions synchronously; SURVEY.md 8b "Errors").
inline void check(int rc, const char *what) {
  if (rc != DRHIP_OK)
    throw std::runtime_error(std::string("shp: ") + what + " failed (" + std::to_string(rc) +
                             "): " + drhip_last_error());
}

inline void hip_check(hipError_t e, const char *what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("shp: ") + what + ": " + hipGetErrorString(e));
}

} // namespace detail

// execution_policy.hpp:13-32
class device_policy {
public:
  device_policy() = default;
  explicit device_policy(std::span<const int> devices) : devices_(devices.begin(), devices.end()) {}
  std::span<const int> get_devices() const noexcept { return devices_; }

private:
  std::vector<int> devices_;
};

inline device_policy par_unseq;

// init.hpp:40-50: ordered device list -> segment ranks.
template <std::ranges::input_range R>
  requires std::convertible_to<std::ranges::range_value_t<R>, int>
void init(R &&devices) {
  std::vector<int> d;
  for (auto &&x : devices) d.push_back(static_cast<int>(x));
  if (d.empty()) throw std::runtime_error("shp::init: empty device list");
  detail::check(drhip_init(d.data(), static_cast<int>(d.size())), "drhip_init");
  detail::device_list() = d;
  par_unseq = device_policy(std::span<const int>(detail::device_list()));
}

namespace detail {
// Host-pinned scratch cache: blocks handed out by detail::pinned and the
// template reduce's partials (algorithms.hpp) go back here instead of to
// hipHostFree -- one hipHostMalloc per call cost more than the kernel of a
// 2 GiB reduce.  Released by finalize().  Single host thread, like the
// reference's global state (init.hpp:18-22).
struct pinned_pool {
  std::vector<std::pair<void *, std::size_t>> free_blocks;
  void *get(std::size_t bytes, std::size_t &cap) {
    for (std::size_t i = 0; i < free_blocks.size(); i++)
      if (free_blocks[i].second >= bytes) {
        auto e = free_blocks[i];
        free_blocks.erase(free_blocks.begin() + static_cast<std::ptrdiff_t>(i));
        cap = e.second;
        return e.first;
      }
    cap = std::max<std::size_t>(bytes, 4096);
    void *p = nullptr;
    check(drhip_host_alloc(cap, &p), "drhip_host_alloc");
    return p;
  }
  void put(void *p, std::size_t cap) {
    if (p) free_blocks.emplace_back(p, cap);
  }
  void release() {
    for (auto &e : free_blocks) (void)drhip_host_free(e.first);
    free_blocks.clear();
  }
};
inline pinned_pool &host_pool() {
  static pinned_pool pool;
  return pool;
}

// Per-segment device scratch (the look-back scan's tile status words, the
// sort's key/histogram workspace): grown on first use to the largest size
// asked for and reused, so repeated algorithm calls allocate nothing.  Work
// that uses it is enqueued on the segment's own stream, so consecutive users
// are ordered by that stream.  Released by finalize().
struct device_scratch_pool {
  std::vector<std::pair<void *, std::size_t>> per_rank;
  void *get(std::size_t rank, std::size_t bytes) {
    if (per_rank.size() <= rank) per_rank.resize(rank + 1, {nullptr, 0});
    auto &e = per_rank[rank];
    if (e.second < bytes) {
      if (e.first) check(drhip_free(static_cast<int>(rank), e.first), "drhip_free"); // stream-synced
      e = {nullptr, 0};
      const std::size_t cap = std::max<std::size_t>((bytes + 4095) & ~std::size_t(4095), std::size_t(1) << 20);
      check(drhip_malloc(static_cast<int>(rank), cap, &e.first), "drhip_malloc");
      e.second = cap;
    }
    return e.first;
  }
  void release() {
    for (std::size_t r = 0; r < per_rank.size(); r++)
      if (per_rank[r].first) (void)drhip_free(static_cast<int>(r), per_rank[r].first);
    per_rank.clear();
  }
};
inline device_scratch_pool &device_scratch() {
  static device_scratch_pool pool;
  return pool;
}
// The look-back scans' status buffers (dr/shp/scan.hpp DR_SHP_LB_EPOCH): one
// per segment, owned by the look-back scans alone (another user's bytes there
// could carry a live epoch's tag).  Every call takes the next epoch.  Two
// layouts share the buffer: T <= 12 bytes publishes {value, tag} 8-B words at
// fixed 128-B granules (every granule word's high half only ever holds a
// tag), larger T a 4-B tag array followed by value arrays whose offset moves
// with the tile count.  So a tag word can only hold a stale TAG -- never user
// data -- while consecutive calls keep the small layout; anything else is
// cleared: a large-T call clears its tag array (the round-4 reset per call),
// and the first small-T call after a large one (or after an allocation, or
// when the 30-bit epoch wraps) clears the whole buffer.  Calls on a segment
// are ordered by its stream.
#ifndef DR_SHP_LB_EPOCH_MAX
#define DR_SHP_LB_EPOCH_MAX ((1u << 30) - 1) // tests build a small wrap to exercise the clear
#endif
// test builds only: DR_SHP_LB_LAYOUT_CLEAR=0 drops the layout rule above (the
// ScanStatusLayoutSwitch test then shows a small-T value read as a tag)
#ifndef DR_SHP_LB_LAYOUT_CLEAR
#define DR_SHP_LB_LAYOUT_CLEAR 1
#endif
struct lb_status_pool {
  struct entry {
    void *p = nullptr;
    std::size_t cap = 0;
    unsigned epoch = 0;
    bool large = false; // the last call used the large-T layout
  };
  std::vector<entry> per_rank;
  // bytes: this call's span; tag_bytes: its head + tag words (what a
  // large-T call clears)
  void *get(std::size_t rank, std::size_t bytes, std::size_t tag_bytes, bool large, hipStream_t st, unsigned &epoch) {
    if (per_rank.size() <= rank) per_rank.resize(rank + 1);
    entry &e = per_rank[rank];
    if (e.cap < bytes) {
      if (e.p) check(drhip_free(static_cast<int>(rank), e.p), "drhip_free"); // stream-synced
      e = entry{};
      const std::size_t cap = std::max<std::size_t>((bytes + 4095) & ~std::size_t(4095), std::size_t(1) << 20);
      check(drhip_malloc(static_cast<int>(rank), cap, &e.p), "drhip_malloc");
      e.cap = cap;
    }
    if (DR_SHP_LB_LAYOUT_CLEAR && large) {
      hip_check(hipMemsetAsync(e.p, 0, tag_bytes, st), "scan status clear");
      e.epoch = 0;
    } else if (e.epoch == 0 || e.epoch >= DR_SHP_LB_EPOCH_MAX || (DR_SHP_LB_LAYOUT_CLEAR && e.large)) {
      hip_check(hipMemsetAsync(e.p, 0, e.cap, st), "scan status clear");
      e.epoch = 0;
    }
    e.large = large;
    epoch = ++e.epoch;
    return e.p;
  }
  void release() {
    for (std::size_t r = 0; r < per_rank.size(); r++)
      if (per_rank[r].p) (void)drhip_free(static_cast<int>(r), per_rank[r].p);
    per_rank.clear();
  }
};
inline lb_status_pool &lb_status_buffers() {
  static lb_status_pool pool;
  return pool;
}

} // namespace detail

inline void finalize() {
  detail::device_scratch().release();
  detail::lb_status_buffers().release();
  detail::host_pool().release();
  detail::check(drhip_finalize(), "drhip_finalize");
  detail::device_list().clear();
  par_unseq = device_policy();
}

inline std::span<const int> devices() { return detail::device_list(); }
inline std::size_t nprocs() { return detail::device_list().size(); }

// init.hpp:27-30 shp::context(): SYCL needs one context over all devices;
// HIP has none, so this is a token the allocator constructors accept.
struct context_type {};
inline context_type context() { return {}; }

namespace detail {
// first segment placed on HIP device `device` (allocations by device)
inline std::size_t segment_of_device(int device) {
  const auto &d = device_list();
  for (std::size_t i = 0; i < d.size(); i++)
    if (d[i] == device) return i;
  throw std::runtime_error("shp: device " + std::to_string(device) + " is not in the shp::init list");
}
} // namespace detail

// The completion handle copy_async / fill_async return (the reference's
// sycl::event, copy.hpp:19-168): one HIP event per segment stream the
// operation was enqueued on; wait() blocks until all of them completed.
class event {
public:
  event() = default;
  void wait() {
    for (auto &e : events_) detail::hip_check(hipEventSynchronize(e.get()), "event wait");
  }
  // record the current end of segment `rank`'s stream
  void add(std::size_t rank) {
    hipEvent_t ev = nullptr;
    detail::hip_check(hipSetDevice(device_list_at(rank)), "hipSetDevice");
    detail::hip_check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
    void *s = nullptr;
    detail::check(drhip_stream(static_cast<int>(rank), &s), "drhip_stream");
    detail::hip_check(hipEventRecord(ev, static_cast<hipStream_t>(s)), "hipEventRecord");
    events_.emplace_back(ev, [](hipEvent_t x) { (void)hipEventDestroy(x); });
  }
  void merge(const event &o) { events_.insert(events_.end(), o.events_.begin(), o.events_.end()); }

private:
  static int device_list_at(std::size_t rank) { return detail::device_list().at(rank); }
  std::vector<std::shared_ptr<std::remove_pointer_t<hipEvent_t>>> events_;
};

// util.hpp:108-117.  MI355X exposes no NUMA sub-devices: every visible HIP
// device is one root device.
inline std::vector<int> get_numa_devices() {
  int n = 0;
  detail::check(drhip_device_count(&n), "drhip_device_count");
  std::vector<int> d(n);
  for (int i = 0; i < n; i++) d[i] = i;
  return d;
}

// util.hpp:121-136 / shp-tests.cpp:34-39: repeat the list up to `count`.
inline std::vector<int> get_duplicated_devices(std::vector<int> devices, std::size_t count) {
  if (devices.empty()) throw std::runtime_error("shp::get_duplicated_devices: no devices");
  std::vector<int> out;
  for (std::size_t i = 0; i < count; i++) out.push_back(devices[i % devices.size()]);
  return out;
}

// The segment's HIP stream (the replacement for a per-call sycl::queue).
inline hipStream_t stream(std::size_t rank) {
  void *s = nullptr;
  detail::check(drhip_stream(static_cast<int>(rank), &s), "drhip_stream");
  return static_cast<hipStream_t>(s);
}

inline void sync(std::size_t rank) { detail::check(drhip_sync(static_cast<int>(rank)), "drhip_sync"); }
inline void sync_all() { detail::check(drhip_sync_all(), "drhip_sync_all"); }

// Run f(rank) for every segment that has work, then wait for all streams
// (the reference's "submit per segment, then event.wait() on all").
template <typename F> void for_each_rank_and_wait(std::span<const std::size_t> ranks, F &&f) {
  for (auto r : ranks) f(r);
  for (auto r : ranks) sync(r);
}

} // namespace shp
