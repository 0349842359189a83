// dr/mhp.hpp -- mhp-style (one process per GPU) layer over the libdrhip
// C-ABI and its RCCL communicators (include/drhip.h "RCCL over xGMI").
//
// the reference's second backend, restated for
// MI355X.  Each process owns ONE segment on ONE GPU; cross-rank steps are
// RCCL calls on the segment's stream instead of MPI.  Mirrors:
//   lib::halo_bounds              details/halo.hpp:315-331
//   mhp::distributed_vector(n, hb) mhp/containers/distributed_vector.hpp:190-207
//                                  (segment size max(ceil(n/P), prev, next),
//                                  buffer [prev | segment | next])
//   dv.halo().exchange()          details/halo.hpp:55-70, 336-387 (span_halo)
//   mhp::iota / mhp::fill         mhp/algorithms/cpu_algorithms.hpp (fill, iota)
//   mhp::transform                cpu_algorithms.hpp:147-167 (aligned ranges;
//                                  op reads neighbours through the pointer)
//   mhp::reduce(root, ...)        cpu_algorithms.hpp:102-140 (locals seeded
//                                  with T(0), gather to root, root folds from
//                                  init; other ranks return 0)
// Cross-rank steps go through a `transport` (halo exchange, gather to a
// root, barrier): the RCCL C-ABI by default (init(rank, nranks, device,
// id): rank 0 makes a communicator id with make_comm_id, every rank
// receives it by any channel -- MPI_Bcast, a file, a torch store); the MPI
// transport of dr/mhp_mpi.hpp (the reference's own transport: MPI messages
// with the reference's halo tags, device buffers staged through the host)
// runs several ranks on ONE GPU, which RCCL refuses.  Both issue the
// message list of dr/details/halo_plan.hpp.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstddef>
#include <cstring>
#include <iterator>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/drhip.h"
#include "details/halo_plan.hpp"

namespace lib {

// details/halo.hpp:315-331
struct halo_bounds {
  halo_bounds(std::size_t radius = 0, bool per = false) : prev(radius), next(radius), periodic(per) {}
  halo_bounds(std::size_t prv, std::size_t nxt, bool per = false) : prev(prv), next(nxt), periodic(per) {}
  std::size_t prev, next;
  bool periodic;
};

} // namespace lib

namespace mhp {

using comm_id = std::array<char, DRHIP_COMM_ID_BYTES>;

// The cross-rank steps of this layer.  Buffers are device pointers of this
// rank's segment (device 0 of drhip_init); every call is blocking, as the
// reference's MPI calls are.
struct transport {
  virtual ~transport() = default;
  virtual const char *name() const = 0;
  // span_halo exchange of a [prev | n_owned | next] buffer of cell_bytes cells
  virtual void halo(void *buf, std::size_t n_owned, std::size_t cell_bytes, std::size_t prev, std::size_t next,
                    bool periodic) = 0;
  // `bytes` from every rank into recv (rank order) on root
  virtual void gather(const void *send, void *recv, std::size_t bytes, int root) = 0;
  virtual void barrier() = 0;
};

namespace detail {

struct state {
  int rank = 0, nranks = 0;
  std::unique_ptr<transport> tr;
};
inline state &st() {
  static state s;
  return s;
}

inline void check(int rc, const char *what) {
  if (rc != DRHIP_OK)
    throw std::runtime_error(std::string("mhp: ") + what + " failed (" + std::to_string(rc) +
                             "): " + drhip_last_error());
}
inline void hip_check(hipError_t e, const char *what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("mhp: ") + what + ": " + hipGetErrorString(e));
}
inline hipStream_t stream() {
  void *s = nullptr;
  check(drhip_stream(0, &s), "drhip_stream");
  return static_cast<hipStream_t>(s);
}
inline void sync() { check(drhip_sync(0), "drhip_sync"); }

constexpr int kThreads = 256;

template <typename T, typename F> __global__ void gen_kernel(T *out, std::size_t n, std::size_t g0, F f) {
  const std::size_t i = blockIdx.x * (std::size_t)kThreads + threadIdx.x;
  if (i < n) out[i] = f(g0 + i);
}

template <typename T, typename U, typename Op>
__global__ void transform_kernel(T *in, U *out, std::size_t n, Op op) {
  const std::size_t i = blockIdx.x * (std::size_t)kThreads + threadIdx.x;
  if (i < n) out[i] = op(in[i]);
}

// per-block folds seeded with T(0) (the reference's std::reduce(..., T(0), op)
// of each local segment); the block partials are folded on the host
template <typename T, typename Op>
__global__ __launch_bounds__(kThreads) void reduce_kernel(const T *in, std::size_t n, Op op, T *part) {
  __shared__ T s[kThreads];
  T acc = T(0);
  for (std::size_t i = blockIdx.x * (std::size_t)kThreads + threadIdx.x; i < n; i += (std::size_t)gridDim.x * kThreads)
    acc = op(acc, in[i]);
  s[threadIdx.x] = acc;
  __syncthreads();
  for (int w = kThreads / 2; w > 0; w /= 2) {
    if ((int)threadIdx.x < w) s[threadIdx.x] = op(s[threadIdx.x], s[threadIdx.x + w]);
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = s[0];
}

inline unsigned grid_for(std::size_t n) { return (unsigned)((n + kThreads - 1) / kThreads); }

// device scratch owned by the caller's scope
template <typename T> struct dev_buf {
  T *p = nullptr;
  explicit dev_buf(std::size_t n) { check(drhip_malloc(0, std::max<std::size_t>(n, 1) * sizeof(T), (void **)&p), "drhip_malloc"); }
  ~dev_buf() {
    if (p) (void)drhip_free(0, p);
  }
  dev_buf(const dev_buf &) = delete;
  dev_buf &operator=(const dev_buf &) = delete;
};

} // namespace detail

inline comm_id make_comm_id() {
  comm_id id{};
  detail::check(drhip_comm_unique_id(id.data()), "drhip_comm_unique_id");
  return id;
}

// The default transport: libdrhip's RCCL communicator of segment 0
// (csrc/comm.hip), every call enqueued on the segment stream, then drained.
struct rccl_transport final : transport {
  const char *name() const override { return "rccl"; }
  void halo(void *buf, std::size_t n_owned, std::size_t cell_bytes, std::size_t prev, std::size_t next,
            bool periodic) override {
    detail::check(drhip_halo_exchange(0, buf, n_owned, cell_bytes, prev, next, periodic ? 1 : 0),
                  "drhip_halo_exchange");
    detail::sync();
  }
  void gather(const void *send, void *recv, std::size_t bytes, int root) override {
    detail::check(drhip_gather(0, send, recv, bytes, root), "drhip_gather");
    detail::sync();
  }
  void barrier() override {
    int *b = nullptr;
    detail::check(drhip_malloc(0, sizeof(int), (void **)&b), "drhip_malloc");
    detail::hip_check(hipMemsetAsync(b, 0, sizeof(int), detail::stream()), "hipMemsetAsync");
    const int rc = drhip_allreduce(0, DRHIP_I32, DRHIP_MAX, b, b, 1);
    detail::sync();
    (void)drhip_free(0, b);
    detail::check(rc, "drhip_allreduce");
  }
};

// Any transport: this process is `rank` of `nranks`, its segment on
// `device` (drhip_init of one device); the transport is owned from here on.
inline void init(int rank, int nranks, int device, std::unique_ptr<transport> tr) {
  if (!tr || nranks < 1 || rank < 0 || rank >= nranks) throw std::runtime_error("mhp::init: bad rank/nranks/transport");
  detail::check(drhip_init(&device, 1), "drhip_init");
  detail::st().rank = rank;
  detail::st().nranks = nranks;
  detail::st().tr = std::move(tr);
}
// One rank per GPU over RCCL: every rank passes the id rank 0 made.
inline void init(int rank, int nranks, int device, const comm_id &id) {
  init(rank, nranks, device, std::make_unique<rccl_transport>());
  detail::check(drhip_comm_init_rank(0, nranks, rank, id.data()), "drhip_comm_init_rank");
}
// A one-rank job on `device` (tests, single-GPU runs).
inline void init(int device = 0) {
  init(0, 1, device, std::make_unique<rccl_transport>());
  comm_id id{};
  detail::check(drhip_comm_unique_id(id.data()), "drhip_comm_unique_id");
  detail::check(drhip_comm_init_rank(0, 1, 0, id.data()), "drhip_comm_init_rank");
}
inline void finalize() {
  detail::st().tr.reset();
  detail::check(drhip_finalize(), "drhip_finalize");
  detail::st().rank = detail::st().nranks = 0;
}
inline transport &comm() {
  if (!detail::st().tr) throw std::runtime_error("mhp: init not called");
  return *detail::st().tr;
}
inline std::size_t rank() { return (std::size_t)detail::st().rank; }
inline std::size_t nprocs() { return (std::size_t)detail::st().nranks; }

// every rank's stream drained and every rank past this point
inline void barrier() {
  detail::sync();
  comm().barrier();
}

template <typename T> class distributed_vector;

template <typename T> struct dv_iterator {
  using value_type = T;
  using difference_type = std::ptrdiff_t;
  distributed_vector<T> *dv = nullptr;
  std::ptrdiff_t i = 0;
  dv_iterator &operator++() { ++i; return *this; }
  dv_iterator operator+(std::ptrdiff_t k) const { return {dv, i + k}; }
  dv_iterator operator-(std::ptrdiff_t k) const { return {dv, i - k}; }
  std::ptrdiff_t operator-(const dv_iterator &o) const { return i - o.i; }
  bool operator==(const dv_iterator &o) const { return dv == o.dv && i == o.i; }
};

template <typename T> struct dv_range {
  dv_iterator<T> first, last;
  dv_iterator<T> begin() const { return first; }
  dv_iterator<T> end() const { return last; }
  std::size_t size() const { return (std::size_t)(last - first); }
};

template <typename T> class halo_ref {
public:
  explicit halo_ref(distributed_vector<T> *dv) : dv_(dv) {}
  // details/halo.hpp:55-70 exchange(): blocking, like the reference
  void exchange() const;

private:
  distributed_vector<T> *dv_;
};

// mhp/containers/distributed_vector.hpp:190-207
template <typename T> class distributed_vector {
public:
  using value_type = T;
  using iterator = dv_iterator<T>;

  distributed_vector(std::size_t n, lib::halo_bounds hb = lib::halo_bounds()) : n_(n), hb_(hb) {
    const dr_plan::block b = dr_plan::block_of(n, nprocs(), rank(), hb.prev, hb.next);
    seg_ = b.segment;
    first_ = b.first;
    local_ = b.local;
    detail::check(drhip_malloc(0, std::max<std::size_t>(hb.prev + seg_ + hb.next, 1) * sizeof(T), (void **)&data_),
                  "drhip_malloc");
    detail::hip_check(hipMemsetAsync(data_, 0, (hb.prev + seg_ + hb.next) * sizeof(T), detail::stream()),
                      "hipMemsetAsync");
    detail::sync();
  }
  ~distributed_vector() {
    if (data_) (void)drhip_free(0, data_);
  }
  distributed_vector(const distributed_vector &) = delete;
  distributed_vector &operator=(const distributed_vector &) = delete;

  std::size_t size() const { return n_; }
  iterator begin() { return {this, 0}; }
  iterator end() { return {this, (std::ptrdiff_t)n_}; }
  halo_ref<T> halo() { return halo_ref<T>(this); }
  const lib::halo_bounds &halo_bounds() const { return hb_; }

  // this rank's segment: global [first_index, first_index + local_size)
  std::size_t segment_size() const { return seg_; }
  std::size_t first_index() const { return first_; }
  std::size_t local_size() const { return local_; }
  T *data() { return data_; }                 // [prev halo | segment | next halo]
  T *owned() { return data_ + hb_.prev; }     // first owned element

private:
  std::size_t n_, seg_ = 0, first_ = 0, local_ = 0;
  lib::halo_bounds hb_;
  T *data_ = nullptr;
};

template <typename T> void halo_ref<T>::exchange() const {
  const auto &hb = dv_->halo_bounds();
  if (hb.prev == 0 && hb.next == 0) return;
  detail::sync(); // the cells written by earlier kernels
  comm().halo(dv_->data(), dv_->segment_size(), sizeof(T), hb.prev, hb.next, hb.periodic);
}

// mhp::halo(range): the halo of the vector a (sub)range belongs to
template <typename T> halo_ref<T> halo(distributed_vector<T> &dv) { return dv.halo(); }
template <typename T> halo_ref<T> halo(const dv_range<T> &r) { return r.first.dv->halo(); }

template <typename T> dv_range<T> subrange(dv_iterator<T> a, dv_iterator<T> b) { return {a, b}; }

namespace detail {
// this rank's part of global [g0, g1): local offset and count
template <typename T> inline std::pair<std::size_t, std::size_t> local_part(distributed_vector<T> &dv, std::size_t g0,
                                                                            std::size_t g1) {
  const std::size_t a = std::max(g0, dv.first_index()), b = std::min(g1, dv.first_index() + dv.local_size());
  return a < b ? std::pair{a - dv.first_index(), b - a} : std::pair{std::size_t(0), std::size_t(0)};
}
} // namespace detail

template <typename T, typename V> void fill(distributed_vector<T> &dv, V value) {
  const T v = static_cast<T>(value);
  auto f = [v](std::size_t) { return v; };
  if (dv.local_size())
    hipLaunchKernelGGL((detail::gen_kernel<T, decltype(f)>), dim3(detail::grid_for(dv.local_size())),
                       dim3(detail::kThreads), 0, detail::stream(), dv.owned(), dv.local_size(), dv.first_index(), f);
  detail::sync();
}

template <typename T, typename V> void iota(distributed_vector<T> &dv, V start) {
  const T s = static_cast<T>(start);
  auto f = [s](std::size_t g) { return static_cast<T>(s + static_cast<T>(g)); };
  if (dv.local_size())
    hipLaunchKernelGGL((detail::gen_kernel<T, decltype(f)>), dim3(detail::grid_for(dv.local_size())),
                       dim3(detail::kThreads), 0, detail::stream(), dv.owned(), dv.local_size(), dv.first_index(), f);
  detail::sync();
}

// cpu_algorithms.hpp:147-167: aligned ranges only (same segmentation, same
// global offsets); op gets a reference into the halo'd buffer
template <typename T, typename U, typename Op>
void transform(dv_iterator<T> first, dv_iterator<T> last, dv_iterator<U> out, Op op) {
  auto &in = *first.dv;
  auto &o = *out.dv;
  if (first.i != out.i || in.segment_size() != o.segment_size() || in.first_index() != o.first_index())
    throw std::runtime_error("mhp::transform: input and output ranges are not aligned");
  auto [off, cnt] = detail::local_part(in, (std::size_t)first.i, (std::size_t)last.i);
  if (cnt)
    hipLaunchKernelGGL((detail::transform_kernel<T, U, Op>), dim3(detail::grid_for(cnt)), dim3(detail::kThreads), 0,
                       detail::stream(), in.owned() + off, o.owned() + off, cnt, op);
  barrier();
}
template <typename T, typename U, typename Op> void transform(const dv_range<T> &in, dv_iterator<U> out, Op op) {
  transform(in.first, in.last, out, op);
}

// cpu_algorithms.hpp:102-140 (aligned branch)
template <typename T, typename V, typename Op> V reduce(int root, dv_iterator<T> first, dv_iterator<T> last, V init, Op op) {
  auto &dv = *first.dv;
  auto [off, cnt] = detail::local_part(dv, (std::size_t)first.i, (std::size_t)last.i);
  V local = V(0);
  if (cnt) {
    const unsigned grid = std::min<unsigned>(detail::grid_for(cnt), 1024u);
    detail::dev_buf<V> part(grid);
    if constexpr (std::is_same_v<T, V>) {
      hipLaunchKernelGGL((detail::reduce_kernel<T, Op>), dim3(grid), dim3(detail::kThreads), 0, detail::stream(),
                         dv.owned() + off, cnt, op, part.p);
      std::vector<V> h(grid);
      detail::check(drhip_memcpy_d2h(0, h.data(), part.p, grid * sizeof(V)), "drhip_memcpy_d2h");
      for (auto x : h) local = op(local, x);
    } else {
      static_assert(std::is_same_v<T, V>, "mhp::reduce: init must have the element type");
    }
  }
  const int p = (int)nprocs();
  detail::dev_buf<V> send(1), all(p);
  detail::check(drhip_memcpy_h2d(0, send.p, &local, sizeof(V)), "drhip_memcpy_h2d");
  comm().gather(send.p, all.p, sizeof(V), root);
  V result = V(0);
  if ((int)rank() == root) {
    std::vector<V> h(p);
    detail::check(drhip_memcpy_d2h(0, h.data(), all.p, p * sizeof(V)), "drhip_memcpy_d2h");
    result = dr_plan::fold_locals(init, h.begin(), h.end(), op);
  }
  return result;
}
template <typename T, typename V, typename Op> V reduce(int root, const dv_range<T> &r, V init, Op op) {
  return reduce(root, r.first, r.last, init, op);
}

// Collect the whole vector on `root` (other ranks get an empty vector): the
// check path of the reference tests (equal(v, dv) reads remote segments).
template <typename T> std::vector<T> gather(distributed_vector<T> &dv, int root = 0) {
  const std::size_t p = nprocs(), seg = dv.segment_size();
  detail::dev_buf<T> all(p * seg);
  detail::sync();
  comm().gather(dv.owned(), all.p, seg * sizeof(T), root);
  std::vector<T> out;
  if ((int)rank() == root) {
    out.resize(p * seg);
    detail::check(drhip_memcpy_d2h(0, out.data(), all.p, p * seg * sizeof(T)), "drhip_memcpy_d2h");
    out.resize(dv.size());
  }
  return out;
}

// This rank's buffer [prev halo | segment | next halo] on the host.
template <typename T> std::vector<T> local_buffer(distributed_vector<T> &dv) {
  const auto &hb = dv.halo_bounds();
  std::vector<T> h(hb.prev + dv.segment_size() + hb.next);
  detail::check(drhip_memcpy_d2h(0, h.data(), dv.data(), h.size() * sizeof(T)), "drhip_memcpy_d2h");
  return h;
}

} // namespace mhp
