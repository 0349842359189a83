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
//   mhp::copy / mhp::for_each     cpu_algorithms.hpp:36-81 (aligned: local
//                                  segments; misaligned copy / transform: one
//                                  collective alltoallv instead of the
//                                  reference's per-element MPI_Put + fence)
//   local_segments, segments      mhp/views.hpp:9-21
//   views::take/drop/zip/transform, subrange  (test/gtest/mhp/views.cpp)
//   aligned(it...)                mhp/alignment.hpp:8-27
//   fence()                       mhp/global.hpp:41-48 (no RMA windows here:
//                                  a barrier; per-element remote access, the
//                                  reference's MPI window, is out of scope --
//                                  SURVEY.md 2.3)
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
  // byte counts / offsets per peer (send from `send`, receive into `recv`);
  // the misaligned copy / transform exchange (dr_plan::exchange_plan)
  virtual void alltoallv(const void *send, const std::size_t *send_bytes, const std::size_t *send_off, void *recv,
                         const std::size_t *recv_bytes, const std::size_t *recv_off) = 0;
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

template <typename T, typename Op> __global__ void for_each_kernel(T *p, std::size_t n, Op op) {
  const std::size_t i = blockIdx.x * (std::size_t)kThreads + threadIdx.x;
  if (i < n) op(p[i]);
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
  void alltoallv(const void *send, const std::size_t *send_bytes, const std::size_t *send_off, void *recv,
                 const std::size_t *recv_bytes, const std::size_t *recv_off) override {
    detail::check(drhip_alltoallv(0, send, send_bytes, send_off, recv, recv_bytes, recv_off), "drhip_alltoallv");
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

// mhp::distributed_vector's iterator: a global position in one vector.
// Dereferencing it would be a remote element access (the reference's MPI
// window, out of scope), so it only positions ranges for the collective
// algorithms below.
template <typename T> struct dv_iterator {
  using value_type = T;
  using difference_type = std::ptrdiff_t;
  distributed_vector<T> *dv = nullptr;
  std::ptrdiff_t i = 0;
  dv_iterator &operator++() { ++i; return *this; }
  dv_iterator &operator+=(std::ptrdiff_t k) { i += k; return *this; }
  dv_iterator operator+(std::ptrdiff_t k) const { return {dv, i + k}; }
  dv_iterator operator-(std::ptrdiff_t k) const { return {dv, i - k}; }
  std::ptrdiff_t operator-(const dv_iterator &o) const { return i - o.i; }
  bool operator==(const dv_iterator &o) const { return dv == o.dv && i == o.i; }
  bool operator!=(const dv_iterator &o) const { return !(*this == o); }
};

// A contiguous global range [first, last) of one vector: subrange, take,
// drop and the vector itself all become one.
template <typename T> struct dv_range {
  using value_type = T;
  dv_iterator<T> first, last;
  dv_iterator<T> begin() const { return first; }
  dv_iterator<T> end() const { return last; }
  std::size_t size() const { return (std::size_t)(last - first); }
};

// One rank's part of a range (details/ranges.hpp:38-165 rank / local):
// global [begin, end) held by `rank`; local() is a device pointer, valid on
// that rank only.
template <typename T> struct dv_segment {
  distributed_vector<T> *dv;
  std::size_t rank_, begin_, end_;
  std::size_t rank() const { return rank_; }
  std::size_t size() const { return end_ - begin_; }
  std::size_t global_begin() const { return begin_; }
  T *local() const;
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
  // every rank's part, in rank order (shp-style segments(): trimmed to size)
  std::vector<dv_segment<T>> segments() {
    std::vector<dv_segment<T>> v;
    for (const auto &p : dr_plan::range_pieces(n_, seg_, nprocs(), 0, n_)) v.push_back({this, p.rank, p.begin, p.end});
    return v;
  }

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

template <typename T> T *dv_segment<T>::local() const {
  if (rank_ != rank()) throw std::runtime_error("mhp: local() of another rank's segment");
  return dv->owned() + (begin_ - dv->first_index());
}

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
template <typename T> dv_range<T> range_of(distributed_vector<T> &dv) { return {dv.begin(), dv.end()}; }
template <typename T> dv_range<T> range_of(const dv_range<T> &r) { return r; }
// what range_of accepts: a vector or a contiguous range of one
template <typename R> concept vector_range = requires(R &&r) { range_of(r); };

// ------------------------------------------------------------- views
// test/gtest/mhp/views.cpp: zip of aligned ranges (elements are pairs of
// references, .first / .second as range-v3's common_pair), take, drop, and
// a read-only transform view.
template <typename A, typename B> struct zip_ref {
  A &first;
  B &second;
};
template <typename A, typename B> struct zip_range {
  dv_range<A> a;
  dv_range<B> b;
  std::size_t size() const { return std::min(a.size(), b.size()); }
};
template <typename T, typename F> struct transform_range {
  dv_range<T> r;
  F f;
  std::size_t size() const { return r.size(); }
};

namespace views {
template <vector_range R> auto take(R &&r, std::size_t k) {
  auto x = range_of(r);
  return dv_range<typename decltype(x)::value_type>{x.first, x.first + (std::ptrdiff_t)std::min(k, x.size())};
}
template <vector_range R> auto drop(R &&r, std::size_t k) {
  auto x = range_of(r);
  return dv_range<typename decltype(x)::value_type>{x.first + (std::ptrdiff_t)std::min(k, x.size()), x.last};
}
template <vector_range R1, vector_range R2> auto zip(R1 &&r1, R2 &&r2) {
  auto a = range_of(r1);
  auto b = range_of(r2);
  return zip_range<typename decltype(a)::value_type, typename decltype(b)::value_type>{a, b};
}
template <vector_range R, typename F> auto transform(R &&r, F f) {
  auto x = range_of(r);
  return transform_range<typename decltype(x)::value_type, F>{x, f};
}
} // namespace views

// segments of a range: every rank's part in rank order (empty parts left
// out), details/segments_tools.hpp:37-94 for subranges
template <typename T> std::vector<dv_segment<T>> segments(const dv_range<T> &r) {
  auto *dv = r.first.dv;
  std::vector<dv_segment<T>> v;
  for (const auto &p : dr_plan::range_pieces(dv->size(), dv->segment_size(), nprocs(), (std::size_t)r.first.i,
                                             (std::size_t)r.last.i))
    v.push_back({dv, p.rank, p.begin, p.end});
  return v;
}
template <typename T> std::vector<dv_segment<T>> segments(distributed_vector<T> &dv) { return dv.segments(); }
template <typename T> std::vector<dv_segment<T>> segments(dv_iterator<T> it) {
  return segments(dv_range<T>{it, it.dv->end()});
}

namespace detail {
template <typename T> std::vector<dr_plan::piece> pieces(const dv_range<T> &r) {
  return dr_plan::range_pieces(r.first.dv->size(), r.first.dv->segment_size(), nprocs(), (std::size_t)r.first.i,
                               (std::size_t)r.last.i);
}
// this rank's part of a range: (device pointer, count); count 0 if none
template <typename T> std::pair<T *, std::size_t> local_span(const dv_range<T> &r) {
  auto &dv = *r.first.dv;
  const std::size_t a = std::max((std::size_t)r.first.i, dv.first_index());
  const std::size_t b = std::min((std::size_t)r.last.i, dv.first_index() + dv.local_size());
  return a < b ? std::pair{dv.owned() + (a - dv.first_index()), b - a} : std::pair{(T *)nullptr, std::size_t(0)};
}
} // namespace detail

// mhp/alignment.hpp:8-27: ranges starting at these iterators (to their
// vectors' ends, the shorter length) pair up segment by segment
template <typename T> bool aligned(dv_iterator<T>) { return true; }
template <typename T, typename U, typename... R> bool aligned(dv_iterator<T> a, dv_iterator<U> b, R... rest) {
  const std::size_t len = std::min(a.dv->size() - (std::size_t)a.i, b.dv->size() - (std::size_t)b.i);
  if (!dr_plan::pieces_aligned(detail::pieces(dv_range<T>{a, a + (std::ptrdiff_t)len}),
                               detail::pieces(dv_range<U>{b, b + (std::ptrdiff_t)len})))
    return false;
  if constexpr (sizeof...(R) == 0) return true;
  else return aligned(b, rest...);
}
template <typename A, typename B> bool aligned(const zip_range<A, B> &z) {
  const std::ptrdiff_t len = (std::ptrdiff_t)z.size();
  return dr_plan::pieces_aligned(detail::pieces(dv_range<A>{z.a.first, z.a.first + len}),
                                 detail::pieces(dv_range<B>{z.b.first, z.b.first + len}));
}

// mhp/views.hpp:9-21: this rank's segments of a range as local device spans
// {data, size}: at most one for a vector's range; for an aligned zip, the
// pair of spans
template <typename T> struct local_span_t {
  T *ptr;
  std::size_t n;
  T *data() const { return ptr; }
  std::size_t size() const { return n; }
};
template <vector_range R> auto local_segments(R &&r) {
  auto x = range_of(r);
  using T = typename decltype(x)::value_type;
  std::vector<local_span_t<T>> v;
  auto [p, c] = detail::local_span(x);
  if (c) v.push_back({p, c});
  return v;
}

// mhp/global.hpp:41-48: there are no MPI windows here (no per-element remote
// access), so the fence is the barrier the reference's algorithms also end
// with
inline void fence() { barrier(); }

namespace detail {
// this rank's part of global [g0, g1): local offset and count
template <typename T> inline std::pair<std::size_t, std::size_t> local_part(distributed_vector<T> &dv, std::size_t g0,
                                                                            std::size_t g1) {
  const std::size_t a = std::max(g0, dv.first_index()), b = std::min(g1, dv.first_index() + dv.local_size());
  return a < b ? std::pair{a - dv.first_index(), b - a} : std::pair{std::size_t(0), std::size_t(0)};
}

template <typename A, typename B, typename Op> __global__ void for_each_zip_kernel(A *a, B *b, std::size_t n, Op op) {
  const std::size_t i = blockIdx.x * (std::size_t)kThreads + threadIdx.x;
  if (i < n) op(zip_ref<A, B>{a[i], b[i]});
}

// The misaligned copy's exchange (dr_plan::exchange_plan): input [a, b) of
// `in` to output positions [o, o + b - a) of `out`; received elements land
// in `recv` (this rank's owned output slots, or a staging buffer laid out
// like them).  Every rank calls it (one collective).
template <typename T, typename U>
void exchange_into(distributed_vector<T> &in, std::size_t a, std::size_t b, distributed_vector<U> &out, std::size_t o,
                   U *recv_base) {
  static_assert(sizeof(T) == sizeof(U), "mhp: misaligned copy between element types of different sizes");
  const auto e = dr_plan::exchange_plan(in.size(), in.segment_size(), a, b, out.size(), out.segment_size(), o,
                                        nprocs(), rank());
  const std::size_t p = nprocs();
  std::vector<std::size_t> sb(p), so(p), rb(p), ro(p);
  for (std::size_t r = 0; r < p; r++) {
    sb[r] = e.send_cnt[r] * sizeof(T);
    so[r] = e.send_off[r] * sizeof(T);
    rb[r] = e.recv_cnt[r] * sizeof(U);
    ro[r] = e.recv_off[r] * sizeof(U);
  }
  sync();
  comm().alltoallv(in.owned(), sb.data(), so.data(), recv_base, rb.data(), ro.data());
}
} // namespace detail

// cpu_algorithms.hpp:13-27 fill (collective; every rank fills its part)
template <vector_range R, typename V> void fill(R &&r, V value) {
  auto x = range_of(r);
  using T = typename decltype(x)::value_type;
  const T v = static_cast<T>(value);
  auto [p, c] = detail::local_span(x);
  auto f = [v](std::size_t) { return v; };
  if (c)
    hipLaunchKernelGGL((detail::gen_kernel<T, decltype(f)>), dim3(detail::grid_for(c)), dim3(detail::kThreads), 0,
                       detail::stream(), p, c, 0, f);
  barrier();
}
template <typename T, typename V> void fill(dv_iterator<T> first, dv_iterator<T> last, V value) {
  mhp::fill(dv_range<T>{first, last}, value);
}

// cpu_algorithms.hpp:83-100 iota: element g of [first, last) = value + (g - first)
template <vector_range R, typename V> void iota(R &&r, V start) {
  auto x = range_of(r);
  using T = typename decltype(x)::value_type;
  const T s = static_cast<T>(start);
  const std::size_t g_first = (std::size_t)x.first.i;
  auto [p, c] = detail::local_span(x);
  const std::size_t g0 = c ? (std::size_t)(p - x.first.dv->owned()) + x.first.dv->first_index() : 0;
  auto f = [s, g_first](std::size_t g) { return static_cast<T>(s + static_cast<T>(g - g_first)); };
  if (c)
    hipLaunchKernelGGL((detail::gen_kernel<T, decltype(f)>), dim3(detail::grid_for(c)), dim3(detail::kThreads), 0,
                       detail::stream(), p, c, g0, f);
  barrier();
}
template <typename T, typename V> void iota(dv_iterator<T> first, dv_iterator<T> last, V start) {
  mhp::iota(dv_range<T>{first, last}, start);
}

// cpu_algorithms.hpp:63-81 for_each: op(element &) on every rank's local
// segment, then a barrier
template <vector_range R, typename Op> void for_each(R &&r, Op op) {
  auto x = range_of(r);
  using T = typename decltype(x)::value_type;
  auto [p, c] = detail::local_span(x);
  if (c)
    hipLaunchKernelGGL((detail::for_each_kernel<T, Op>), dim3(detail::grid_for(c)), dim3(detail::kThreads), 0,
                       detail::stream(), p, c, op);
  barrier();
}
template <typename A, typename B, typename Op> void for_each(const zip_range<A, B> &z, Op op) {
  if (!aligned(z)) throw std::runtime_error("mhp::for_each: zip of misaligned ranges (it has no segments)");
  const std::ptrdiff_t len = (std::ptrdiff_t)z.size();
  auto [pa, ca] = detail::local_span(dv_range<A>{z.a.first, z.a.first + len});
  auto [pb, cb] = detail::local_span(dv_range<B>{z.b.first, z.b.first + len});
  (void)cb;
  if (ca)
    hipLaunchKernelGGL((detail::for_each_zip_kernel<A, B, Op>), dim3(detail::grid_for(ca)), dim3(detail::kThreads), 0,
                       detail::stream(), pa, pb, ca, op);
  barrier();
}
template <typename T, typename Op> void for_each(dv_iterator<T> first, dv_iterator<T> last, Op op) {
  mhp::for_each(dv_range<T>{first, last}, op);
}

// cpu_algorithms.hpp:36-61 copy: aligned ranges copy their local segments;
// misaligned ones run ONE alltoallv of the owned pieces (the reference
// copies element by element through its MPI window, then fences)
template <vector_range R, typename U> void copy(R &&in_r, dv_iterator<U> out) {
  auto in = range_of(in_r);
  using T = typename decltype(in)::value_type;
  const std::size_t len = in.size();
  const dv_range<U> o{out, out + (std::ptrdiff_t)len};
  if (dr_plan::pieces_aligned(detail::pieces(in), detail::pieces(o))) {
    auto [pi, ci] = detail::local_span(in);
    auto [po, co] = detail::local_span(o);
    (void)co;
    const char *a0 = reinterpret_cast<const char *>(pi), *b0 = reinterpret_cast<const char *>(po);
    const bool overlap = ci && a0 < b0 + ci * sizeof(U) && b0 < a0 + ci * sizeof(T);
    if (ci && overlap && pi != (T *)po) {
      // overlapping pieces of one vector: through a staging buffer (a
      // device memcpy between overlapping ranges is undefined)
      detail::dev_buf<T> stage(ci);
      detail::check(drhip_memcpy_d2d(0, stage.p, pi, ci * sizeof(T)), "drhip_memcpy_d2d");
      detail::check(drhip_memcpy_d2d(0, po, stage.p, ci * sizeof(T)), "drhip_memcpy_d2d");
      detail::sync();
    } else if (ci && pi != (T *)po) {
      detail::check(drhip_memcpy_d2d(0, po, pi, ci * sizeof(T)), "drhip_memcpy_d2d");
    }
  } else if (len) {
    auto &dst = *out.dv;
    const bool same = (void *)in.first.dv == (void *)out.dv;
    if (!same) {
      detail::exchange_into(*in.first.dv, (std::size_t)in.first.i, (std::size_t)in.last.i, dst, (std::size_t)out.i,
                            dst.owned());
    } else {
      // overlapping source and destination in one vector: receive into a
      // staging copy of the owned segment, then copy the received slots back
      detail::dev_buf<U> stage(dst.segment_size());
      detail::exchange_into(*in.first.dv, (std::size_t)in.first.i, (std::size_t)in.last.i, dst, (std::size_t)out.i,
                            stage.p);
      auto [po, co] = detail::local_span(o);
      if (co)
        detail::check(drhip_memcpy_d2d(0, po, stage.p + (po - dst.owned()), co * sizeof(U)), "drhip_memcpy_d2d");
      detail::sync();
    }
  }
  barrier();
}
template <typename T, typename U> void copy(dv_iterator<T> first, dv_iterator<T> last, dv_iterator<U> out) {
  mhp::copy(dv_range<T>{first, last}, out);
}

template <typename T> std::vector<T> gather(distributed_vector<T> &dv, int root = 0);
template <typename T> std::vector<T> gather(const dv_range<T> &r, int root = 0);

// Collective host <-> distributed copies from / to `root` -- what the
// reference's tests do with std::copy through rank 0's window
// (test/gtest/mhp/distributed_vector.cpp:58-86): root's host elements
// [src, src + len) to global positions [out, out + len) (one alltoallv from
// root, into the owners' segments), and a range's elements to root's host
// memory (gather).
template <typename T> void copy(int root, const T *src, std::size_t len, dv_iterator<T> out) {
  auto &dv = *out.dv;
  const std::size_t p = nprocs(), me = rank();
  detail::dev_buf<T> stage((int)me == root ? len : 0);
  if ((int)me == root && len) detail::check(drhip_memcpy_h2d(0, stage.p, src, len * sizeof(T)), "drhip_memcpy_h2d");
  std::vector<std::size_t> sb(p, 0), so(p, 0), rb(p, 0), ro(p, 0);
  for (const auto &pc : dr_plan::range_pieces(dv.size(), dv.segment_size(), p, (std::size_t)out.i,
                                              (std::size_t)out.i + len)) {
    if ((int)me == root) {
      sb[pc.rank] = (pc.end - pc.begin) * sizeof(T);
      so[pc.rank] = (pc.begin - (std::size_t)out.i) * sizeof(T);
    }
    if (pc.rank == me) {
      rb[root] = (pc.end - pc.begin) * sizeof(T);
      ro[root] = (pc.begin - dv.first_index()) * sizeof(T);
    }
  }
  detail::sync();
  comm().alltoallv(stage.p, sb.data(), so.data(), dv.owned(), rb.data(), ro.data());
  barrier();
}
template <typename T> void copy(int root, const dv_range<T> &r, T *dst) {
  auto v = gather(r, root);
  if ((int)rank() == root) std::copy(v.begin(), v.end(), dst);
  barrier();
}

// cpu_algorithms.hpp:147-167 transform.  Aligned ranges: op gets a
// reference into the halo'd buffer (a stencil op reads its neighbours
// through the pointer).  Misaligned: the input elements are first moved to
// the output's owners (the copy's alltoallv, into a staging buffer), then
// op runs there -- values only, no neighbour access (the reference's
// serial fallback likewise applies op to single remote elements).
template <typename T, typename U, typename Op>
void transform(dv_iterator<T> first, dv_iterator<T> last, dv_iterator<U> out, Op op) {
  auto &in = *first.dv;
  auto &o = *out.dv;
  const std::size_t len = (std::size_t)(last - first);
  const dv_range<T> ri{first, last};
  const dv_range<U> ro{out, out + (std::ptrdiff_t)len};
  if (len && !dr_plan::pieces_aligned(detail::pieces(ri), detail::pieces(ro))) {
    detail::dev_buf<T> stage(o.segment_size());
    detail::exchange_into(in, (std::size_t)first.i, (std::size_t)last.i, o, (std::size_t)out.i,
                          reinterpret_cast<U *>(stage.p));
    auto [po, co] = detail::local_span(ro);
    if (co)
      hipLaunchKernelGGL((detail::transform_kernel<T, U, Op>), dim3(detail::grid_for(co)), dim3(detail::kThreads), 0,
                         detail::stream(), stage.p + (po - o.owned()), po, co, op);
    barrier();
    return;
  }
  auto [off, cnt] = detail::local_part(in, (std::size_t)first.i, (std::size_t)last.i);
  auto [ooff, ocnt] = detail::local_part(o, (std::size_t)out.i, (std::size_t)out.i + len);
  (void)ocnt;
  if (cnt)
    hipLaunchKernelGGL((detail::transform_kernel<T, U, Op>), dim3(detail::grid_for(cnt)), dim3(detail::kThreads), 0,
                       detail::stream(), in.owned() + off, o.owned() + ooff, cnt, op);
  barrier();
}
template <typename T, typename U, typename Op> void transform(const dv_range<T> &in, dv_iterator<U> out, Op op) {
  transform(in.first, in.last, out, op);
}
template <typename T, typename U, typename Op> void transform(distributed_vector<T> &in, dv_iterator<U> out, Op op) {
  transform(in.begin(), in.end(), out, op);
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
template <typename T, typename V, typename Op> V reduce(int root, distributed_vector<T> &dv, V init, Op op) {
  return reduce(root, dv.begin(), dv.end(), init, op);
}

// Collect the whole vector on `root` (other ranks get an empty vector): the
// check path of the reference tests (equal(v, dv) reads remote segments).
template <typename T> std::vector<T> gather(distributed_vector<T> &dv, int root) {
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
// a range's elements on root (collective)
template <typename T> std::vector<T> gather(const dv_range<T> &r, int root) {
  auto all = gather(*r.first.dv, root);
  if ((int)rank() != root) return {};
  return std::vector<T>(all.begin() + r.first.i, all.begin() + r.last.i);
}
// a transform view's values on root: the underlying elements gathered, f
// applied on the host (the reference's check reads the view element by
// element through its window)
template <typename T, typename F> auto gather(const transform_range<T, F> &t, int root = 0) {
  auto v = gather(t.r, root);
  std::vector<std::remove_cvref_t<decltype(t.f(std::declval<T &>()))>> out;
  for (auto &x : v) out.push_back(t.f(x));
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
