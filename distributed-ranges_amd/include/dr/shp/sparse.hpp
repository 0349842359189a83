// dr/shp/sparse.hpp -- shp::sparse_matrix (CSR tiles on a block-cyclic tile
// grid), shp::block_cyclic, shp::mmread and shp::gemv.
//
// Mirrors containers/sparse_matrix.hpp:126-353, containers/
// matrix_partition.hpp:13-86 and algorithms/gemv.hpp:13-71:
//   * tile (i, j) holds rows [i*tm, ...) x columns [j*tn, ...) as tile-local
//     CSR on the device block_cyclic assigns it (rowptr from 0, column
//     indices local to the tile); tiles() are views with tile-local
//     coordinates, segments() the same views carrying their global origin.
//   * sparse_matrix(shape, density[, partition]) generates the nonzeros on
//     each tile's own device (drhip_csr_gen_density).  The reference builds
//     every tile on the host from a std::map of all entries with density
//     ignored and seed 0 for every tile (sparse_matrix.hpp:306,
//     generate_random.hpp:29-90; it cannot reach the 2^26-row benchmark).
//     Here floor(density*m*n) entries are spread evenly over rows; with a
//     {P, 1} grid the matrix is defined globally, so it is the same for any
//     device count.
//   * sparse_matrix(shape, csr_kind, k, seed): the C4 benchmark matrices
//     (banded offsets -4..+5 or k random columns per row, float / int32).
//   * sparse_matrix(shape, rowptr, colind, values[, partition]) and
//     mmread(path[, partition]) (Matrix Market coordinate files) build the
//     tiles from host CSR.
//   * iterating a sparse_matrix yields matrix_entry {index, value} in tile
//     order with global indices (sparse_matrix.hpp:15-121); here it walks a
//     host snapshot of the device tiles (read-only).
//
// gemv(c, a, b) computes the INTENDED c += A * b (the
// reference reads colind from rowptr, sparse_matrix.hpp:187, and
// accumulates with a racy non-atomic +=, gemv.hpp:62).  It requires a
// {P, 1} tile grid (gemv.hpp:21).  The reference replicates b whole to
// every tile's device before the tile SpMV (gemv.hpp:30-42); here each tile
// receives only the window of b its columns span (column_range: the rows'
// +-5 band for banded C4, all of b for a random matrix), by
// device-to-device (xGMI peer) copies of the overlapping parts of b's
// segments, and the SpMV reads it through a base shifted by the window's
// first column.  float / double values with 4- or 8-byte
// indices run the C-ABI kernel (drhip_spmv_csr); any other value type runs
// a one-row-per-thread template kernel compiled in the caller's TU.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <limits>
#include <memory>
#include <sstream>
#include <string>
#include <tuple>
#include <vector>

#include "algorithms.hpp"
#include "index.hpp"

namespace shp {

namespace tile {
// matrix_partition.hpp:15-20: {ceil(m / p_m), ceil(n / p_n)} tiles
inline constexpr std::size_t div = std::numeric_limits<std::size_t>::max();
} // namespace tile

namespace detail {
// containers/detail.hpp:13-24: n = p*q, p >= q, as square as possible
inline index<> factor(std::size_t n) {
  std::size_t q = static_cast<std::size_t>(std::sqrt(static_cast<double>(n)));
  while (q > 1 && n % q != 0) q--;
  if (q == 0) q = 1;
  return {n / q, q};
}
template <typename I> constexpr int index_code() {
  static_assert(std::is_integral_v<I> && (sizeof(I) == 4 || sizeof(I) == 8), "4- or 8-byte index type");
  return sizeof(I) == 4 ? DRHIP_I32 : DRHIP_I64;
}
} // namespace detail

// matrix_partition.hpp:22-31
class matrix_partition {
public:
  virtual std::size_t tile_rank(index<> matrix_shape, index<> tile_id) const = 0;
  virtual index<> grid_shape(index<> matrix_shape) const = 0;
  virtual index<> tile_shape(index<> matrix_shape) const = 0;
  virtual std::unique_ptr<matrix_partition> clone() const = 0;
  virtual ~matrix_partition() = default;
};

// matrix_partition.hpp:33-86.  grid_shape is the processor grid; tile (i, j)
// goes to processor (i mod g0, j mod g1), i.e. rank (i mod g0)*g1 + (j mod
// g1) (taken mod nprocs()).  With tile::div the tile grid equals the
// processor grid; with an explicit tile shape the tile grid is whatever
// covers the matrix (the reference keeps the processor grid there, which
// leaves part of the matrix untiled) and tiles are dealt cyclically.
class block_cyclic final : public matrix_partition {
public:
  block_cyclic(index<> tile_shape = {tile::div, tile::div}, index<> grid_shape = detail::factor(nprocs()))
      : tile_shape_(tile_shape), grid_shape_(grid_shape) {
    if (grid_shape_[0] == 0 || grid_shape_[1] == 0) throw std::runtime_error("block_cyclic: empty processor grid");
  }

  index<> tile_shape() const { return tile_shape_; }

  std::size_t tile_rank(index<>, index<> tile_id) const override {
    return ((tile_id[0] % grid_shape_[0]) * grid_shape_[1] + tile_id[1] % grid_shape_[1]) % nprocs();
  }
  index<> tile_shape(index<> shape) const override {
    std::size_t t[2] = {tile_shape_[0], tile_shape_[1]};
    for (int d = 0; d < 2; d++)
      if (t[d] == tile::div) t[d] = std::max<std::size_t>(1, (shape[d] + grid_shape_[d] - 1) / grid_shape_[d]);
    return {t[0], t[1]};
  }
  index<> grid_shape(index<> shape) const override {
    const index<> t = tile_shape(shape);
    return {std::max<std::size_t>(1, (shape[0] + t[0] - 1) / t[0]),
            std::max<std::size_t>(1, (shape[1] + t[1] - 1) / t[1])};
  }
  std::unique_ptr<matrix_partition> clone() const override { return std::make_unique<block_cyclic>(*this); }

private:
  index<> tile_shape_;
  index<> grid_shape_;
};

// containers/matrix_entry.hpp: {index, value}, tuple-like for
// `auto &&[idx, v] = entry`.
template <typename T, typename I = std::size_t> class matrix_entry {
public:
  using value_type = T;
  using index_type = I;
  matrix_entry() = default;
  matrix_entry(index<I> idx, T v) : index_(idx), value_(v) {}
  index<I> index() const noexcept { return index_; }
  T value() const noexcept { return value_; }
  template <std::size_t N>
    requires(N <= 1)
  auto get() const noexcept {
    if constexpr (N == 0) return index_;
    else return value_;
  }
  bool operator==(const matrix_entry &) const = default;

private:
  shp::index<I> index_;
  T value_{};
};

} // namespace shp

namespace std {
template <typename T, typename I> struct tuple_size<shp::matrix_entry<T, I>> : integral_constant<std::size_t, 2> {};
template <typename T, typename I> struct tuple_element<0, shp::matrix_entry<T, I>> {
  using type = shp::index<I>;
};
template <typename T, typename I> struct tuple_element<1, shp::matrix_entry<T, I>> {
  using type = T;
};
} // namespace std

namespace shp {

// views/csr_matrix_view.hpp:13-185: a tile's device CSR arrays, its shape,
// nonzero count, device rank and global origin.
namespace detail {
inline bool check_columns() {
  static const bool on = [] {
    const char *e = std::getenv("DRHIP_CHECK_COLUMNS");
    return e && e[0] == '1';
  }();
  return on;
}
} // namespace detail

namespace detail {
template <typename I> __global__ void widen_indices_kernel(const std::int32_t *in, I *out, std::size_t n) {
  const std::size_t i = static_cast<std::size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) out[i] = static_cast<I>(static_cast<std::uint32_t>(in[i])); // indices are >= 0
}
// out[i] = in[i] on segment rank's stream (asynchronous)
template <typename I> void widen_indices(int rank, const std::int32_t *in, I *out, std::size_t n) {
  if (!n) return;
  hipLaunchKernelGGL((widen_indices_kernel<I>), dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0,
                     stream(static_cast<std::size_t>(rank)), in, out, n);
  hip_check(hipGetLastError(), "widen_indices launch");
}
} // namespace detail

template <typename T, typename I> class csr_matrix_view {
public:
  using value_type = T;
  using index_type = I;
  csr_matrix_view() = default;
  csr_matrix_view(T *values, I *rowptr, I *colind, index<> shape, std::size_t nnz, std::size_t rank,
                  index<> origin = {0, 0})
      : values_(values), rowptr_(rowptr), colind_(colind), shape_(shape), nnz_(nnz), rank_(rank), origin_(origin) {}

  index<> shape() const noexcept { return shape_; }
  std::size_t size() const noexcept { return nnz_; }
  std::size_t rank() const noexcept { return rank_; }
  index<> origin() const noexcept { return origin_; }
  T *values_data() const { return values_; }
  I *rowptr_data() const { return rowptr_; }
  I *colind_data() const { return colind_; }

  // host copy of the tile's entries, indices offset by origin()
  std::vector<matrix_entry<T>> entries() const {
    std::vector<I> rp(shape_[0] + 1), ci(nnz_);
    std::vector<T> va(nnz_);
    const int rk = static_cast<int>(rank_);
    detail::check(drhip_memcpy_d2h(rk, rp.data(), rowptr_, rp.size() * sizeof(I)), "csr view d2h");
    if (nnz_) {
      detail::check(drhip_memcpy_d2h(rk, ci.data(), colind_, nnz_ * sizeof(I)), "csr view d2h");
      detail::check(drhip_memcpy_d2h(rk, va.data(), values_, nnz_ * sizeof(T)), "csr view d2h");
    }
    std::vector<matrix_entry<T>> out;
    out.reserve(nnz_);
    for (std::size_t r = 0; r < shape_[0]; r++)
      for (std::size_t k = static_cast<std::size_t>(rp[r]); k < static_cast<std::size_t>(rp[r + 1]); k++)
        out.emplace_back(index<>{origin_[0] + r, origin_[1] + static_cast<std::size_t>(ci[k])}, va[k]);
    return out;
  }

private:
  T *values_ = nullptr;
  I *rowptr_ = nullptr;
  I *colind_ = nullptr;
  index<> shape_{0, 0};
  std::size_t nnz_ = 0, rank_ = 0;
  index<> origin_{0, 0};
};

enum class csr_kind : int { banded = 0, random = 1 };

template <typename T, typename I = std::size_t> class sparse_matrix {
public:
  using value_type = T;
  using index_type = I;
  using size_type = std::size_t;
  using key_type = index<>;
  using segment_type = csr_matrix_view<T, I>;
  using entry_type = matrix_entry<T>;

  // sparse_matrix.hpp:152-175
  explicit sparse_matrix(key_type shape) : sparse_matrix(shape, block_cyclic()) {}
  sparse_matrix(key_type shape, double density, std::uint64_t seed = 0)
      : sparse_matrix(shape, density, block_cyclic(), seed) {}
  sparse_matrix(key_type shape, double density, const matrix_partition &partition, std::uint64_t seed = 0)
      : shape_(shape), partition_(partition.clone()) {
    static_assert(detail::abi_type<T>, "device generator: int32/uint32/int64/uint64/float/double values");
    layout();
    const bool global_rows = grid_shape_[1] == 1; // {P, 1}: one matrix for any P
    for (std::size_t t = 0; t < store_.size(); t++) {
      auto &s = store_[t];
      const std::size_t ti = t / grid_shape_[1];
      const std::size_t r0 = global_rows ? ti * tile_shape_[0] : 0;
      const std::size_t m = global_rows ? shape_[0] : s.shape[0];
      const std::uint64_t sd = global_rows ? seed : seed + t;
      std::size_t nnz = 0;
      detail::check(drhip_csr_density_nnz(r0, s.shape[0], m, s.shape[1] ? s.shape[1] : 1, density, &nnz),
                    "drhip_csr_density_nnz");
      if (s.shape[1] == 0) nnz = 0;
      alloc(s, nnz);
      if (s.shape[1] == 0) {
        zero_rowptr(s);
        continue;
      }
      detail::check(drhip_csr_gen_density(static_cast<int>(s.rank), detail::dtype_code<T>(), detail::index_code<I>(),
                                          r0, s.shape[0], m, s.shape[1], density, sd, s.rowptr, s.colind, s.values),
                    "drhip_csr_gen_density");
    }
    sync_all();
  }
  // empty matrix on the partition's tiles (sparse_matrix.hpp:168-175)
  sparse_matrix(key_type shape, const matrix_partition &partition) : shape_(shape), partition_(partition.clone()) {
    layout();
    for (auto &s : store_) {
      alloc(s, 0);
      zero_rowptr(s);
    }
    sync_all();
  }

  // C4 benchmark matrices, generated on each {P, 1} row tile's device:
  // banded (10 diagonals at offsets -4..+5, clipped) or `k` random distinct
  // sorted columns per row.  Identical to oracle.c's generators.  Float
  // values; int32 indices, or 8-byte ones (the reference's default I =
  // std::size_t, sparse_matrix.hpp:126): generated as int32 in scratch and
  // widened on the device.
  sparse_matrix(key_type shape, csr_kind kind, int k = 10, std::uint64_t seed = 1)
      : shape_(shape), partition_(block_cyclic({tile::div, tile::div}, {nprocs(), 1}).clone()) {
    static_assert(std::is_same_v<T, float> && std::is_integral_v<I> && (sizeof(I) == 4 || sizeof(I) == 8),
                  "benchmark generator: float values, 4- or 8-byte indices");
    layout();
    for (auto &s : store_) {
      const std::size_t r0 = s.origin[0];
      std::size_t nnz = 0;
      detail::check(drhip_csr_nnz(static_cast<int>(kind), r0, s.shape[0], shape_[1], k, &nnz), "drhip_csr_nnz");
      if (nnz > static_cast<std::size_t>(std::numeric_limits<std::int32_t>::max()))
        throw std::runtime_error("sparse_matrix: benchmark tile above 2^31 nonzeros");
      alloc(s, nnz);
      const int rk = static_cast<int>(s.rank);
      if constexpr (sizeof(I) == 4) {
        detail::check(drhip_csr_gen(rk, static_cast<int>(kind), r0, s.shape[0], shape_[1], k, seed, s.rowptr, s.colind,
                                    s.values),
                      "drhip_csr_gen");
      } else {
        void *rp32 = nullptr, *ci32 = nullptr;
        detail::check(drhip_malloc(rk, (s.shape[0] + 1) * 4, &rp32), "drhip_malloc");
        detail::check(drhip_malloc(rk, std::max<std::size_t>(nnz, 1) * 4, &ci32), "drhip_malloc");
        detail::check(drhip_csr_gen(rk, static_cast<int>(kind), r0, s.shape[0], shape_[1], k, seed, rp32, ci32, s.values),
                      "drhip_csr_gen");
        detail::widen_indices(rk, static_cast<const std::int32_t *>(rp32), s.rowptr, s.shape[0] + 1);
        detail::widen_indices(rk, static_cast<const std::int32_t *>(ci32), s.colind, nnz);
        sync(s.rank);
        detail::check(drhip_free(rk, rp32), "drhip_free");
        detail::check(drhip_free(rk, ci32), "drhip_free");
      }
    }
    sync_all();
  }

  // From host CSR arrays of the whole matrix (global rowptr of m+1 entries,
  // global column indices), cut into the partition's tiles.
  sparse_matrix(key_type shape, const std::vector<I> &rowptr, const std::vector<I> &colind,
                const std::vector<T> &values, const matrix_partition &partition)
      : shape_(shape), partition_(partition.clone()) {
    if (rowptr.size() != shape_[0] + 1 || colind.size() != values.size() ||
        static_cast<std::size_t>(rowptr.back()) != colind.size())
      throw std::runtime_error("sparse_matrix: inconsistent CSR arrays");
    layout();
    for (auto &s : store_) {
      std::vector<I> rp(s.shape[0] + 1), ci;
      std::vector<T> va;
      rp[0] = 0;
      const std::size_t c0 = s.origin[1], c1 = c0 + s.shape[1];
      for (std::size_t r = 0; r < s.shape[0]; r++) {
        const std::size_t g = s.origin[0] + r;
        for (auto k = static_cast<std::size_t>(rowptr[g]); k < static_cast<std::size_t>(rowptr[g + 1]); k++) {
          const auto c = static_cast<std::size_t>(colind[k]);
          if (c >= shape_[1]) throw std::runtime_error("sparse_matrix: column index out of range");
          if (c >= c0 && c < c1) {
            ci.push_back(static_cast<I>(c - c0));
            va.push_back(values[k]);
          }
        }
        rp[r + 1] = static_cast<I>(ci.size());
      }
      alloc(s, ci.size());
      const int rk = static_cast<int>(s.rank);
      detail::check(drhip_memcpy_h2d(rk, s.rowptr, rp.data(), rp.size() * sizeof(I)), "h2d");
      if (s.nnz) {
        detail::check(drhip_memcpy_h2d(rk, s.colind, ci.data(), s.nnz * sizeof(I)), "h2d");
        detail::check(drhip_memcpy_h2d(rk, s.values, va.data(), s.nnz * sizeof(T)), "h2d");
      }
    }
    sync_all();
  }
  sparse_matrix(key_type shape, const std::vector<I> &rowptr, const std::vector<I> &colind,
                const std::vector<T> &values)
      : sparse_matrix(shape, rowptr, colind, values, block_cyclic({tile::div, tile::div}, {nprocs(), 1})) {}

  sparse_matrix(const sparse_matrix &) = delete;
  sparse_matrix &operator=(const sparse_matrix &) = delete;
  sparse_matrix(sparse_matrix &&o) noexcept { *this = std::move(o); }
  sparse_matrix &operator=(sparse_matrix &&o) noexcept {
    if (this != &o) {
      release();
      shape_ = o.shape_;
      tile_shape_ = o.tile_shape_;
      grid_shape_ = o.grid_shape_;
      partition_ = std::move(o.partition_);
      store_ = std::move(o.store_);
      snapshot_ = std::move(o.snapshot_);
      have_snapshot_ = o.have_snapshot_;
      o.store_.clear();
    }
    return *this;
  }
  ~sparse_matrix() { release(); }

  size_type size() const noexcept { // sparse_matrix.hpp:173
    std::size_t s = 0;
    for (auto &t : store_) s += t.nnz;
    return s;
  }
  key_type shape() const noexcept { return shape_; }
  key_type tile_shape() const noexcept { return tile_shape_; }
  key_type grid_shape() const noexcept { return grid_shape_; }
  const matrix_partition &partition() const { return *partition_; }

  // sparse_matrix.hpp:183-197 (with colind read from colind, not rowptr)
  segment_type tile(key_type tile_index) const {
    const auto &s = store_.at(tile_index[0] * grid_shape_[1] + tile_index[1]);
    return segment_type(s.values, s.rowptr, s.colind, s.shape, s.nnz, s.rank);
  }
  std::vector<segment_type> tiles() const {
    std::vector<segment_type> v;
    for (auto &s : store_) v.emplace_back(s.values, s.rowptr, s.colind, s.shape, s.nnz, s.rank);
    return v;
  }
  std::vector<segment_type> segments() const {
    std::vector<segment_type> v;
    for (auto &s : store_) v.emplace_back(s.values, s.rowptr, s.colind, s.shape, s.nnz, s.rank, s.origin);
    return v;
  }

  // The columns tile k reads: [lo, hi) of its tile-local column indices
  // (min and max of colind, two drhip_reduce calls on the tile's device,
  // computed once and cached; {0, 0} for an empty tile).  gemv replicates
  // only this window of b to the tile's device: +-5 columns around the rows
  // for the banded C4 matrix, everything for a random one.
  // The cache assumes the tiles' column indices are not rewritten after the
  // first gemv (colind_data() hands out the device pointer, as the
  // reference's view does): a caller that rewrites them calls
  // columns_changed().  DRHIP_CHECK_COLUMNS=1 makes every gemv recompute
  // the range and throw if a column left the cached window.
  std::pair<std::size_t, std::size_t> column_range(std::size_t k) const {
    auto &s = store_.at(k);
    if (s.cols_known && detail::check_columns()) {
      const auto cached = std::pair{s.col_lo, s.col_hi};
      s.cols_known = false;
      const auto now = column_range(k);
      if (now.first < cached.first || now.second > cached.second)
        throw std::runtime_error("shp::sparse_matrix: column indices changed after the first gemv; call "
                                 "columns_changed()");
    }
    if (!s.cols_known) {
      s.col_lo = s.col_hi = 0;
      if (s.nnz) {
        detail::pinned<I> mm(2);
        const int rk = static_cast<int>(s.rank);
        detail::check(drhip_reduce(rk, detail::index_code<I>(), DRHIP_MIN, s.colind, s.nnz, &mm[0]), "colind min");
        detail::check(drhip_reduce(rk, detail::index_code<I>(), DRHIP_MAX, s.colind, s.nnz, &mm[1]), "colind max");
        sync(s.rank);
        s.col_lo = static_cast<std::size_t>(mm[0]);
        s.col_hi = static_cast<std::size_t>(mm[1]) + 1;
      }
      s.cols_known = true;
    }
    return {s.col_lo, s.col_hi};
  }

  // forget the cached column ranges (after rewriting colind on the device)
  void columns_changed() {
    for (auto &s : store_) s.cols_known = false;
    have_snapshot_ = false;
  }

  // entries in tile order, global indices (host snapshot, read-only)
  auto begin() const {
    snapshot();
    return snapshot_.cbegin();
  }
  auto end() const {
    snapshot();
    return snapshot_.cend();
  }

private:
  struct store {
    std::size_t rank = 0;
    index<> shape{0, 0}, origin{0, 0};
    std::size_t nnz = 0;
    I *rowptr = nullptr;
    I *colind = nullptr;
    T *values = nullptr;
    mutable std::size_t col_lo = 0, col_hi = 0; // column_range cache
    mutable bool cols_known = false;
  };

  void layout() {
    grid_shape_ = partition_->grid_shape(shape_);
    tile_shape_ = partition_->tile_shape(shape_);
    for (std::size_t i = 0; i < grid_shape_[0]; i++)
      for (std::size_t j = 0; j < grid_shape_[1]; j++) {
        store s;
        s.rank = partition_->tile_rank(shape_, {i, j});
        s.origin = {std::min(shape_[0], i * tile_shape_[0]), std::min(shape_[1], j * tile_shape_[1])};
        s.shape = {std::min(tile_shape_[0], shape_[0] - s.origin[0]), std::min(tile_shape_[1], shape_[1] - s.origin[1])};
        store_.push_back(s);
      }
  }
  void alloc(store &s, std::size_t nnz) {
    if (nnz > static_cast<std::size_t>(std::numeric_limits<I>::max()))
      throw std::runtime_error("sparse_matrix: tile nonzeros exceed the index type");
    const int rk = static_cast<int>(s.rank);
    s.nnz = nnz;
    void *p = nullptr;
    detail::check(drhip_malloc(rk, (s.shape[0] + 1) * sizeof(I), &p), "drhip_malloc");
    s.rowptr = static_cast<I *>(p);
    detail::check(drhip_malloc(rk, std::max<std::size_t>(nnz, 1) * sizeof(I), &p), "drhip_malloc");
    s.colind = static_cast<I *>(p);
    detail::check(drhip_malloc(rk, std::max<std::size_t>(nnz, 1) * sizeof(T), &p), "drhip_malloc");
    s.values = static_cast<T *>(p);
  }
  void zero_rowptr(store &s) {
    const I zero = 0;
    detail::check(drhip_fill(static_cast<int>(s.rank), s.rowptr, s.shape[0] + 1, &zero, sizeof(I)), "drhip_fill");
  }
  void release() {
    for (auto &s : store_) {
      const int rk = static_cast<int>(s.rank);
      (void)drhip_free(rk, s.rowptr);
      (void)drhip_free(rk, s.colind);
      (void)drhip_free(rk, s.values);
    }
    store_.clear();
  }
  void snapshot() const {
    if (have_snapshot_) return;
    snapshot_.clear();
    for (auto &v : segments()) {
      auto e = v.entries();
      snapshot_.insert(snapshot_.end(), e.begin(), e.end());
    }
    have_snapshot_ = true;
  }

  key_type shape_{0, 0}, tile_shape_{0, 0}, grid_shape_{0, 0};
  std::unique_ptr<matrix_partition> partition_;
  std::vector<store> store_;
  mutable std::vector<entry_type> snapshot_;
  mutable bool have_snapshot_ = false;
};

// ------------------------------------------------------------------ mmread
// Matrix Market coordinate reader (real / integer / pattern; general /
// symmetric / skew-symmetric), 1-indexed entries by default.  Duplicate
// entries are summed; the result is cut into the partition's tiles.
template <typename T, typename I = std::size_t>
sparse_matrix<T, I> mmread(const std::string &path,
                           const matrix_partition &partition = block_cyclic({tile::div, tile::div}, {nprocs(), 1}),
                           bool one_indexed = true) {
  std::ifstream f(path);
  if (!f) throw std::runtime_error("mmread: cannot open " + path);
  std::string line;
  if (!std::getline(f, line)) throw std::runtime_error("mmread: empty file");
  std::string banner, object, format, field, symmetry;
  {
    std::istringstream h(line);
    h >> banner >> object >> format >> field >> symmetry;
  }
  auto lower = [](std::string s) {
    for (auto &c : s) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
    return s;
  };
  object = lower(object), format = lower(format), field = lower(field), symmetry = lower(symmetry);
  if (banner != "%%MatrixMarket" || object != "matrix" || format != "coordinate")
    throw std::runtime_error("mmread: only '%%MatrixMarket matrix coordinate' files");
  if (field != "real" && field != "integer" && field != "pattern" && field != "double")
    throw std::runtime_error("mmread: field must be real, integer or pattern");
  const bool sym = symmetry == "symmetric", skew = symmetry == "skew-symmetric";
  if (!sym && !skew && symmetry != "general") throw std::runtime_error("mmread: unsupported symmetry " + symmetry);
  while (std::getline(f, line))
    if (!line.empty() && line[0] != '%') break;
  std::size_t m = 0, n = 0, nz = 0;
  {
    std::istringstream h(line);
    if (!(h >> m >> n >> nz)) throw std::runtime_error("mmread: bad size line");
  }
  std::vector<std::tuple<std::size_t, std::size_t, T>> e;
  e.reserve(sym || skew ? 2 * nz : nz);
  const std::size_t base = one_indexed ? 1 : 0;
  for (std::size_t k = 0; k < nz; k++) {
    if (!std::getline(f, line)) throw std::runtime_error("mmread: truncated entries");
    if (line.empty() || line[0] == '%') {
      k--;
      continue;
    }
    std::istringstream h(line);
    std::size_t i, j;
    double v = 1.0;
    if (!(h >> i >> j)) throw std::runtime_error("mmread: bad entry line");
    if (field != "pattern" && !(h >> v)) throw std::runtime_error("mmread: missing value");
    if (i < base || j < base || i - base >= m || j - base >= n) throw std::runtime_error("mmread: index out of range");
    i -= base, j -= base;
    e.emplace_back(i, j, static_cast<T>(v));
    if ((sym || skew) && i != j) e.emplace_back(j, i, static_cast<T>(skew ? -v : v));
  }
  std::sort(e.begin(), e.end(), [](const auto &a, const auto &b) {
    return std::get<0>(a) != std::get<0>(b) ? std::get<0>(a) < std::get<0>(b) : std::get<1>(a) < std::get<1>(b);
  });
  std::vector<I> rowptr(m + 1, 0), colind;
  std::vector<T> values;
  for (std::size_t k = 0; k < e.size(); k++) {
    const auto [i, j, v] = e[k];
    if (!colind.empty() && k > 0 && std::get<0>(e[k - 1]) == i && std::get<1>(e[k - 1]) == j) {
      values.back() += v; // duplicate entry
      continue;
    }
    colind.push_back(static_cast<I>(j));
    values.push_back(v);
    rowptr[i + 1]++;
  }
  for (std::size_t r = 0; r < m; r++) rowptr[r + 1] += rowptr[r];
  return sparse_matrix<T, I>({m, n}, rowptr, colind, values, partition);
}

// ------------------------------------------------------------------- gemv
namespace detail {
// one owner per row: c[r] = c[r] + v0*b[j0] + v1*b[j1] + ... (the
// reference's per-nonzero `c_v += a_v * b_v` order, gemv.hpp:58-63)
template <typename T, typename I, typename BT, typename CT>
__global__ void gemv_rows_kernel(std::size_t rows, const I *rowptr, const I *colind, const T *vals, const BT *b,
                                 CT *c) {
  const std::size_t r = static_cast<std::size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  CT acc = c[r];
  for (I k = rowptr[r]; k < rowptr[r + 1]; k++) acc += vals[k] * b[colind[k]];
  c[r] = acc;
}
} // namespace detail

// gemv.hpp:13-71 (intended semantics): c += a * b.
template <typename C, typename T, typename I, typename B>
  requires lib::distributed_contiguous_range<C> && lib::distributed_contiguous_range<B>
void gemv(C &&c, const sparse_matrix<T, I> &a, B &&b) {
  const auto m = a.shape()[0], n = a.shape()[1];
  if (a.grid_shape()[1] != 1) throw std::runtime_error("shp::gemv: needs a {P, 1} tile grid (gemv.hpp:21)");
  if (std::ranges::size(c) != m || std::ranges::size(b) != n)
    throw std::runtime_error("shp::gemv: shape mismatch"); // gemv.hpp:18-21
  using BT = std::ranges::range_value_t<B>;
  using CT = std::ranges::range_value_t<C>;
  constexpr bool abi = (std::is_same_v<T, float> || std::is_same_v<T, double>) && std::is_same_v<BT, T> &&
                       std::is_same_v<CT, T> && std::is_integral_v<I> && (sizeof(I) == 4 || sizeof(I) == 8);
  auto bsegs = lib::ranges::segments(b);
  auto csegs = lib::ranges::segments(c);
  const auto tiles = a.segments();
  // every tile's window of b on its device (peer copies of the parts of
  // b's segments that overlap the tile's column range)
  std::vector<void *> local_b(tiles.size(), nullptr);
  std::vector<std::size_t> lo_b(tiles.size(), 0);
  for (std::size_t k = 0; k < tiles.size(); k++) {
    const auto &t = tiles[k];
    if (!t.shape()[0] || !t.size()) continue;
    const auto [lo, hi] = a.column_range(k);
    lo_b[k] = lo;
    detail::check(drhip_malloc(static_cast<int>(t.rank()), std::max<std::size_t>(hi - lo, 1) * sizeof(BT), &local_b[k]),
                  "drhip_malloc");
    std::size_t off = 0;
    for (auto &s : bsegs) {
      const std::size_t a0 = std::max(off, lo), a1 = std::min(off + s.size(), hi);
      if (a0 < a1)
        detail::check(drhip_memcpy_d2d(static_cast<int>(t.rank()), static_cast<BT *>(local_b[k]) + (a0 - lo),
                                       s.data() + (a0 - off), (a1 - a0) * sizeof(BT)),
                      "gemv b copy");
      off += s.size();
    }
  }
  // every tile's row range must lie inside one segment of c
  std::size_t ci = 0, crow = 0;
  for (std::size_t k = 0; k < tiles.size(); k++) {
    const auto &t = tiles[k];
    const std::size_t rows = t.shape()[0], row0 = t.origin()[0];
    if (!rows || !t.size()) continue; // no nonzeros: c += 0
    while (crow + csegs[ci].size() <= row0) crow += csegs[ci++].size();
    if (row0 + rows > crow + csegs[ci].size() || lib::ranges::rank(csegs[ci]) != t.rank())
      throw std::runtime_error("shp::gemv: c is not partitioned like a's row tiles");
    CT *cp = csegs[ci].data() + (row0 - crow);
    const int rk = static_cast<int>(t.rank());
    // b[j] for j in the window sits at local_b[k][j - lo]: the kernels index
    // this shifted base with the tile's own column indices (all >= lo)
    const BT *bw = reinterpret_cast<const BT *>(reinterpret_cast<std::uintptr_t>(local_b[k]) -
                                                 lo_b[k] * sizeof(BT));
    if constexpr (abi) {
      detail::check(drhip_spmv_csr(rk, detail::dtype_code<T>(), detail::index_code<I>(), rows, t.size(),
                                   t.rowptr_data(), t.colind_data(), t.values_data(), bw, cp),
                    "drhip_spmv_csr");
    } else {
      hipLaunchKernelGGL((detail::gemv_rows_kernel<T, I, BT, CT>), dim3((unsigned)((rows + 255) / 256)), dim3(256), 0,
                         stream(t.rank()), rows, t.rowptr_data(), t.colind_data(), t.values_data(), bw, cp);
      detail::hip_check(hipGetLastError(), "gemv launch");
    }
  }
  sync_all();
  for (std::size_t k = 0; k < local_b.size(); k++)
    if (local_b[k]) detail::check(drhip_free(static_cast<int>(tiles[k].rank()), local_b[k]), "drhip_free");
}

} // namespace shp
