// dr/shp/sparse.hpp -- shp::sparse_matrix (CSR row tiles, one per segment)
// and shp::gemv.
//
// Mirrors containers/sparse_matrix.hpp:126-353 with the {P, 1} tile grid
// gemv requires (algorithms/gemv.hpp:21): tile k holds rows
// [k*ceil(m/P), min((k+1)*ceil(m/P), m)) on segment k as tile-local CSR
// (rowptr starting at 0, global column indices).  The reference builds its
// random matrix on the host from a std::map of every nonzero
// (util/generate_random.hpp:29-90), which cannot reach the 2^26-row
// benchmark; here tiles are generated on their own device
// (drhip_csr_gen: banded or k random distinct sorted columns per row), or
// copied from host CSR arrays.
//
// gemv(c, a, b) computes the INTENDED c += A * b (the
// reference reads colind from rowptr, sparse_matrix.hpp:187, and
// accumulates with a racy non-atomic +=, gemv.hpp:62).  b is replicated
// whole to every segment before the tile SpMV (gemv.hpp:30-42), by
// device-to-device (xGMI peer) copies of b's segments.
#pragma once

#include <cstdint>
#include <vector>

#include "algorithms.hpp"

namespace shp {

enum class csr_kind : int { banded = 0, random = 1 };

template <typename T, typename I = std::int32_t> class sparse_matrix {
public:
  using value_type = T;
  using index_type = I;

  struct tile {
    std::size_t rank = 0;
    std::size_t row0 = 0, rows = 0, nnz = 0;
    I *rowptr = nullptr;
    I *colind = nullptr;
    T *values = nullptr;
  };

  // Device-generated synthetic matrix (float values, int32 indices):
  // banded (10 diagonals at offsets -4..+5, clipped) or `k` random distinct
  // sorted columns per row.  Identical to oracle.c's generators.
  sparse_matrix(std::pair<std::size_t, std::size_t> shape, csr_kind kind, int k = 10, std::uint64_t seed = 1)
      : m_(shape.first), n_(shape.second) {
    static_assert(std::is_same_v<T, float> && std::is_same_v<I, std::int32_t>,
                  "device generator: float values, int32 indices");
    partition();
    for (auto &t : tiles_) {
      std::size_t nnz = 0;
      detail::check(drhip_csr_nnz(static_cast<int>(kind), t.row0, t.rows, n_, k, &nnz), "drhip_csr_nnz");
      alloc(t, nnz);
      detail::check(drhip_csr_gen(static_cast<int>(t.rank), static_cast<int>(kind), t.row0, t.rows, n_, k, seed,
                                  t.rowptr, t.colind, t.values),
                    "drhip_csr_gen");
    }
    sync_all();
  }

  // From host CSR arrays of the whole matrix (global rowptr of m+1 entries).
  sparse_matrix(std::pair<std::size_t, std::size_t> shape, const std::vector<I> &rowptr, const std::vector<I> &colind,
                const std::vector<T> &values)
      : m_(shape.first), n_(shape.second) {
    partition();
    for (auto &t : tiles_) {
      const std::size_t b = static_cast<std::size_t>(rowptr[t.row0]);
      const std::size_t e = static_cast<std::size_t>(rowptr[t.row0 + t.rows]);
      alloc(t, e - b);
      std::vector<I> rp(t.rows + 1);
      for (std::size_t r = 0; r <= t.rows; r++) rp[r] = static_cast<I>(rowptr[t.row0 + r] - static_cast<I>(b));
      const int rk = static_cast<int>(t.rank);
      detail::check(drhip_memcpy_h2d(rk, t.rowptr, rp.data(), rp.size() * sizeof(I)), "h2d");
      if (t.nnz) {
        detail::check(drhip_memcpy_h2d(rk, t.colind, colind.data() + b, t.nnz * sizeof(I)), "h2d");
        detail::check(drhip_memcpy_h2d(rk, t.values, values.data() + b, t.nnz * sizeof(T)), "h2d");
      }
    }
    sync_all();
  }

  sparse_matrix(const sparse_matrix &) = delete;
  sparse_matrix &operator=(const sparse_matrix &) = delete;
  ~sparse_matrix() {
    for (auto &t : tiles_) {
      const int rk = static_cast<int>(t.rank);
      (void)drhip_free(rk, t.rowptr);
      (void)drhip_free(rk, t.colind);
      (void)drhip_free(rk, t.values);
    }
  }

  std::pair<std::size_t, std::size_t> shape() const { return {m_, n_}; }
  std::size_t size() const { // nonzeros (sparse_matrix.hpp:150)
    std::size_t s = 0;
    for (auto &t : tiles_) s += t.nnz;
    return s;
  }
  // {P, 1} grid: the reference's grid_shape() (sparse_matrix.hpp:163)
  std::pair<std::size_t, std::size_t> grid_shape() const { return {tiles_.size(), 1}; }
  const tile &tile_at(std::size_t k) const { return tiles_[k]; }
  const std::vector<tile> &tiles() const { return tiles_; }

private:
  void partition() {
    const std::size_t p = nprocs();
    const std::size_t rs = std::max<std::size_t>(1, (m_ + p - 1) / p);
    for (std::size_t k = 0; k < p; k++) {
      tile t;
      t.rank = k;
      t.row0 = std::min(m_, k * rs);
      t.rows = std::min(m_, (k + 1) * rs) - t.row0;
      tiles_.push_back(t);
    }
  }
  void alloc(tile &t, std::size_t nnz) {
    const int rk = static_cast<int>(t.rank);
    t.nnz = nnz;
    void *p = nullptr;
    detail::check(drhip_malloc(rk, (t.rows + 1) * sizeof(I), &p), "drhip_malloc");
    t.rowptr = static_cast<I *>(p);
    detail::check(drhip_malloc(rk, std::max<std::size_t>(nnz, 1) * sizeof(I), &p), "drhip_malloc");
    t.colind = static_cast<I *>(p);
    detail::check(drhip_malloc(rk, std::max<std::size_t>(nnz, 1) * sizeof(T), &p), "drhip_malloc");
    t.values = static_cast<T *>(p);
  }

  std::size_t m_, n_;
  std::vector<tile> tiles_;
};

// gemv.hpp:13-71 (intended semantics): c += a * b.
template <typename C, typename T, typename I, typename B>
  requires lib::distributed_contiguous_range<C> && lib::distributed_contiguous_range<B>
void gemv(C &&c, const sparse_matrix<T, I> &a, B &&b) {
  const auto [m, n] = a.shape();
  if (std::ranges::size(c) != m || std::ranges::size(b) != n)
    throw std::runtime_error("shp::gemv: shape mismatch"); // gemv.hpp:18-21
  constexpr int vdt = detail::dtype_code<T>();
  constexpr int idt = detail::dtype_code<I>();
  static_assert(vdt == DRHIP_F32 || vdt == DRHIP_F64, "gemv: float or double values");
  static_assert(idt == DRHIP_I32 || idt == DRHIP_I64, "gemv: int32 or int64 indices");
  auto bsegs = lib::ranges::segments(b);
  auto csegs = lib::ranges::segments(c);
  // replicate b to every tile's device (an allgather by peer copies)
  std::vector<void *> local_b(a.tiles().size(), nullptr);
  for (std::size_t k = 0; k < a.tiles().size(); k++) {
    const auto &t = a.tile_at(k);
    if (!t.rows) continue;
    detail::check(drhip_malloc(static_cast<int>(t.rank), n * sizeof(T), &local_b[k]), "drhip_malloc");
    std::size_t off = 0;
    for (auto &s : bsegs) {
      detail::check(drhip_memcpy_d2d(static_cast<int>(t.rank), static_cast<T *>(local_b[k]) + off, s.data(),
                                     s.size() * sizeof(T)),
                    "gemv b copy");
      off += s.size();
    }
  }
  // c's segments align with the row tiles (same ceil(m/P) partition)
  std::size_t ci = 0, crow = 0;
  for (std::size_t k = 0; k < a.tiles().size(); k++) {
    const auto &t = a.tile_at(k);
    if (!t.rows) continue;
    while (crow + csegs[ci].size() <= t.row0) crow += csegs[ci++].size();
    if (crow != t.row0 || csegs[ci].size() < t.rows)
      throw std::runtime_error("shp::gemv: c is not partitioned like a's row tiles");
    detail::check(drhip_spmv_csr(static_cast<int>(t.rank), vdt, idt, t.rows, t.nnz, t.rowptr, t.colind, t.values,
                                 local_b[k], csegs[ci].data()),
                  "drhip_spmv_csr");
  }
  sync_all();
  for (std::size_t k = 0; k < local_b.size(); k++)
    if (local_b[k]) detail::check(drhip_free(static_cast<int>(a.tile_at(k).rank), local_b[k]), "drhip_free");
}

} // namespace shp
