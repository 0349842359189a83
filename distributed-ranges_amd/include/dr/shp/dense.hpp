// dr/shp/dense.hpp -- shp::dense_matrix (row-major tiles on a block-cyclic
// tile grid) and its views: dense_matrix_view, dense_matrix_row_view,
// dense_matrix_column_view, matrix_ref.
//
// Mirrors containers/dense_matrix.hpp:14-274, views/dense_matrix_view.hpp,
// views/dense_row_view.hpp, views/dense_column_view.hpp and matrix_ref in
// containers/matrix_entry.hpp:103-185:
//   * tile (i, j) is a row-major block of tile_shape() elements (leading
//     dimension tile_shape()[1], full size even for the trimmed edge tiles,
//     dense_matrix.hpp:245-263) on the device block_cyclic assigns it.  Here
//     the tiles are zero-filled at construction (the reference leaves them
//     indeterminate).
//   * operator[]({i, j}) is a device_ref to the element (dense_matrix.hpp:
//     167-189); begin()/end() walk the matrix in global row-major order and
//     yield matrix_ref {index, device_ref} (dense_matrix.hpp:16-127).
//   * tiles() are views in tile-local coordinates, segments() the same views
//     carrying their global origin (dense_matrix.hpp:198-242); both are
//     trimmed to the matrix edge.
//   * shp::for_each(policy, dense_matrix | segment, fn) runs fn(matrix_ref
//     {global index, T&}) for every element on the tile's own device (the
//     reference's generic for_each over the segment iterators,
//     for_each.hpp:49-86), so `auto &&[idx, v] = entry; v = v + 12;` works
//     as in examples/shp/matrix_example.cpp.  The element's row and column
//     come from a 32-bit multiply-high divider when the tile has fewer than
//     2^31 elements (no 64-bit division per element).
#pragma once

#include <cstdint>
#include <iterator>
#include <memory>
#include <vector>

#include "algorithms.hpp"
#include "index.hpp"
#include "sparse.hpp"

namespace shp {

// matrix_entry.hpp:103-185: an {index, reference} pair that binds as
// `auto &&[idx, v]`, with v a reference to the stored element (T& on the
// device, device_ref<T> on the host).
template <typename T, typename I = std::size_t, typename TRef = T &> class matrix_ref {
public:
  using scalar_type = T;
  using index_type = I;
  using key_type = shp::index<I>;
  using scalar_reference = TRef;
  using value_type = matrix_entry<std::remove_const_t<T>, I>;

  __host__ __device__ matrix_ref(shp::index<I> idx, TRef v) : index_(idx), value_(v) {}
  matrix_ref(const matrix_ref &) = default;

  operator value_type() const { return value_type(index_, static_cast<std::remove_const_t<T>>(value_)); }

  template <std::size_t N>
    requires(N <= 1)
  __host__ __device__ decltype(auto) get() const noexcept {
    if constexpr (N == 0) return index_;
    else return value_;
  }
  __host__ __device__ shp::index<I> index() const noexcept { return index_; }
  __host__ __device__ TRef value() const noexcept { return value_; }

private:
  shp::index<I> index_;
  TRef value_;
};

} // namespace shp

namespace std {
template <typename T, typename I, typename TRef>
struct tuple_size<shp::matrix_ref<T, I, TRef>> : integral_constant<std::size_t, 2> {};
template <typename T, typename I, typename TRef> struct tuple_element<0, shp::matrix_ref<T, I, TRef>> {
  using type = shp::index<I>;
};
template <typename T, typename I, typename TRef> struct tuple_element<1, shp::matrix_ref<T, I, TRef>> {
  using type = TRef;
};
} // namespace std

namespace shp {

namespace detail {

// n / d and n % d for a fixed d: t = umulhi(n, m); q = (t + n) >> s, exact
// for n, d < 2^31 (Granlund-Montgomery with a 33-bit magic folded into the
// add).  Larger tiles take the 64-bit division path.
struct row_divider {
  std::uint64_t d = 1;
  std::uint32_t m = 0, s = 0;
  bool small = true;
  row_divider() = default;
  row_divider(std::uint64_t divisor, std::uint64_t extent) : d(divisor ? divisor : 1) {
    small = d < (1ull << 31) && extent < (1ull << 31);
    if (small) {
      while ((1ull << s) < d) s++;
      m = static_cast<std::uint32_t>(((1ull << 32) * ((1ull << s) - d)) / d + 1);
    }
  }
  __host__ __device__ void divmod(std::uint64_t n, std::uint64_t &q, std::uint64_t &r) const {
    if (small) {
      const std::uint32_t n32 = static_cast<std::uint32_t>(n);
#if defined(__HIP_DEVICE_COMPILE__)
      const std::uint32_t t = __umulhi(n32, m);
#else
      const std::uint32_t t = static_cast<std::uint32_t>((static_cast<std::uint64_t>(n32) * m) >> 32);
#endif
      const std::uint32_t q32 = (t + n32) >> s;
      q = q32;
      r = n32 - q32 * static_cast<std::uint32_t>(d);
    } else {
      q = n / d;
      r = n - q * d;
    }
  }
};

// Device accessor of one tile: element i of the trimmed tile (row-major
// over its shape) -> matrix_ref {global index, T&}.
template <typename T> struct dense_tile_accessor {
  T *data;
  std::size_t ld;
  shp::index<> origin;
  row_divider cols;
  __device__ matrix_ref<T, std::size_t, T &> operator()(std::size_t i) const {
    std::uint64_t r, c;
    cols.divmod(i, r, c);
    return matrix_ref<T, std::size_t, T &>(shp::index<>(origin[0] + r, origin[1] + c), data[r * ld + c]);
  }
};

// Branch-free variants for for_each: Contig (shape()[1] == ld, address
// data + i, so the unrolled loads are provably distinct) x Small (32-bit
// multiply-high row division, else 64-bit).
template <typename T, bool Contig, bool Small> struct dense_fixed_accessor {
  T *data;
  std::size_t ld;
  shp::index<> origin;
  row_divider cols;
  __device__ matrix_ref<T, std::size_t, T &> operator()(std::size_t i) const {
    std::uint64_t r, c;
    if constexpr (Small) {
      const std::uint32_t n32 = static_cast<std::uint32_t>(i);
      const std::uint32_t q32 = (__umulhi(n32, cols.m) + n32) >> cols.s;
      r = q32;
      c = n32 - q32 * static_cast<std::uint32_t>(cols.d);
    } else {
      r = i / cols.d;
      c = i - r * cols.d;
    }
    T &v = Contig ? data[i] : data[r * ld + c];
    return matrix_ref<T, std::size_t, T &>(shp::index<>(origin[0] + r, origin[1] + c), v);
  }
  // staged for_each protocol (algorithms.hpp): an untrimmed tile is data + i
  static constexpr bool stageable = Contig;
  T *staged_base() const { return data; }
  __device__ matrix_ref<T, std::size_t, T &> bind(std::size_t i, T &v) const {
    std::uint64_t r, c;
    if constexpr (Small) {
      const std::uint32_t n32 = static_cast<std::uint32_t>(i);
      const std::uint32_t q32 = (__umulhi(n32, cols.m) + n32) >> cols.s;
      r = q32;
      c = n32 - q32 * static_cast<std::uint32_t>(cols.d);
    } else {
      r = i / cols.d;
      c = i - r * cols.d;
    }
    return matrix_ref<T, std::size_t, T &>(shp::index<>(origin[0] + r, origin[1] + c), v);
  }
};

} // namespace detail

// views/dense_row_view.hpp: row `i` of a tile, entries {i, j}.
template <typename T> class dense_matrix_row_view {
public:
  using size_type = std::size_t;
  using key_type = shp::index<>;
  using reference = matrix_ref<T, std::size_t, device_ref<T>>;

  dense_matrix_row_view(T *data, size_type row_idx, size_type size, size_type rank)
      : data_(data), row_idx_(row_idx), size_(size), rank_(rank) {}

  class iterator {
  public:
    using value_type = matrix_entry<std::remove_const_t<T>>;
    using difference_type = std::ptrdiff_t;
    using iterator_category = std::random_access_iterator_tag;
    iterator() = default;
    iterator(const dense_matrix_row_view *v, size_type j) : v_(v), j_(j) {}
    reference operator*() const { return reference(key_type{v_->row_idx_, j_}, (*v_)[j_]); }
    iterator &operator++() { ++j_; return *this; }
    iterator operator++(int) { auto t = *this; ++j_; return t; }
    iterator &operator+=(difference_type d) { j_ += d; return *this; }
    friend iterator operator+(iterator a, difference_type d) { return a += d; }
    friend difference_type operator-(const iterator &a, const iterator &b) {
      return static_cast<difference_type>(a.j_) - static_cast<difference_type>(b.j_);
    }
    friend bool operator==(const iterator &a, const iterator &b) { return a.j_ == b.j_; }

  private:
    const dense_matrix_row_view *v_ = nullptr;
    size_type j_ = 0;
  };

  device_ref<T> operator[](size_type j) const { return device_ref<T>(data_ + j, rank_); }
  iterator begin() const { return iterator(this, 0); }
  iterator end() const { return iterator(this, size_); }
  size_type size() const noexcept { return size_; }
  size_type rank() const noexcept { return rank_; }
  T *data() const noexcept { return data_; }

private:
  T *data_;
  size_type row_idx_, size_, rank_;
};

// views/dense_column_view.hpp: column `j` of a tile (stride ld), entries {i, j}.
template <typename T> class dense_matrix_column_view {
public:
  using size_type = std::size_t;
  using key_type = shp::index<>;
  using reference = matrix_ref<T, std::size_t, device_ref<T>>;

  dense_matrix_column_view(T *data, size_type column_idx, size_type size, size_type ld, size_type rank)
      : data_(data), column_idx_(column_idx), size_(size), ld_(ld), rank_(rank) {}

  class iterator {
  public:
    using value_type = matrix_entry<std::remove_const_t<T>>;
    using difference_type = std::ptrdiff_t;
    using iterator_category = std::random_access_iterator_tag;
    iterator() = default;
    iterator(const dense_matrix_column_view *v, size_type i) : v_(v), i_(i) {}
    reference operator*() const { return reference(key_type{i_, v_->column_idx_}, (*v_)[i_]); }
    iterator &operator++() { ++i_; return *this; }
    iterator operator++(int) { auto t = *this; ++i_; return t; }
    iterator &operator+=(difference_type d) { i_ += d; return *this; }
    friend iterator operator+(iterator a, difference_type d) { return a += d; }
    friend difference_type operator-(const iterator &a, const iterator &b) {
      return static_cast<difference_type>(a.i_) - static_cast<difference_type>(b.i_);
    }
    friend bool operator==(const iterator &a, const iterator &b) { return a.i_ == b.i_; }

  private:
    const dense_matrix_column_view *v_ = nullptr;
    size_type i_ = 0;
  };

  device_ref<T> operator[](size_type i) const { return device_ref<T>(data_ + i * ld_, rank_); }
  iterator begin() const { return iterator(this, 0); }
  iterator end() const { return iterator(this, size_); }
  size_type size() const noexcept { return size_; }
  size_type rank() const noexcept { return rank_; }

private:
  T *data_;
  size_type column_idx_, size_, ld_, rank_;
};

// views/dense_matrix_view.hpp:108-163: a shape x ld row-major block on one
// device.  Iteration is row-major over shape() and yields global indices
// (local + origin()).  It is also a segment: for_each runs on its device.
template <typename T> class dense_matrix_view {
public:
  using size_type = std::size_t;
  using key_type = shp::index<>;
  using value_type = matrix_entry<std::remove_const_t<T>>;
  using reference = matrix_ref<T, std::size_t, device_ref<T>>;
  using scalar_reference = device_ref<T>;

  dense_matrix_view(T *data, key_type shape, size_type ld, size_type rank)
      : data_(data), shape_(shape), origin_{0, 0}, ld_(ld), rank_(rank) {}
  dense_matrix_view(T *data, key_type shape, key_type origin, size_type ld, size_type rank)
      : data_(data), shape_(shape), origin_(origin), ld_(ld), rank_(rank) {}

  class iterator {
  public:
    using value_type = matrix_entry<std::remove_const_t<T>>;
    using difference_type = std::ptrdiff_t;
    using reference = dense_matrix_view::reference;
    using iterator_category = std::random_access_iterator_tag;
    iterator() = default;
    iterator(const dense_matrix_view *v, size_type k) : v_(v), k_(k) {}
    reference operator*() const { return (*this)[0]; }
    reference operator[](difference_type d) const {
      const size_type k = k_ + d, n = std::max<size_type>(v_->shape_[1], 1);
      const size_type i = k / n, j = k % n;
      return reference(key_type{i + v_->origin_[0], j + v_->origin_[1]}, (*v_)[key_type{i, j}]);
    }
    iterator &operator++() { ++k_; return *this; }
    iterator operator++(int) { auto t = *this; ++k_; return t; }
    iterator &operator--() { --k_; return *this; }
    iterator &operator+=(difference_type d) { k_ += d; return *this; }
    friend iterator operator+(iterator a, difference_type d) { return a += d; }
    friend difference_type operator-(const iterator &a, const iterator &b) {
      return static_cast<difference_type>(a.k_) - static_cast<difference_type>(b.k_);
    }
    friend bool operator==(const iterator &a, const iterator &b) { return a.k_ == b.k_; }
    friend auto operator<=>(const iterator &a, const iterator &b) { return a.k_ <=> b.k_; }

  private:
    const dense_matrix_view *v_ = nullptr;
    size_type k_ = 0;
  };

  key_type shape() const noexcept { return shape_; }
  size_type size() const noexcept { return shape_[0] * shape_[1]; }
  key_type origin() const noexcept { return origin_; }
  size_type ld() const noexcept { return ld_; }
  size_type rank() const noexcept { return rank_; }
  T *data() const noexcept { return data_; }

  // dense_matrix_view.hpp:133-135: local index
  device_ref<T> operator[](key_type idx) const { return device_ref<T>(data_ + idx[0] * ld_ + idx[1], rank_); }

  iterator begin() const { return iterator(this, 0); }
  iterator end() const { return iterator(this, size()); }

  // dense_matrix_view.hpp:145-151 (local row / column index)
  dense_matrix_row_view<T> row(size_type i) const { return {data_ + i * ld_, i, shape_[1], rank_}; }
  dense_matrix_column_view<T> column(size_type j) const { return {data_ + j, j, shape_[0], ld_, rank_}; }

  // a tile view is a distributed range of one segment: itself
  std::vector<dense_matrix_view> segments() const { return {*this}; }

  // the segment protocol of the algorithms (ranges.hpp accessor_of)
  auto accessor() const {
    return detail::dense_tile_accessor<T>{data_, ld_, origin_, detail::row_divider(shape_[1], size())};
  }
  using dispatches_accessor = void;
  template <typename F> void visit_accessor(F &&f) const {
    const detail::row_divider dv(shape_[1], size());
    const bool contig = shape_[1] == ld_;
    if (contig && dv.small) f(detail::dense_fixed_accessor<T, true, true>{data_, ld_, origin_, dv});
    else if (contig) f(detail::dense_fixed_accessor<T, true, false>{data_, ld_, origin_, dv});
    else if (dv.small) f(detail::dense_fixed_accessor<T, false, true>{data_, ld_, origin_, dv});
    else f(detail::dense_fixed_accessor<T, false, false>{data_, ld_, origin_, dv});
  }

private:
  T *data_;
  key_type shape_;
  key_type origin_;
  size_type ld_;
  size_type rank_;
};

template <typename T> class dense_matrix_iterator;

// containers/dense_matrix.hpp:133-272
template <typename T> class dense_matrix {
public:
  using size_type = std::size_t;
  using difference_type = std::ptrdiff_t;
  using value_type = matrix_entry<T>;
  using scalar_reference = device_ref<T>;
  using const_scalar_reference = device_ref<const T>;
  using reference = matrix_ref<T, std::size_t, device_ref<T>>;
  using key_type = shp::index<>;
  using segment_type = dense_matrix_view<T>;
  using iterator = dense_matrix_iterator<T>;

  explicit dense_matrix(key_type shape) : dense_matrix(shape, block_cyclic()) {}
  dense_matrix(key_type shape, const matrix_partition &partition) : shape_(shape), partition_(partition.clone()) {
    if (nprocs() == 0) throw std::runtime_error("shp::dense_matrix: shp::init not called");
    grid_shape_ = partition_->grid_shape(shape_);
    tile_shape_ = partition_->tile_shape(shape_);
    const std::size_t tsize = tile_shape_[0] * tile_shape_[1];
    const T zero{};
    tiles_.reserve(grid_shape_[0] * grid_shape_[1]);
    for (std::size_t i = 0; i < grid_shape_[0]; i++)
      for (std::size_t j = 0; j < grid_shape_[1]; j++) {
        const std::size_t rank = partition_->tile_rank(shape_, {i, j});
        auto &t = tiles_.emplace_back(tsize, device_allocator<T>(rank), rank);
        if (tsize) detail::check(drhip_fill(static_cast<int>(rank), t.data(), tsize, &zero, sizeof(T)), "fill");
      }
    sync_all();
  }
  dense_matrix(const dense_matrix &) = delete;
  dense_matrix &operator=(const dense_matrix &) = delete;
  dense_matrix(dense_matrix &&) = default;
  dense_matrix &operator=(dense_matrix &&) = default;

  size_type size() const noexcept { return shape_[0] * shape_[1]; }
  key_type shape() const noexcept { return shape_; }
  key_type tile_shape() const noexcept { return tile_shape_; }
  key_type grid_shape() const noexcept { return grid_shape_; }
  const matrix_partition &partition() const { return *partition_; }

  // dense_matrix.hpp:167-189
  scalar_reference operator[](key_type idx) const {
    const auto &t = tiles_[(idx[0] / tile_shape_[0]) * grid_shape_[1] + idx[1] / tile_shape_[1]];
    return scalar_reference(t.data() + (idx[0] % tile_shape_[0]) * tile_shape_[1] + idx[1] % tile_shape_[1],
                            t.rank());
  }

  iterator begin() const { return iterator(this, 0); }
  iterator end() const { return iterator(this, size()); }

  segment_type tile(key_type tile_index) const { return view(tile_index[0], tile_index[1], false); }
  std::vector<segment_type> tiles() const { return views(false); }
  std::vector<segment_type> segments() const { return views(true); }

private:
  segment_type view(std::size_t i, std::size_t j, bool global) const {
    const auto &t = tiles_.at(i * grid_shape_[1] + j);
    const key_type org{std::min(shape_[0], i * tile_shape_[0]), std::min(shape_[1], j * tile_shape_[1])};
    const key_type shp{std::min(tile_shape_[0], shape_[0] - org[0]), std::min(tile_shape_[1], shape_[1] - org[1])};
    return global ? segment_type(t.data(), shp, org, tile_shape_[1], t.rank())
                  : segment_type(t.data(), shp, tile_shape_[1], t.rank());
  }
  std::vector<segment_type> views(bool global) const {
    std::vector<segment_type> v;
    v.reserve(tiles_.size());
    for (std::size_t i = 0; i < grid_shape_[0]; i++)
      for (std::size_t j = 0; j < grid_shape_[1]; j++) v.push_back(view(i, j, global));
    return v;
  }

  key_type shape_{0, 0}, grid_shape_{0, 0}, tile_shape_{0, 0};
  std::unique_ptr<matrix_partition> partition_;
  std::vector<device_vector<T>> tiles_;
};

// dense_matrix.hpp:16-131: global row-major order, entry {index, device_ref}.
template <typename T> class dense_matrix_iterator {
public:
  using value_type = matrix_entry<T>;
  using difference_type = std::ptrdiff_t;
  using reference = matrix_ref<T, std::size_t, device_ref<T>>;
  using iterator_category = std::random_access_iterator_tag;

  dense_matrix_iterator() = default;
  dense_matrix_iterator(const dense_matrix<T> *m, std::size_t g) : m_(m), g_(g) {}

  reference operator*() const { return (*this)[0]; }
  reference operator[](difference_type d) const {
    const std::size_t g = g_ + d, n = std::max<std::size_t>(m_->shape()[1], 1);
    const shp::index<> idx{g / n, g % n};
    return reference(idx, (*m_)[idx]);
  }
  dense_matrix_iterator &operator++() { ++g_; return *this; }
  dense_matrix_iterator operator++(int) { auto t = *this; ++g_; return t; }
  dense_matrix_iterator &operator--() { --g_; return *this; }
  dense_matrix_iterator operator--(int) { auto t = *this; --g_; return t; }
  dense_matrix_iterator &operator+=(difference_type d) { g_ += d; return *this; }
  dense_matrix_iterator &operator-=(difference_type d) { g_ -= d; return *this; }
  friend dense_matrix_iterator operator+(dense_matrix_iterator a, difference_type d) { return a += d; }
  friend dense_matrix_iterator operator+(difference_type d, dense_matrix_iterator a) { return a += d; }
  friend dense_matrix_iterator operator-(dense_matrix_iterator a, difference_type d) { return a -= d; }
  friend difference_type operator-(const dense_matrix_iterator &a, const dense_matrix_iterator &b) {
    return static_cast<difference_type>(a.g_) - static_cast<difference_type>(b.g_);
  }
  friend bool operator==(const dense_matrix_iterator &a, const dense_matrix_iterator &b) { return a.g_ == b.g_; }
  friend auto operator<=>(const dense_matrix_iterator &a, const dense_matrix_iterator &b) { return a.g_ <=> b.g_; }

private:
  const dense_matrix<T> *m_ = nullptr;
  std::size_t g_ = 0;
};

} // namespace shp
