// dr/shp/ranges.hpp -- lib::ranges customization points, the distributed
// concepts, distributed_vector and the distributed views (take / drop /
// subrange / slice, zip, enumerate, transform) of the shp drop-in layer.
//
// Mirrors details/ranges.hpp:38-165 (segments / rank / local CPOs),
// concepts/concepts.hpp:11-52, shp/distributed_vector.hpp:18-207
// (block distribution: segment i = [i*s, min((i+1)*s, n)), s = ceil(n/P)),
// details/segments_tools.hpp:37-94 (take/drop of segments),
// shp/zip_view.hpp:89-337 (zipped_segments intersect segment boundaries),
// views/transform.hpp:9-77 and shp/range_adaptors.hpp:12-15 (enumerate; the
// index is 64-bit here, SURVEY.md 5: uint32 overflows at 2^32 cells).
//
// Every segment type also exposes `accessor()`: a small trivially-copyable
// object with `__device__ reference operator()(size_t i)` that the HIP
// template kernels (algorithms.hpp) use to read/write element i of the
// segment on the device.
#pragma once

#include <algorithm>
#include <functional>
#include <iterator>
#include <numeric>
#include <ranges>
#include <tuple>
#include <utility>
#include <vector>

#include "memory.hpp"

namespace shp {

// ------------------------------------------------------------ accessors

template <typename T> struct span_accessor {
  T *p;
  __host__ __device__ T &operator()(std::size_t i) const { return p[i]; }
  // staged for_each protocol (algorithms.hpp): element i lives at p + i and
  // fn may run on a register copy of it
  static constexpr bool stageable = true;
  T *staged_base() const { return p; }
  __host__ __device__ T &bind(std::size_t, T &r) const { return r; }
};

template <typename I> struct iota_accessor {
  I start;
  __host__ __device__ I operator()(std::size_t i) const { return static_cast<I>(start + static_cast<I>(i)); }
};

template <typename... A> struct zip_accessor {
  std::tuple<A...> a;
  __host__ __device__ auto operator()(std::size_t i) const {
    return std::apply([i](const auto &...x) { return std::tuple<decltype(x(i))...>(x(i)...); }, a);
  }
};

template <typename A, typename F> struct transform_accessor {
  A a;
  F f;
  __host__ __device__ auto operator()(std::size_t i) const { return f(a(i)); }
};

// A device_span as a segment with an accessor.
template <typename T> span_accessor<T> make_accessor(const device_span<T> &s) { return {s.data()}; }

// Segment of a std::views::iota zipped with distributed ranges: adopts the
// boundaries of its zip partners.
template <typename I> struct iota_segment {
  I start;
  std::size_t n;
  std::size_t rank_ = 0;
  std::size_t size() const { return n; }
  std::size_t rank() const { return rank_; }
  iota_accessor<I> accessor() const { return {start}; }
  iota_segment subspan(std::size_t off, std::size_t cnt) const {
    return {static_cast<I>(start + static_cast<I>(off)), cnt, rank_};
  }
};

} // namespace shp

// ----------------------------------------------------------- lib CPOs
namespace lib {
namespace ranges {

namespace detail {
template <typename R>
concept has_segments_member = requires(R &r) { r.segments(); };
template <typename S>
concept has_rank_member = requires(S &s) { s.rank(); };
template <typename I>
concept has_distributed_iter = requires(I i) { i.segments_to(i); };
} // namespace detail

// details/ranges.hpp:94-116
struct segments_fn {
  template <typename R> auto operator()(R &&r) const {
    if constexpr (detail::has_segments_member<R>) {
      return r.segments();
    } else if constexpr (std::ranges::range<R> && detail::has_distributed_iter<std::ranges::iterator_t<R>>) {
      // subrange / take / drop / views::all of a distributed range
      auto first = std::ranges::begin(r);
      return first.segments_to(first + std::ranges::distance(r));
    } else {
      static_assert(sizeof(R) == 0, "lib::ranges::segments: not a distributed range");
    }
  }
};
inline constexpr segments_fn segments{};

// details/ranges.hpp:38-70
struct rank_fn {
  template <typename S>
    requires detail::has_rank_member<S>
  std::size_t operator()(S &&s) const {
    return s.rank();
  }
};
inline constexpr rank_fn rank{};

// details/ranges.hpp:133-163: the raw local pointer of a device iterator /
// the raw pointer range of a device span.
struct local_fn {
  template <typename T> T *operator()(shp::device_ptr<T> p) const { return p.local(); }
  template <typename T> std::span<T> operator()(const shp::device_span<T> &s) const {
    return std::span<T>(s.data(), s.size());
  }
};
inline constexpr local_fn local{};

} // namespace ranges

// concepts/concepts.hpp:11-52 (reduced to what the algorithms require)
template <typename R>
concept distributed_range = std::ranges::sized_range<R> && requires(R &r) { lib::ranges::segments(r); };

template <typename I>
concept distributed_iterator = requires(I i) { i.segments_to(i); };

template <typename R>
concept distributed_contiguous_range =
    distributed_range<R> && requires(R &r) { lib::ranges::segments(r)[0].data(); };

} // namespace lib

namespace shp {

template <typename T> class distributed_vector_iterator;

// ----------------------------------------------------- distributed_vector
// distributed_vector.hpp:115-205.  Allocator defaults to shared_allocator
// like the reference (device memory here, memory.hpp).
template <typename T, typename Allocator = shared_allocator<T>> class distributed_vector {
public:
  using value_type = T;
  using size_type = std::size_t;
  using difference_type = std::ptrdiff_t;
  using segment_type = device_span<T>;
  using iterator = distributed_vector_iterator<T>;
  using const_iterator = distributed_vector_iterator<const T>;
  using reference = device_ref<T>;

  distributed_vector() = default;

  explicit distributed_vector(std::size_t count) {
    const std::size_t p = nprocs();
    if (p == 0) throw std::runtime_error("shp::distributed_vector: shp::init not called");
    size_ = count;
    segment_size_ = std::max<std::size_t>(1, (count + p - 1) / p); // :142
    for (std::size_t r = 0; r < p; r++) {
      auto &v = storage_.emplace_back(segment_size_, rebind_alloc(r), r);
      spans_.emplace_back(v.data(), v.size(), r);
    }
    // :153 -- the zero fill that defines the contents, one per segment
    const T zero{};
    for (std::size_t r = 0; r < p; r++)
      detail::fill_segment_async(r, spans_[r].data(), segment_size_, zero);
    sync_all();
  }

  distributed_vector(std::size_t count, const T &value) : distributed_vector(count) {
    for (auto &s : segments())
      detail::fill_segment_async(s.rank(), s.data(), s.size(), value);
    sync_all();
  }

  distributed_vector(const distributed_vector &) = delete;
  distributed_vector &operator=(const distributed_vector &) = delete;
  distributed_vector(distributed_vector &&) = default;
  distributed_vector &operator=(distributed_vector &&) = default;

  reference operator[](size_type pos) const {
    return spans_[pos / segment_size_][pos % segment_size_]; // :164-174
  }
  size_type size() const noexcept { return size_; }
  bool empty() const noexcept { return size_ == 0; }

  // segments() trimmed to size() (:178-182 -> take_segments)
  std::vector<segment_type> segments() const { return begin().segments_to(end()); }

  iterator begin() const { return iterator(&spans_, 0, segment_size_); }
  iterator end() const { return iterator(&spans_, size_, segment_size_); }
  std::size_t segment_size() const { return segment_size_; }

private:
  template <typename A> static constexpr bool is_device_alloc = std::is_same_v<A, device_allocator<T>>;
  static Allocator rebind_alloc(std::size_t r) { return Allocator(r); }

  std::vector<device_vector<T, Allocator>> storage_;
  std::vector<device_span<T>> spans_;
  std::size_t size_ = 0;
  std::size_t segment_size_ = 0;
};

// Random-access iterator over the whole distributed range
// (distributed_vector.hpp:18-111 accessor + iterator_adaptor).
template <typename T> class distributed_vector_iterator {
public:
  using value_type = std::remove_const_t<T>;
  using difference_type = std::ptrdiff_t;
  using reference = device_ref<T>;
  using iterator_category = std::random_access_iterator_tag;
  using iterator_concept = std::random_access_iterator_tag;

  distributed_vector_iterator() = default;
  distributed_vector_iterator(const std::vector<device_span<std::remove_const_t<T>>> *segs, std::size_t g,
                              std::size_t ss)
      : segs_(segs), g_(g), ss_(ss) {}

  reference operator*() const { return (*this)[0]; }
  reference operator[](difference_type d) const {
    const std::size_t g = g_ + d;
    const auto &s = (*segs_)[g / ss_];
    return reference(s.data() + g % ss_, s.rank());
  }
  distributed_vector_iterator &operator++() { ++g_; return *this; }
  distributed_vector_iterator operator++(int) { auto t = *this; ++g_; return t; }
  distributed_vector_iterator &operator--() { --g_; return *this; }
  distributed_vector_iterator operator--(int) { auto t = *this; --g_; return t; }
  distributed_vector_iterator &operator+=(difference_type d) { g_ += d; return *this; }
  distributed_vector_iterator &operator-=(difference_type d) { g_ -= d; return *this; }
  friend distributed_vector_iterator operator+(distributed_vector_iterator a, difference_type d) { return a += d; }
  friend distributed_vector_iterator operator+(difference_type d, distributed_vector_iterator a) { return a += d; }
  friend distributed_vector_iterator operator-(distributed_vector_iterator a, difference_type d) { return a -= d; }
  friend difference_type operator-(const distributed_vector_iterator &a, const distributed_vector_iterator &b) {
    return static_cast<difference_type>(a.g_) - static_cast<difference_type>(b.g_);
  }
  friend bool operator==(const distributed_vector_iterator &a, const distributed_vector_iterator &b) {
    return a.g_ == b.g_;
  }
  friend auto operator<=>(const distributed_vector_iterator &a, const distributed_vector_iterator &b) {
    return a.g_ <=> b.g_;
  }

  // Segments of [*this, last): one device_span per touched segment, in rank
  // order (segments_tools.hpp:37-94 take/drop semantics).
  std::vector<device_span<T>> segments_to(const distributed_vector_iterator &last) const {
    std::vector<device_span<T>> out;
    std::size_t g = g_;
    while (g < last.g_) {
      const std::size_t si = g / ss_, off = g % ss_;
      const std::size_t cnt = std::min(ss_ - off, last.g_ - g);
      const auto &s = (*segs_)[si];
      out.emplace_back(const_cast<T *>(s.data()) + off, cnt, s.rank());
      g += cnt;
    }
    return out;
  }
  // lib::ranges::segments(iterator): the segments from here to the end of
  // the container (test/gtest/shp/containers.cpp:34-41).
  std::vector<device_span<T>> segments() const {
    std::size_t total = 0;
    for (auto &s : *segs_) total += s.size();
    return segments_to(distributed_vector_iterator(segs_, total, ss_));
  }
  std::size_t global_index() const { return g_; }

private:
  const std::vector<device_span<std::remove_const_t<T>>> *segs_ = nullptr;
  std::size_t g_ = 0;
  std::size_t ss_ = 1;
};

// --------------------------------------------------------------- views

namespace detail {

// Segments of any accepted range as a vector of segment objects.
template <typename R> auto segments_of(R &&r) { return lib::ranges::segments(r); }

template <typename S> auto accessor_of(const S &s) {
  if constexpr (requires { s.accessor(); }) return s.accessor();
  else return make_accessor(s);
}

} // namespace detail

// Piece of a zip: one sub-segment per zipped range, same length, same rank
// (zip_view.hpp:172-206).
template <typename... S> struct zip_segment {
  std::tuple<S...> parts;
  std::size_t size() const { return std::get<0>(parts).size(); }
  std::size_t rank() const { return std::get<0>(parts).rank(); }
  auto accessor() const {
    return std::apply([](const auto &...p) { return zip_accessor<decltype(detail::accessor_of(p))...>{
                                                  std::tuple(detail::accessor_of(p)...)}; },
                      parts);
  }
  zip_segment subspan(std::size_t off, std::size_t cnt) const {
    return std::apply([&](const auto &...p) { return zip_segment{std::tuple(p.subspan(off, cnt)...)}; }, parts);
  }
};

namespace detail {

template <typename R>
concept iota_like = requires { typename std::remove_cvref_t<R>; } &&
                    std::same_as<std::remove_cvref_t<R>,
                                 std::ranges::iota_view<std::ranges::range_value_t<R>,
                                                        std::ranges::range_value_t<R>>>;

// Boundaries of the segments of a distributed range (prefix of sizes).
template <typename Segs> std::vector<std::size_t> boundaries(const Segs &segs) {
  std::vector<std::size_t> b{0};
  for (auto &s : segs) b.push_back(b.back() + s.size());
  return b;
}

// Cut a segment list at the given global boundaries.
template <typename Segs> auto cut(const Segs &segs, const std::vector<std::size_t> &bounds) {
  using S = std::remove_cvref_t<decltype(segs[0])>;
  std::vector<S> out;
  std::size_t si = 0, pos = 0; // pos = global start of segs[si]
  for (std::size_t k = 0; k + 1 < bounds.size(); k++) {
    const std::size_t lo = bounds[k], hi = bounds[k + 1];
    while (pos + segs[si].size() <= lo) pos += segs[si++].size();
    out.push_back(segs[si].subspan(lo - pos, hi - lo));
  }
  return out;
}

} // namespace detail

// shp::views::zip over distributed ranges (and at most iota views, which
// adopt the partners' boundaries): zip_view.hpp:89-337.
template <typename... R> class zip_view : public std::ranges::view_interface<zip_view<R...>> {
public:
  explicit zip_view(R &&...r) : ranges_(std::forward<R>(r)...) {}

  std::size_t size() const {
    return std::apply([](const auto &...r) { return std::min({std::size_t(std::ranges::size(r))...}); }, ranges_);
  }

  // zip_view.hpp:172-206: the union of all segment boundaries, each piece
  // on the rank of the FIRST distributed range (:53).
  auto zipped_segments() const {
    const std::size_t n = size();
    std::vector<std::size_t> bounds{0, n};
    std::size_t rank_src = 0;
    std::vector<std::size_t> first_bounds;
    std::apply(
        [&](const auto &...r) {
          (
              [&](const auto &x) {
                if constexpr (!detail::iota_like<decltype(x)>) {
                  auto b = detail::boundaries(lib::ranges::segments(x));
                  if (first_bounds.empty()) first_bounds = b;
                  for (auto v : b)
                    if (v < n) bounds.push_back(v);
                }
              }(r),
              ...);
        },
        ranges_);
    (void)rank_src;
    std::sort(bounds.begin(), bounds.end());
    bounds.erase(std::unique(bounds.begin(), bounds.end()), bounds.end());
    auto parts = std::apply([&](const auto &...r) { return std::tuple(pieces_of(r, bounds)...); }, ranges_);
    using Z = decltype(make_piece(parts, 0));
    std::vector<Z> out;
    for (std::size_t k = 0; k + 1 < bounds.size(); k++) out.push_back(make_piece(parts, k));
    return out;
  }
  auto segments() const { return zipped_segments(); }

  // host iteration: tuples of element values (for equality checks)
  struct iterator {
    const zip_view *z;
    std::size_t i;
    using value_type = std::tuple<std::ranges::range_value_t<R>...>;
    using difference_type = std::ptrdiff_t;
    value_type operator*() const {
      return std::apply([&](const auto &...r) { return value_type(value_at(r, i)...); }, z->ranges_);
    }
    iterator &operator++() { ++i; return *this; }
    iterator operator++(int) { auto t = *this; ++i; return t; }
    bool operator==(const iterator &o) const { return i == o.i; }
  };
  iterator begin() const { return {this, 0}; }
  iterator end() const { return {this, size()}; }

private:
  template <typename X> static auto value_at(const X &r, std::size_t i) {
    return static_cast<std::ranges::range_value_t<X>>(std::ranges::begin(r)[i]);
  }
  template <typename X> auto pieces_of(const X &r, const std::vector<std::size_t> &bounds) const {
    if constexpr (detail::iota_like<X>) {
      using I = std::ranges::range_value_t<X>;
      std::vector<iota_segment<I>> out;
      const I s0 = *std::ranges::begin(r);
      for (std::size_t k = 0; k + 1 < bounds.size(); k++)
        out.push_back({static_cast<I>(s0 + static_cast<I>(bounds[k])), bounds[k + 1] - bounds[k], 0});
      return out;
    } else {
      return detail::cut(lib::ranges::segments(r), bounds);
    }
  }
  template <typename Parts> static auto make_piece(const Parts &parts, std::size_t k) {
    auto z = std::apply([k](const auto &...p) { return zip_segment<std::remove_cvref_t<decltype(p[k])>...>{
                                                    std::tuple(p[k]...)}; },
                        parts);
    // iota pieces take the rank of the first distributed piece
    std::size_t rk = 0;
    bool found = false;
    std::apply(
        [&](const auto &...p) {
          (
              [&](const auto &x) {
                if constexpr (requires { x.data(); })
                  if (!found) {
                    rk = x.rank();
                    found = true;
                  }
              }(p),
              ...);
        },
        z.parts);
    std::apply(
        [&](auto &...p) {
          (
              [&](auto &x) {
                if constexpr (requires { x.rank_; }) x.rank_ = rk;
              }(p),
              ...);
        },
        z.parts);
    return z;
  }

  std::tuple<R...> ranges_;
};

template <typename... R> zip_view(R &&...) -> zip_view<R...>;

// Segment of a transform view: a segment plus the function.
template <typename S, typename F> struct transform_segment {
  S base;
  F f;
  std::size_t size() const { return base.size(); }
  std::size_t rank() const { return base.rank(); }
  auto accessor() const { return transform_accessor<decltype(detail::accessor_of(base)), F>{detail::accessor_of(base), f}; }
  transform_segment subspan(std::size_t off, std::size_t cnt) const { return {base.subspan(off, cnt), f}; }
};

// lib::views::transform (views/transform.hpp:9-77): segments are the base
// segments with the function attached; F must be device-callable (a lambda,
// or a functor whose operator() is __host__ __device__ / constexpr).
template <typename R, typename F> class transform_view : public std::ranges::view_interface<transform_view<R, F>> {
public:
  transform_view(R &&r, F f) : r_(std::forward<R>(r)), f_(f) {}
  std::size_t size() const { return std::ranges::size(r_); }
  auto segments() const {
    auto segs = lib::ranges::segments(r_);
    using S = std::remove_cvref_t<decltype(segs[0])>;
    std::vector<transform_segment<S, F>> out;
    for (auto &s : segs) out.push_back({s, f_});
    return out;
  }
  struct iterator {
    const transform_view *t;
    std::size_t i;
    using value_type = std::remove_cvref_t<decltype(std::declval<F>()(
        std::declval<std::ranges::range_value_t<std::remove_cvref_t<R>>>()))>;
    using difference_type = std::ptrdiff_t;
    value_type operator*() const {
      return t->f_(static_cast<std::ranges::range_value_t<std::remove_cvref_t<R>>>(std::ranges::begin(t->r_)[i]));
    }
    iterator &operator++() { ++i; return *this; }
    iterator operator++(int) { auto x = *this; ++i; return x; }
    bool operator==(const iterator &o) const { return i == o.i; }
  };
  iterator begin() const { return {this, 0}; }
  iterator end() const { return {this, size()}; }

private:
  R r_;
  F f_;
};

namespace views {

template <typename... R> auto zip(R &&...r) { return zip_view<R...>(std::forward<R>(r)...); }

// shp::views::slice (views/standard_views.hpp:15-42)
struct slice_adaptor {
  std::size_t lo, hi;
};
inline slice_adaptor slice(std::pair<std::size_t, std::size_t> r) { return {r.first, r.second}; }
template <typename R> auto operator|(R &&r, slice_adaptor s) {
  auto b = std::ranges::begin(r);
  return std::ranges::subrange(b + s.lo, b + s.hi);
}

// shp::views::enumerate (range_adaptors.hpp:12-15) with a 64-bit index.
template <typename R> auto enumerate(R &&r) {
  const std::int64_t n = static_cast<std::int64_t>(std::ranges::size(r));
  return zip(std::views::iota(std::int64_t(0), n), std::forward<R>(r));
}

} // namespace views

template <typename R> auto enumerate(R &&r) { return views::enumerate(std::forward<R>(r)); }

} // namespace shp

namespace lib::views {

template <typename R, typename F> auto transform(R &&r, F f) { return shp::transform_view<R, F>(std::forward<R>(r), f); }

template <typename F> struct transform_adaptor {
  F f;
};
template <typename F> transform_adaptor<F> transform(F f) { return {f}; }
template <typename R, typename F>
  requires lib::distributed_range<R>
auto operator|(R &&r, transform_adaptor<F> a) {
  return shp::transform_view<R, F>(std::forward<R>(r), a.f);
}

} // namespace lib::views

