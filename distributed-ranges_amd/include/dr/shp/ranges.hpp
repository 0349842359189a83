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
#include <memory>
#include <numeric>
#include <ranges>
#include <span>
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
template <typename T, typename L> span_accessor<T> make_accessor(const device_span<T, L> &s) { return {s.data()}; }

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

// details/ranges.hpp:15: types opt out of rank() detection
template <typename> inline constexpr bool disable_rank = false;

namespace detail {
template <typename T>
concept has_rank_method = requires(T t) {
  { t.rank() } -> std::weakly_incrementable;
};
template <typename R>
concept has_rank_adl = requires(R &r) {
  { rank_(r) } -> std::weakly_incrementable;
};
// an iterator into one segment (device_ptr): forward iterator with rank()
template <typename I>
concept remote_iterator_ =
    std::forward_iterator<I> && has_rank_method<I> && !disable_rank<std::remove_cv_t<I>>;
template <typename R>
concept has_segments_member = requires(R &r) { r.segments(); };
template <typename R>
concept has_segments_adl = requires(R &r) { segments_(r); };
template <typename I>
concept has_distributed_iter = requires(I i) { i.segments_to(i); };
template <typename I>
concept has_local_method = requires(I i) { i.local(); };
template <typename I>
concept has_local_adl = requires(I &i) { local_(i); };
} // namespace detail

// details/ranges.hpp:38-72: rank of a remote range -- r.rank(), else the rank
// of its first iterator (a remote iterator), else ADL rank_(r); rank of a
// remote iterator -- it.rank().
struct rank_fn {
  template <typename R>
    requires((detail::has_rank_method<R &> && !disable_rank<std::remove_cvref_t<R>>) ||
             (std::ranges::forward_range<R> && detail::remote_iterator_<std::ranges::iterator_t<R>>) ||
             (detail::has_rank_adl<R> && !disable_rank<std::remove_cvref_t<R>>))
  std::size_t operator()(R &&r) const {
    // (a remote iterator such as device_ptr takes the first branch too:
    //  details/ranges.hpp:60-67 rank(iter) = iter.rank())
    if constexpr (detail::has_rank_method<R &> && !disable_rank<std::remove_cvref_t<R>>) {
      return static_cast<std::size_t>(r.rank());
    } else if constexpr (std::ranges::forward_range<R> && detail::remote_iterator_<std::ranges::iterator_t<R>>) {
      return static_cast<std::size_t>(std::ranges::begin(r).rank());
    } else {
      return static_cast<std::size_t>(rank_(r));
    }
  }
};
inline constexpr rank_fn rank{};

// details/ranges.hpp:94-116: segments of a distributed range -- r.segments(),
// else ADL segments_(r), else (subrange / take / drop / views::all of a
// distributed range) the segments between its distributed iterators; of a
// distributed iterator -- it.segments() or ADL segments_(it).
struct segments_fn {
  template <typename R>
    requires(detail::has_segments_member<R> || detail::has_segments_adl<R> ||
             (std::ranges::range<R> && detail::has_distributed_iter<std::ranges::iterator_t<R>>))
  auto operator()(R &&r) const {
    if constexpr (detail::has_segments_member<R>) {
      return r.segments();
    } else if constexpr (detail::has_segments_adl<R>) {
      return segments_(r);
    } else {
      auto first = std::ranges::begin(r);
      return first.segments_to(first + std::ranges::distance(r));
    }
  }
};
inline constexpr segments_fn segments{};

// details/ranges.hpp:120-163: the local (device) form of a remote iterator
// or range -- it.local(), ADL local_(it), or the iterator itself when it is
// already contiguous; for ranges a std::span over the local pointer.
struct local_fn {
  template <typename I>
    requires(std::input_or_output_iterator<I> &&
             (detail::has_local_method<I> || detail::has_local_adl<I> || std::contiguous_iterator<I>))
  auto operator()(I it) const {
    if constexpr (detail::has_local_method<I>) return it.local();
    else if constexpr (detail::has_local_adl<I>) return local_(it);
    else return it;
  }
  template <typename R>
    requires(std::ranges::forward_range<R> && !std::input_or_output_iterator<std::remove_cvref_t<R>>)
  auto operator()(R &&r) const {
    using I = std::ranges::iterator_t<R>;
    if constexpr (detail::has_local_method<I>) {
      return std::span(std::ranges::begin(r).local(), std::ranges::size(r));
    } else if constexpr (detail::has_local_adl<R>) {
      return local_(r);
    } else {
      static_assert(std::ranges::contiguous_range<R>, "lib::ranges::local: no local form");
      return std::span(std::ranges::data(r), std::ranges::size(r));
    }
  }
};
inline constexpr local_fn local{};

} // namespace ranges

// concepts/concepts.hpp:11-52
template <typename R>
concept remote_range = std::ranges::forward_range<R> && requires(R &r) { lib::ranges::rank(r); };

template <typename R>
concept distributed_range = std::ranges::sized_range<R> && requires(R &r) { lib::ranges::segments(r); };

template <typename I>
concept remote_iterator = std::forward_iterator<I> && requires(I i) { lib::ranges::rank(i); };

template <typename I>
concept distributed_iterator = requires(I i) { i.segments_to(i); };

template <typename R>
concept remote_contiguous_range = remote_range<R> && std::ranges::random_access_range<R> &&
                                  requires(R &r) { lib::ranges::local(std::ranges::begin(r)); };

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

// ------------------------------------------------------ distributed_span
// distributed_span.hpp:124-242: a non-owning view over an ordered list of
// device segments of any sizes (a distributed_vector's segments, spans the
// user allocated per device, a sub-span of either).  The segment list is
// shared by the span's copies and iterators, so sub-spans and iterators stay
// valid after the span object that made them is gone.
template <typename T> struct dspan_data {
  std::vector<device_span<T>> segs;
  std::vector<std::size_t> pre{0}; // pre[k] = elements before segment k
};

template <typename T> class distributed_span_iterator {
public:
  using value_type = std::remove_const_t<T>;
  using difference_type = std::ptrdiff_t;
  using reference = device_ref<T>;
  using iterator_category = std::random_access_iterator_tag;
  using iterator_concept = std::random_access_iterator_tag;

  distributed_span_iterator() = default;
  distributed_span_iterator(std::shared_ptr<const dspan_data<T>> d, std::size_t g) : d_(std::move(d)), g_(g) {}

  reference operator*() const { return (*this)[0]; }
  reference operator[](difference_type off) const {
    const std::size_t g = g_ + off;
    const std::size_t k = segment_of(g);
    const auto &s = d_->segs[k];
    return reference(s.data() + (g - d_->pre[k]), s.rank());
  }
  distributed_span_iterator &operator++() { ++g_; return *this; }
  distributed_span_iterator operator++(int) { auto t = *this; ++g_; return t; }
  distributed_span_iterator &operator--() { --g_; return *this; }
  distributed_span_iterator operator--(int) { auto t = *this; --g_; return t; }
  distributed_span_iterator &operator+=(difference_type n) { g_ += n; return *this; }
  distributed_span_iterator &operator-=(difference_type n) { g_ -= n; return *this; }
  friend distributed_span_iterator operator+(distributed_span_iterator a, difference_type n) { return a += n; }
  friend distributed_span_iterator operator+(difference_type n, distributed_span_iterator a) { return a += n; }
  friend distributed_span_iterator operator-(distributed_span_iterator a, difference_type n) { return a -= n; }
  friend difference_type operator-(const distributed_span_iterator &a, const distributed_span_iterator &b) {
    return static_cast<difference_type>(a.g_) - static_cast<difference_type>(b.g_);
  }
  friend bool operator==(const distributed_span_iterator &a, const distributed_span_iterator &b) { return a.g_ == b.g_; }
  friend auto operator<=>(const distributed_span_iterator &a, const distributed_span_iterator &b) { return a.g_ <=> b.g_; }

  // segments of [*this, last) (distributed_span.hpp:102-104: drop_segments)
  std::vector<device_span<T>> segments_to(const distributed_span_iterator &last) const {
    std::vector<device_span<T>> out;
    std::size_t g = g_;
    while (g < last.g_) {
      const std::size_t k = segment_of(g), off = g - d_->pre[k];
      const std::size_t cnt = std::min(d_->segs[k].size() - off, last.g_ - g);
      out.push_back(d_->segs[k].subspan(off, cnt));
      g += cnt;
    }
    return out;
  }
  std::vector<device_span<T>> segments() const {
    return segments_to(distributed_span_iterator(d_, d_ ? d_->pre.back() : 0));
  }

private:
  std::size_t segment_of(std::size_t g) const {
    // last segment k with pre[k] <= g that is not empty
    auto it = std::upper_bound(d_->pre.begin(), d_->pre.end() - 1, g);
    std::size_t k = static_cast<std::size_t>(it - d_->pre.begin()) - 1;
    while (k + 1 < d_->segs.size() && d_->segs[k].size() == 0) k++;
    return k;
  }
  std::shared_ptr<const dspan_data<T>> d_;
  std::size_t g_ = 0;
};

template <typename T, typename L = T *>
class distributed_span : public std::ranges::view_interface<distributed_span<T, L>> {
public:
  using element_type = T;
  using value_type = std::remove_cv_t<T>;
  using segment_type = device_span<T>;
  using size_type = std::size_t;
  using difference_type = std::ptrdiff_t;
  using reference = device_ref<T>;
  using iterator = distributed_span_iterator<T>;

  distributed_span() : d_(std::make_shared<dspan_data<T>>()) {}

  // from a list of remote segments (distributed_span.hpp:154-163): each
  // segment's local pointer, size and rank
  template <std::ranges::input_range R>
    requires(lib::remote_range<std::ranges::range_reference_t<R>> && !lib::distributed_range<R>)
  distributed_span(R &&segments) : distributed_span() {
    auto d = std::make_shared<dspan_data<T>>();
    for (auto &&seg : segments) push(*d, seg);
    d_ = std::move(d);
  }
  // from a distributed range (:165-172)
  template <lib::distributed_range R>
    requires(!std::is_same_v<std::remove_cvref_t<R>, distributed_span>)
  distributed_span(R &&r) : distributed_span() {
    auto d = std::make_shared<dspan_data<T>>();
    for (auto &&seg : lib::ranges::segments(r)) push(*d, seg);
    d_ = std::move(d);
  }

  size_type size() const noexcept { return d_->pre.back(); }
  size_type size_bytes() const noexcept { return size() * sizeof(element_type); }
  [[nodiscard]] bool empty() const noexcept { return size() == 0; }
  reference operator[](size_type idx) const { return begin()[static_cast<difference_type>(idx)]; }

  // :191-217
  distributed_span subspan(size_type offset, size_type count = std::dynamic_extent) const {
    count = std::min(count, size() - offset);
    distributed_span out;
    auto d = std::make_shared<dspan_data<T>>();
    for (auto &s : (begin() + offset).segments_to(begin() + offset + count)) {
      d->segs.push_back(s);
      d->pre.push_back(d->pre.back() + s.size());
    }
    out.d_ = std::move(d);
    return out;
  }
  distributed_span first(size_type count) const { return subspan(0, count); }
  distributed_span last(size_type count) const { return subspan(size() - count, count); }

  iterator begin() const { return iterator(d_, 0); }
  iterator end() const { return iterator(d_, size()); }
  reference front() const { return (*this)[0]; }
  reference back() const { return (*this)[size() - 1]; }

  std::vector<segment_type> segments() const { return d_->segs; }

private:
  template <typename S> static void push(dspan_data<T> &d, S &&seg) {
    const std::size_t n = std::ranges::size(seg);
    const std::size_t rk = lib::ranges::rank(seg);
    T *p;
    if constexpr (requires { seg.data(); }) p = seg.data();
    else p = lib::ranges::local(std::ranges::begin(seg));
    d.segs.push_back(device_span<T>(p, n, rk));
    d.pre.push_back(d.pre.back() + n);
  }
  std::shared_ptr<const dspan_data<T>> d_;
};

namespace detail {
template <typename S> struct span_elem {
  using type = std::ranges::range_value_t<S>;
};
template <typename S>
  requires requires { typename S::element_type; }
struct span_elem<S> {
  using type = typename S::element_type;
};
} // namespace detail

template <std::ranges::input_range R>
  requires(lib::remote_range<std::ranges::range_reference_t<R>> && !lib::distributed_range<R>)
distributed_span(R &&) -> distributed_span<typename detail::span_elem<std::ranges::range_value_t<R>>::type>;

template <lib::distributed_range R>
distributed_span(R &&) -> distributed_span<std::ranges::range_value_t<R>>;

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

// shp::views::take (views/standard_views.hpp:17): the standard adaptor; its
// segments come from the distributed iterators (lib::ranges::segments).
inline constexpr auto take = std::views::take;
inline constexpr auto drop = std::views::drop;

// shp::views::slice (views/standard_views.hpp:19-42): the distributed_span of
// elements [lo, hi) of a distributed range
template <lib::distributed_range R> auto slice(R &&r, std::pair<std::size_t, std::size_t> idx) {
  using T = std::remove_reference_t<decltype(*lib::ranges::segments(r)[0].data())>;
  return distributed_span<T>(lib::ranges::segments(r)).subspan(idx.first, idx.second - idx.first);
}
struct slice_adaptor {
  std::pair<std::size_t, std::size_t> idx;
  template <lib::distributed_range R> auto operator()(R &&r) const { return slice(std::forward<R>(r), idx); }
};
inline slice_adaptor slice(std::pair<std::size_t, std::size_t> r) { return {r}; }
template <lib::distributed_range R> auto operator|(R &&r, slice_adaptor s) { return s(std::forward<R>(r)); }

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

