// dr/shp/memory.hpp -- device pointers, element proxies, allocators and the
// per-segment span/vector of the shp drop-in layer.
//
// Mirrors device_ptr.hpp:13-143, device_ref.hpp:12-50,
// allocators.hpp:13-72, device_span.hpp:43-84, vector.hpp:14-247 and
// device_vector.hpp:12-31.  Memory is HIP device memory on the segment's
// device (drhip_malloc); host element access through device_ref is a
// blocking one-element copy on the segment's stream, as in the reference
// (device_ref.hpp:23-44).  shared_allocator keeps the reference's name and
// default but allocates device memory too (SURVEY.md 7 "Memory model").
#pragma once

#include <compare>
#include <cstddef>
#include <iterator>
#include <type_traits>

#include "runtime.hpp"

namespace shp {

template <typename T> class device_ref {
public:
  using value_type = std::remove_const_t<T>;
  device_ref() = delete;
  device_ref(T *p, std::size_t rank) : p_(p), rank_(rank) {}
  device_ref(const device_ref &) = default;

  operator value_type() const {
    value_type v;
    detail::check(drhip_memcpy_d2h(static_cast<int>(rank_), &v, p_, sizeof(T)), "device_ref read");
    return v;
  }
  device_ref operator=(const value_type &v) const
    requires(!std::is_const_v<T>)
  {
    detail::check(drhip_memcpy_h2d(static_cast<int>(rank_), p_, &v, sizeof(T)), "device_ref write");
    return *this;
  }
  device_ref operator=(const device_ref &o) const
    requires(!std::is_const_v<T>)
  {
    return *this = value_type(o);
  }
  // read-modify-write helpers used by host loops such as std::iota
  device_ref operator++() const { return *this = value_type(*this) + 1; }
  device_ref operator+=(const value_type &v) const { return *this = value_type(*this) + v; }

  friend bool operator==(const device_ref &a, const value_type &b) { return value_type(a) == b; }
  friend bool operator==(const device_ref &a, const device_ref &b) { return value_type(a) == value_type(b); }

  T *raw() const { return p_; }
  std::size_t rank() const { return rank_; }

private:
  T *p_;
  std::size_t rank_;
};

// A random-access iterator over one segment's device memory.  `local()`
// is the raw device pointer (lib::ranges::local, details/ranges.hpp:133).
template <typename T> class device_ptr {
public:
  using value_type = std::remove_const_t<T>;
  using difference_type = std::ptrdiff_t;
  using reference = device_ref<T>;
  using pointer = device_ptr;
  using iterator_category = std::random_access_iterator_tag;
  using iterator_concept = std::random_access_iterator_tag;

  device_ptr() = default;
  device_ptr(T *p, std::size_t rank) : p_(p), rank_(rank) {}
  operator device_ptr<const T>() const { return device_ptr<const T>(p_, rank_); }

  reference operator*() const { return reference(p_, rank_); }
  reference operator[](difference_type i) const { return reference(p_ + i, rank_); }
  device_ptr &operator++() { ++p_; return *this; }
  device_ptr operator++(int) { auto t = *this; ++p_; return t; }
  device_ptr &operator--() { --p_; return *this; }
  device_ptr operator--(int) { auto t = *this; --p_; return t; }
  device_ptr &operator+=(difference_type d) { p_ += d; return *this; }
  device_ptr &operator-=(difference_type d) { p_ -= d; return *this; }
  friend device_ptr operator+(device_ptr a, difference_type d) { return a += d; }
  friend device_ptr operator+(difference_type d, device_ptr a) { return a += d; }
  friend device_ptr operator-(device_ptr a, difference_type d) { return a -= d; }
  friend difference_type operator-(const device_ptr &a, const device_ptr &b) { return a.p_ - b.p_; }
  friend bool operator==(const device_ptr &a, const device_ptr &b) { return a.p_ == b.p_; }
  friend auto operator<=>(const device_ptr &a, const device_ptr &b) { return a.p_ <=> b.p_; }

  T *local() const { return p_; }
  T *get_raw_pointer() const { return p_; }
  std::size_t rank() const { return rank_; }

private:
  T *p_ = nullptr;
  std::size_t rank_ = 0;
};

// allocators.hpp:17-72: allocates on the segment (rank) it is bound to.
// The reference binds an allocator to (context, device); here the device is
// a HIP ordinal and the allocation goes to the first segment on it
// (test_range.cpp: device_allocator<T>(context, devices[rank])).
template <typename T> class device_allocator {
public:
  using value_type = T;
  using pointer = device_ptr<T>;
  using const_pointer = device_ptr<const T>;
  device_allocator() = default;
  explicit device_allocator(std::size_t rank) : rank_(rank) {}
  device_allocator(const context_type &, int device) : rank_(detail::segment_of_device(device)) {}
  template <typename U> device_allocator(const device_allocator<U> &o) : rank_(o.rank()) {}

  pointer allocate(std::size_t n) {
    void *p = nullptr;
    detail::check(drhip_malloc(static_cast<int>(rank_), n * sizeof(T), &p), "drhip_malloc");
    return pointer(static_cast<T *>(p), rank_);
  }
  void deallocate(pointer p, std::size_t) { (void)drhip_free(static_cast<int>(rank_), p.local()); }
  std::size_t rank() const { return rank_; }
  bool operator==(const device_allocator &) const = default;

private:
  std::size_t rank_ = 0;
};

// allocators.hpp:13-15 (USM shared in the reference; device memory here).
template <typename T> using shared_allocator = device_allocator<T>;

// One segment's contiguous device range: device_span.hpp:43-84.  The second
// parameter is the reference's iterator type (T* for USM, device_ptr<T> for
// device allocations); every form stores the raw device pointer and its
// segment rank, and converts to device_span<T>.
template <typename T, typename L = T *>
class device_span : public std::ranges::view_interface<device_span<T, L>> {
public:
  using value_type = std::remove_const_t<T>;
  using element_type = T;
  using iterator = device_ptr<T>;
  using size_type = std::size_t;
  using difference_type = std::ptrdiff_t;
  device_span() = default;
  device_span(T *data, std::size_t size, std::size_t rank) : data_(data), size_(size), rank_(rank) {}
  device_span(device_ptr<T> first, std::size_t size) : data_(first.local()), size_(size), rank_(first.rank()) {}
  device_span(device_ptr<T> first, std::size_t size, std::size_t rank)
      : data_(first.local()), size_(size), rank_(rank) {}
  template <typename L2>
    requires(!std::is_same_v<L, L2>)
  device_span(const device_span<T, L2> &o) : data_(o.data()), size_(o.size()), rank_(o.rank()) {}

  iterator begin() const { return iterator(data_, rank_); }
  iterator end() const { return iterator(data_ + size_, rank_); }
  std::size_t size() const { return size_; }
  bool empty() const { return size_ == 0; }
  device_ref<T> operator[](std::size_t i) const { return device_ref<T>(data_ + i, rank_); }
  T *data() const { return data_; }
  std::size_t rank() const { return rank_; }
  device_span subspan(std::size_t off, std::size_t count) const {
    return device_span(data_ + off, count, rank_);
  }
  device_span first(std::size_t count) const { return subspan(0, count); }
  device_span last(std::size_t count) const { return subspan(size_ - count, count); }

private:
  T *data_ = nullptr;
  std::size_t size_ = 0;
  std::size_t rank_ = 0;
};

namespace detail {

template <typename S> constexpr bool is_device_span = false;
template <typename T, typename L> constexpr bool is_device_span<device_span<T, L>> = true;

template <typename T> __global__ void fill_any_kernel(T *p, std::size_t n, T v) {
  for (std::size_t i = blockIdx.x * (std::size_t)blockDim.x + threadIdx.x; i < n;
       i += (std::size_t)gridDim.x * blockDim.x)
    p[i] = v;
}

// Asynchronous fill of one segment on its stream: the C-ABI kernel for
// 1/2/4/8-byte elements, a template kernel for any other trivially copyable
// T (copy.hpp:147-168 fill_async accepts any T).
template <typename T> void fill_segment_async(std::size_t rank, T *p, std::size_t n, const T &value) {
  if (n == 0) return;
  if constexpr (sizeof(T) == 1 || sizeof(T) == 2 || sizeof(T) == 4 || sizeof(T) == 8) {
    check(drhip_fill(static_cast<int>(rank), p, n, &value, sizeof(T)), "drhip_fill");
  } else {
    void *s = nullptr;
    check(drhip_stream(static_cast<int>(rank), &s), "drhip_stream");
    const std::size_t blocks = std::min<std::size_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL((fill_any_kernel<T>), dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                       static_cast<hipStream_t>(s), p, n, value);
    hip_check(hipGetLastError(), "fill launch");
  }
}

} // namespace detail

// vector.hpp:14-247 + device_vector.hpp:12-31: an owning segment.  The
// reference fills twice at construction (vector.hpp:43 with an indeterminate
// T, then distributed_vector.hpp:153 with T{}); here the zero fill is done
// once by the distributed_vector.
template <typename T, typename Alloc = device_allocator<T>> class device_vector {
public:
  using value_type = T;
  device_vector() = default;
  device_vector(std::size_t n, Alloc alloc, std::size_t rank) : alloc_(alloc), size_(n), rank_(rank) {
    if (n) data_ = alloc_.allocate(n).local();
  }
  device_vector(const device_vector &) = delete;
  device_vector &operator=(const device_vector &) = delete;
  device_vector(device_vector &&o) noexcept { swap(o); }
  device_vector &operator=(device_vector &&o) noexcept {
    swap(o);
    return *this;
  }
  ~device_vector() {
    if (data_) alloc_.deallocate(device_ptr<T>(data_, rank_), size_);
  }
  void swap(device_vector &o) noexcept {
    std::swap(alloc_, o.alloc_);
    std::swap(data_, o.data_);
    std::swap(size_, o.size_);
    std::swap(rank_, o.rank_);
  }
  T *data() const { return data_; }
  std::size_t size() const { return size_; }
  std::size_t rank() const { return rank_; }
  device_span<T> span() const { return device_span<T>(data_, size_, rank_); }

private:
  Alloc alloc_{};
  T *data_ = nullptr;
  std::size_t size_ = 0;
  std::size_t rank_ = 0;
};

} // namespace shp
