// dr/shp/vector.hpp -- shp::vector<T, Allocator>: a growable array whose
// storage comes from Allocator (vector.hpp:14-247 of the reference).  With
// std::allocator it is a host vector; with shp::device_allocator<T> its
// pointer and iterators are device_ptr<T> into one segment's HIP memory, so
// element access is a device_ref (blocking one-element copy) and bulk moves
// (reserve, copy construction, assign) go through shp::copy -- one HIP copy
// each instead of an element loop.  Like the reference, elements are not
// constructed or destroyed: T must be trivially copyable.
#pragma once

#include <initializer_list>
#include <iterator>
#include <memory>

#include "algorithms.hpp"

namespace shp {

template <typename T, typename Allocator = std::allocator<T>> class vector {
  static_assert(std::is_trivially_copyable_v<T>, "shp::vector: T must be trivially copyable");

public:
  using value_type = T;
  using allocator_type = Allocator;
  using size_type = std::size_t;
  using difference_type = std::ptrdiff_t;
  using pointer = typename std::allocator_traits<allocator_type>::pointer;
  using const_pointer = typename std::allocator_traits<allocator_type>::const_pointer;
  using reference = decltype(*std::declval<pointer>());
  using const_reference = decltype(*std::declval<const_pointer>());
  using iterator = pointer;
  using const_iterator = const_pointer;

  vector() noexcept {}
  explicit vector(const Allocator &allocator) noexcept : allocator_(allocator) {}

  // vector.hpp:33-40: count copies of value
  vector(size_type count, const T &value, const Allocator &alloc = Allocator()) : allocator_(alloc) {
    change_capacity_impl_(count);
    fill_impl_(begin(), end(), value);
  }
  // vector.hpp:42-48: count elements (the reference fills with an
  // indeterminate T; here value-initialised, i.e. zero for arithmetic T)
  explicit vector(size_type count, const Allocator &alloc = Allocator()) : allocator_(alloc) {
    change_capacity_impl_(count);
    fill_impl_(begin(), end(), T{});
  }
  template <std::forward_iterator Iter>
  vector(Iter first, Iter last, const Allocator &alloc = Allocator()) : allocator_(alloc) {
    change_capacity_impl_(static_cast<size_type>(std::distance(first, last)));
    copy_impl_(first, last, begin());
  }
  vector(const vector &other)
      : allocator_(std::allocator_traits<allocator_type>::select_on_container_copy_construction(other.allocator_)) {
    change_capacity_impl_(other.size());
    copy_impl_(other.begin(), other.end(), begin());
  }
  vector(const vector &other, const Allocator &alloc) : allocator_(alloc) {
    change_capacity_impl_(other.size());
    copy_impl_(other.begin(), other.end(), begin());
  }
  vector(vector &&other) noexcept : allocator_(std::move(other.allocator_)) { steal_(other); }
  vector(vector &&other, const Allocator &alloc) noexcept : allocator_(alloc) { steal_(other); }
  vector(std::initializer_list<T> init, const Allocator &alloc = Allocator()) : allocator_(alloc) {
    change_capacity_impl_(init.size());
    copy_impl_(init.begin(), init.end(), begin());
  }

  vector &operator=(const vector &other) {
    if (this != &other) assign(other.begin(), other.end());
    return *this;
  }
  vector &operator=(vector &&other) noexcept {
    if (this != &other) {
      release_();
      allocator_ = std::move(other.allocator_);
      steal_(other);
    }
    return *this;
  }

  template <std::forward_iterator Iter> void assign(Iter first, Iter last) {
    const auto new_size = static_cast<size_type>(std::distance(first, last));
    reserve(new_size);
    copy_impl_(first, last, begin());
    size_ = new_size;
  }

  ~vector() noexcept { release_(); }

  size_type size() const noexcept { return size_; }
  bool empty() const noexcept { return size() == 0; }
  size_type capacity() const noexcept { return capacity_; }
  pointer data() noexcept { return data_; }
  const_pointer data() const noexcept { return data_; }
  allocator_type get_allocator() const noexcept { return allocator_; }

  iterator begin() noexcept { return data_; }
  iterator end() noexcept { return begin() + size(); }
  const_iterator begin() const noexcept { return data_; }
  const_iterator end() const noexcept { return begin() + size(); }

  reference operator[](size_type pos) { return *(begin() + pos); }
  const_reference operator[](size_type pos) const { return *(begin() + pos); }

  // vector.hpp:149-167: grow to new_cap, moving the contents with one copy
  void reserve(size_type new_cap) {
    if (new_cap <= capacity()) return;
    pointer new_data = allocator_.allocate(new_cap);
    if (size()) copy_impl_(begin(), end(), new_data);
    if (data_ != pointer{}) allocator_.deallocate(data_, capacity());
    data_ = new_data;
    capacity_ = new_cap;
  }

  // vector.hpp:169-188: capacity doubles (next power of two)
  void push_back(const T &value) {
    if (size() + 1 > capacity()) reserve(next_pow2_(capacity() + 1));
    data()[size()] = value;
    ++size_;
  }
  void push_back(T &&value) { push_back(static_cast<const T &>(value)); }
  bool try_push_back(const T &value) {
    if (size() + 1 > capacity()) return false;
    data()[size()] = value;
    ++size_;
    return true;
  }

  // vector.hpp:199-225
  void resize(size_type count) { resize(count, T{}); }
  void resize(size_type count, const value_type &value) {
    if (count > capacity()) reserve(count);
    if (count > size()) fill_impl_(end(), begin() + count, value);
    size_ = count;
  }

private:
  static constexpr bool on_device = !std::is_pointer_v<pointer>;

  template <typename In, typename Out> static void copy_impl_(In first, In last, Out d_first) {
    if (first == last) return;
    if constexpr (requires { d_first.local(); } || requires { first.local(); })
      shp::copy(first, last, d_first); // one HIP copy (h2d, d2h or d2d)
    else
      std::copy(first, last, d_first);
  }
  static void fill_impl_(iterator first, iterator last, const T &value) {
    if (first == last) return;
    if constexpr (on_device) shp::fill(first, last, value);
    else std::fill(first, last, value);
  }
  void change_capacity_impl_(size_type count) {
    release_();
    size_ = capacity_ = count;
    data_ = count ? allocator_.allocate(count) : pointer{};
  }
  void release_() noexcept {
    if (data_ != pointer{}) allocator_.deallocate(data_, capacity_);
    data_ = pointer{};
    size_ = capacity_ = 0;
  }
  void steal_(vector &other) noexcept {
    data_ = other.data_;
    size_ = other.size_;
    capacity_ = other.capacity_;
    other.data_ = pointer{};
    other.size_ = other.capacity_ = 0;
  }
  static constexpr size_type next_pow2_(size_type n) {
    size_type p = 1;
    while (p < n) p <<= 1;
    return p;
  }

  allocator_type allocator_{};
  pointer data_{};
  size_type size_ = 0;
  size_type capacity_ = 0;
};

} // namespace shp
