// dr/shp/index.hpp -- shp::index<T>, the 2-D matrix index / shape type.
//
// Same interface as containers/index.hpp:36-105: public `first` / `second`,
// operator[](dim), construction from two integers or any 2-tuple-like
// (std::pair, std::tuple, std::array, brace lists), widening conversion,
// equality and structured bindings (`auto [i, j] = idx`).
#pragma once

#include <array>
#include <concepts>
#include <cstddef>
#include <limits>
#include <tuple>
#include <utility>

namespace shp {

template <std::integral T = std::size_t> class index {
public:
  using index_type = T;
  using first_type = T;
  using second_type = T;

  index() = default;
  constexpr index(index_type f, index_type s) : first(f), second(s) {}
  template <typename Tuple>
    requires requires(Tuple t) {
      { std::get<0>(t) } -> std::convertible_to<T>;
      { std::get<1>(t) } -> std::convertible_to<T>;
      requires std::tuple_size_v<std::remove_cvref_t<Tuple>> == 2;
    }
  constexpr index(const Tuple &t) : first(static_cast<T>(std::get<0>(t))), second(static_cast<T>(std::get<1>(t))) {}

  constexpr index_type operator[](index_type dim) const noexcept { return dim == 0 ? first : second; }

  template <std::integral U>
    requires(std::numeric_limits<U>::max() >= std::numeric_limits<T>::max())
  constexpr operator index<U>() const noexcept {
    return index<U>(first, second);
  }

  constexpr bool operator==(const index &) const noexcept = default;

  template <std::size_t I>
    requires(I <= 1)
  constexpr T get() const noexcept {
    return I == 0 ? first : second;
  }

  index_type first = 0;
  index_type second = 0;
};

} // namespace shp

namespace std {
template <std::size_t I, std::integral T>
struct tuple_element<I, shp::index<T>> : tuple_element<I, std::tuple<T, T>> {};
template <std::integral T> struct tuple_size<shp::index<T>> : integral_constant<std::size_t, 2> {};
template <std::size_t I, std::integral T>
  requires(I <= 1)
constexpr T get(shp::index<T> idx) {
  return I == 0 ? idx.first : idx.second;
}
} // namespace std
