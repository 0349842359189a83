// dr/shp/util.hpp -- printing helpers of shp/util.hpp:138-210
// (print_range, print_matrix, print_range_details).  Device data is copied
// to the host once per call instead of element by element through
// device_ref proxies.
#pragma once

#include <iostream>
#include <string>
#include <vector>

#include "algorithms.hpp"
#include "sparse.hpp"

namespace shp {

namespace detail {
template <typename R> auto host_values(R &&r) {
  using V = std::remove_cvref_t<std::ranges::range_value_t<R>>;
  std::vector<V> h;
  if constexpr (lib::distributed_contiguous_range<R>) {
    h.resize(std::ranges::size(r));
    std::size_t off = 0;
    for (auto &&s : lib::ranges::segments(r)) {
      if (s.size())
        detail::check(drhip_memcpy_d2h(static_cast<int>(lib::ranges::rank(s)), h.data() + off, s.data(),
                                       s.size() * sizeof(V)),
                      "print d2h");
      off += s.size();
    }
  } else {
    for (auto &&v : r) h.push_back(static_cast<V>(v));
  }
  return h;
}
} // namespace detail

// util.hpp:138-166: "[a, b, ...]" with 10 values per line, aligned under
// the label
template <typename Range> void print_range(Range &&r, std::string label = "") {
  std::size_t indent = 1;
  if (!label.empty()) {
    std::cout << "\"" << label << "\": ";
    indent += label.size() + 4;
  }
  const std::string pad(indent, ' ');
  const auto h = detail::host_values(r);
  std::cout << "[";
  for (std::size_t i = 0; i < h.size(); i++) {
    std::cout << h[i];
    if (i + 1 < h.size()) {
      std::cout << ", ";
      if ((i + 1) % 10 == 0) std::cout << "\n" << pad;
    }
  }
  std::cout << "]" << std::endl;
}

// util.hpp:167-182
template <typename Matrix> void print_matrix(Matrix &&m, std::string label = "") {
  std::cout << m.shape()[0] << " x " << m.shape()[1] << " matrix with " << m.size() << " stored values";
  if (!label.empty()) std::cout << " \"" << label << "\"";
  std::cout << std::endl;
  for (auto &&entry : m) {
    auto &&[index, value] = entry;
    auto &&[i, j] = index;
    std::cout << "(" << i << ", " << j << "): " << value << std::endl;
  }
}

// util.hpp:184-197
template <typename R> void print_range_details(R &&r, std::string label = "") {
  if (!label.empty()) std::cout << "\"" << label << "\" ";
  auto segs = lib::ranges::segments(r);
  std::cout << "distributed range with " << std::ranges::size(segs) << " segments." << std::endl;
  std::size_t idx = 0;
  for (auto &&s : segs)
    std::cout << "Seg " << idx++ << ", size " << s.size() << " (rank " << lib::ranges::rank(s) << ")" << std::endl;
}

} // namespace shp
