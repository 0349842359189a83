// dr/shp.hpp -- the shp drop-in API on MI355X (include/dr/shp/shp.hpp of the
// reference).  Header-only C++20, compiled with hipcc --offload-arch=gfx950
// and linked against libdrhip.so (the C-ABI of include/drhip.h).
#pragma once

#include "shp/runtime.hpp"
#include "shp/memory.hpp"
#include "shp/ranges.hpp"
#include "shp/algorithms.hpp"
#include "shp/sort.hpp"
#include "shp/vector.hpp"
#include "shp/sparse.hpp"
#include "shp/dense.hpp"
#include "shp/util.hpp"

namespace rng = std::ranges;

namespace dr {
namespace shp = ::shp;
} // namespace dr
