// shp_tests.cpp -- the reference's shp gtests (test/gtest/shp/*.cpp) restated
// against the MI355X drop-in layer (distributed-ranges_amd/include/dr/shp.hpp),
// plus the float / large-n / sort / gemv / dot coverage SURVEY.md 4 asks for.
//
// gtest and cxxopts are not available offline, so this carries a minimal
// runner with the same test names and the same --devicesCount option as
// test/gtest/shp/shp-tests.cpp:14-41 (duplicate the device list up to N:
// one MI355X then hosts N segments, each with its own stream).
//
// Host-side oracles are the std:: algorithms on a std::vector, exactly the
// reference's pattern (algorithms.cpp:46-47, :74).
#include <dr/shp.hpp>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <random>
#include <string>
#include <vector>
#include <tuple>
#include <unistd.h>

// ------------------------------------------------------------ mini runner
struct TestCase {
  const char *suite, *name;
  void (*fn)();
};
static std::vector<TestCase> &registry() {
  static std::vector<TestCase> r;
  return r;
}
static int g_fail = 0;
static bool g_cur_failed = false;
#define TEST(S, N)                                                                       \
  static void S##_##N();                                                                 \
  static const int S##_##N##_reg = (registry().push_back({#S, #N, &S##_##N}), 0);         \
  static void S##_##N()
#define EXPECT_TRUE(c)                                                                   \
  do {                                                                                   \
    if (!(c)) {                                                                          \
      std::printf("  %s:%d: EXPECT_TRUE(%s) failed\n", __FILE__, __LINE__, #c);          \
      g_cur_failed = true;                                                               \
    }                                                                                    \
  } while (0)
#define EXPECT_EQ(a, b)                                                                  \
  do {                                                                                   \
    auto va_ = (a);                                                                      \
    auto vb_ = (b);                                                                      \
    if (!(va_ == vb_)) {                                                                 \
      std::printf("  %s:%d: EXPECT_EQ(%s, %s) failed: %s vs %s\n", __FILE__, __LINE__, #a, #b, \
                  std::to_string(va_).c_str(), std::to_string(vb_).c_str());              \
      g_cur_failed = true;                                                               \
    }                                                                                    \
  } while (0)
#define EXPECT_NEAR_REL(a, b, tol)                                                       \
  do {                                                                                   \
    const double va_ = (double)(a), vb_ = (double)(b);                                   \
    if (!(std::fabs(va_ - vb_) <= (tol) * std::max(std::fabs(vb_), 1e-30))) {            \
      std::printf("  %s:%d: |%s - %s| rel > %g: %.9g vs %.9g\n", __FILE__, __LINE__, #a, #b, (double)(tol), va_, vb_); \
      g_cur_failed = true;                                                               \
    }                                                                                    \
  } while (0)

// common-tests.hpp:12-69
template <typename R1, typename R2> bool is_equal(R1 &&r1, R2 &&r2) {
  auto a = std::ranges::begin(r1);
  auto b = std::ranges::begin(r2);
  for (; a != std::ranges::end(r1) && b != std::ranges::end(r2); ++a, ++b)
    if (!(*a == *b)) return false;
  return true;
}
template <typename R1, typename R2> bool equal(R1 &&r1, R2 &&r2) { return is_equal(r1, r2); }
template <typename R1, typename R2, typename R3> bool unary_check(R1 &&, R2 &&ref, R3 &&tst) { return is_equal(ref, tst); }

template <typename T> std::vector<T> to_host(const shp::distributed_vector<T> &dv) {
  std::vector<T> h(dv.size());
  shp::copy(dv.begin(), dv.end(), h.begin());
  return h;
}

using T = int;
using DV = shp::distributed_vector<T, shp::shared_allocator<T>>;
using V = std::vector<T>;

// ------------------------------------------------- algorithms.cpp:11-149
TEST(ShpTests, Iota) {
  const int n = 10;
  V a(n);
  DV dv_a(n);
  std::iota(a.begin(), a.end(), 20);
  std::iota(dv_a.begin(), dv_a.end(), 20);
  EXPECT_TRUE(equal(a, dv_a));
}

struct negate {
  __host__ __device__ void operator()(auto &v) const { v = -v; }
};

TEST(ShpTests, ForEach) {
  std::size_t n = 10;
  V a(n), a_in(n);
  std::iota(a.begin(), a.end(), 100);
  std::iota(a_in.begin(), a_in.end(), 100);
  std::ranges::for_each(a, negate{});
  DV dv_a(n);
  std::iota(dv_a.begin(), dv_a.end(), 100);
  shp::for_each(shp::par_unseq, dv_a, negate{});
  EXPECT_TRUE(unary_check(a_in, a, dv_a));
}

TEST(ShpTests, ReduceBasic) {
  std::size_t n = 10;
  V v(n);
  std::iota(v.begin(), v.end(), 10);
  DV dv(n);
  std::iota(dv.begin(), dv.end(), 10);
  auto dvalue = shp::reduce(shp::par_unseq, dv, int(0), std::plus<>());
  auto value = std::reduce(v.begin(), v.end(), int(0), std::plus<>());
  EXPECT_EQ(dvalue, value);
  EXPECT_EQ(dvalue, 145); // tests/golden/shp_known_answers.json reduce_basic
  EXPECT_EQ(dvalue, shp::reduce(shp::par_unseq, dv.begin(), dv.end(), int(0), std::plus<>()));
  EXPECT_EQ(dvalue, shp::reduce(shp::par_unseq, dv.begin(), dv.end(), int(0)));
  EXPECT_EQ(dvalue, shp::reduce(shp::par_unseq, dv.begin(), dv.end()));
  EXPECT_EQ(dvalue, shp::reduce(shp::par_unseq, dv, int(0)));
  EXPECT_EQ(dvalue, shp::reduce(shp::par_unseq, dv));
}

TEST(ShpTests, InclusiveScan) {
  std::size_t n = 100;
  shp::distributed_vector<int, shp::device_allocator<int>> v(n);
  shp::distributed_vector<int, shp::device_allocator<int>> o(v.size() * 2);
  std::vector<int> lv(n);
  auto check = [&](auto &&out) {
    for (std::size_t i = 0; i < lv.size(); i++) EXPECT_EQ((int)out[i], lv[i]);
  };
  // Range case, no binary op or init, perfectly aligned
  for (auto &&x : lv) x = lrand48() % 100;
  shp::copy(lv.begin(), lv.end(), v.begin());
  std::inclusive_scan(lv.begin(), lv.end(), lv.begin());
  shp::inclusive_scan(shp::par_unseq, v, v);
  check(v);
  // Range case, binary op no init, non-aligned ranges
  for (auto &&x : lv) x = lrand48() % 100;
  shp::copy(lv.begin(), lv.end(), v.begin());
  std::inclusive_scan(lv.begin(), lv.end(), lv.begin());
  shp::inclusive_scan(shp::par_unseq, v, o, std::plus<>());
  check(o);
  // Range case, binary op, init, non-aligned ranges (wrapping int32 products)
  for (auto &&x : lv) x = lrand48() % 100;
  shp::copy(lv.begin(), lv.end(), v.begin());
  {
    std::vector<unsigned> u(lv.begin(), lv.end());
    std::inclusive_scan(u.begin(), u.end(), u.begin(), std::multiplies<>(), 12u);
    for (std::size_t i = 0; i < n; i++) lv[i] = (int)u[i];
  }
  shp::inclusive_scan(shp::par_unseq, v, o, std::multiplies<>(), 12);
  check(o);
  // Iterator case, no binary op or init, perfectly aligned
  for (auto &&x : lv) x = lrand48() % 100;
  shp::copy(lv.begin(), lv.end(), v.begin());
  std::inclusive_scan(lv.begin(), lv.end(), lv.begin());
  shp::inclusive_scan(shp::par_unseq, v.begin(), v.end(), v.begin());
  check(v);
  // Iterator case, binary op no init, non-aligned ranges
  for (auto &&x : lv) x = lrand48() % 100;
  shp::copy(lv.begin(), lv.end(), v.begin());
  std::inclusive_scan(lv.begin(), lv.end(), lv.begin());
  auto d_last = shp::inclusive_scan(shp::par_unseq, v.begin(), v.end(), o.begin(), std::plus<>());
  EXPECT_TRUE(d_last == o.begin() + n);
  check(o);
  // Iterator case, binary op, init, non-aligned ranges
  for (auto &&x : lv) x = lrand48() % 100;
  shp::copy(lv.begin(), lv.end(), v.begin());
  {
    std::vector<unsigned> u(lv.begin(), lv.end());
    std::inclusive_scan(u.begin(), u.end(), u.begin(), std::multiplies<>(), 12u);
    for (std::size_t i = 0; i < n; i++) lv[i] = (int)u[i];
  }
  shp::inclusive_scan(shp::par_unseq, v.begin(), v.end(), o.begin(), std::multiplies<>(), 12);
  check(o);
}

// --------------------------------------------------------- views.cpp
struct increment {
  __host__ __device__ void operator()(auto &&v) const { v++; }
};

TEST(ShpTests, Take) {
  const int n = 10;
  V a(n);
  DV dv_a(n);
  std::iota(a.begin(), a.end(), 20);
  std::iota(dv_a.begin(), dv_a.end(), 20);
  auto aview = a | rng::views::take(2);
  auto dv_aview = dv_a | rng::views::take(2);
  EXPECT_TRUE(equal(aview, dv_aview));
  std::ranges::for_each(aview, increment{});
  shp::for_each(shp::par_unseq, dv_aview, increment{});
  EXPECT_TRUE(equal(aview, dv_aview));
}

TEST(ShpTests, Zip) {
  const int n = 10;
  DV dv_a(n), dv_b(n);
  shp::iota(dv_a, 100);
  shp::iota(dv_b, 200);
  auto dz = shp::views::zip(dv_a, dv_b, dv_a);
  auto dzi = shp::views::zip(rng::views::iota(1, 10), dv_b, dv_a);
  V v_a(n), v_b(n);
  std::iota(v_a.begin(), v_a.end(), 100);
  std::iota(v_b.begin(), v_b.end(), 200);
  std::vector<std::tuple<int, int, int>> z, zi;
  for (int i = 0; i < n; i++) z.emplace_back(v_a[i], v_b[i], v_a[i]);
  for (int i = 0; i < 9; i++) zi.emplace_back(i + 1, v_b[i], v_a[i]);
  EXPECT_TRUE(equal(z, dz));
  EXPECT_TRUE(equal(zi, dzi));
  EXPECT_EQ(dzi.size(), std::size_t(9));
  // zipped segments cover the range, one piece per intersected segment
  std::size_t tot = 0;
  for (auto &s : dz.zipped_segments()) tot += s.size();
  EXPECT_EQ(tot, std::size_t(n));
}

TEST(ShpTests, Drop) {
  const int n = 10;
  V a(n);
  DV dv_a(n);
  auto incr = [](auto &&v) { v++; };
  std::iota(a.begin(), a.end(), 20);
  std::iota(dv_a.begin(), dv_a.end(), 20);
  auto aview = a | rng::views::drop(2);
  auto dv_aview = dv_a | rng::views::drop(2);
  EXPECT_TRUE(equal(aview, dv_aview));
  std::ranges::for_each(aview, incr);
  shp::for_each(shp::par_unseq, dv_aview, incr);
  EXPECT_TRUE(equal(aview, dv_aview));
  EXPECT_TRUE(equal(a, dv_a));
}

TEST(ShpTests, Transform) {
  const int n = 10;
  DV dv_a(n);
  shp::iota(dv_a, 20);
  auto plus1 = [](auto x) { return x + 1; };
  auto dv_a_view = lib::views::transform(dv_a, plus1);
  V v_a(n);
  std::iota(v_a.begin(), v_a.end(), 20);
  auto v_a_view = rng::views::transform(v_a, plus1);
  EXPECT_TRUE(equal(v_a_view, dv_a_view));
  // a transform view reduces on the device through the template kernel
  EXPECT_EQ(shp::reduce(shp::par_unseq, dv_a_view, 0, std::plus<>()), std::reduce(v_a_view.begin(), v_a_view.end()));
}

// ----------------------------------------------------------- copy.cpp
TEST(ShpTests, Copy_Dist2Local) {
  const int n = 100;
  std::size_t n_to_copy = 20;
  V a(n_to_copy);
  shp::distributed_vector<T, shp::device_allocator<T>> dv_a(n);
  shp::iota(dv_a, 0);
  for (std::size_t i = 0; i + n_to_copy <= n; i += n_to_copy) {
    shp::copy(dv_a.begin() + i, dv_a.begin() + i + n_to_copy, a.begin());
    auto dv_aview = dv_a | shp::views::slice({i, i + n_to_copy});
    EXPECT_TRUE(equal(a, dv_aview));
  }
}

TEST(ShpTests, Copy_Local2Dist) {
  const int n = 100;
  std::size_t n_to_copy = 20;
  V a(n_to_copy);
  shp::distributed_vector<T, shp::device_allocator<T>> dv_a(n);
  std::iota(a.begin(), a.end(), 0);
  for (std::size_t i = 0; i + n_to_copy <= n; i += n_to_copy) {
    shp::copy(a.begin(), a.end(), dv_a.begin() + i);
    auto dv_aview = dv_a | shp::views::slice({i, i + n_to_copy});
    EXPECT_TRUE(equal(a, dv_aview));
  }
}

// ------------------------------------------------------ containers.cpp
TEST(ShpTests, DistributedVector) {
  using CDV = const shp::distributed_vector<int>;
  static_assert(rng::random_access_range<DV>);
  static_assert(rng::random_access_range<CDV>);
  static_assert(lib::distributed_range<DV>);
  static_assert(lib::distributed_contiguous_range<DV>);
}

TEST(ShpTests, DistributedVectorSegments) {
  const int n = 10;
  DV dv_a(n);
  std::iota(dv_a.begin(), dv_a.end(), 20);
  auto second = dv_a.begin() + 2;
  EXPECT_EQ((int)second[0], (int)lib::ranges::segments(second)[0][0]);
  // block distribution: segment i = [i*s, min((i+1)*s, n)), s = ceil(n/P)
  const std::size_t P = shp::nprocs(), s = (n + P - 1) / P;
  std::size_t k = 0, tot = 0;
  for (auto &seg : dv_a.segments()) {
    EXPECT_EQ(lib::ranges::rank(seg), k);
    EXPECT_EQ(seg.size(), std::min<std::size_t>(s, n - k * s));
    tot += seg.size();
    k++;
  }
  EXPECT_EQ(tot, std::size_t(n));
}

// --------------------------------------- beyond the reference's int tests
TEST(ShpExtra, ReduceFloatLarge) {
  const std::size_t n = (1 << 22) + 7;
  std::vector<float> h(n);
  std::mt19937_64 g(1);
  std::uniform_real_distribution<float> u(0, 1);
  for (auto &x : h) x = u(g);
  shp::distributed_vector<float> dv(n);
  shp::copy(h.begin(), h.end(), dv.begin());
  double ref = 0;
  for (float x : h) ref += x;
  EXPECT_NEAR_REL(shp::reduce(shp::par_unseq, dv, 0.0f, std::plus<>()), ref, 1e-5);
  EXPECT_NEAR_REL(shp::reduce(shp::par_unseq, dv, 0.0f, shp::maximum<>()), *std::max_element(h.begin(), h.end()), 0);
  // generic lambda operator -> template kernel path
  auto mx = shp::reduce(shp::par_unseq, dv, 0.0f, [](float a, float b) { return a < b ? b : a; });
  EXPECT_NEAR_REL(mx, *std::max_element(h.begin(), h.end()), 0);
}

TEST(ShpExtra, DotProduct) {
  // examples/shp/dot_product.cpp:11-18
  const std::size_t n = 1000003;
  std::vector<float> hx(n), hy(n);
  std::mt19937_64 g(2);
  std::uniform_real_distribution<float> u(0, 1);
  for (std::size_t i = 0; i < n; i++) hx[i] = u(g), hy[i] = u(g);
  shp::distributed_vector<float> x(n), y(n);
  shp::copy(hx.begin(), hx.end(), x.begin());
  shp::copy(hy.begin(), hy.end(), y.begin());
  double ref = 0;
  for (std::size_t i = 0; i < n; i++) ref += (double)hx[i] * hy[i];
  auto z = shp::views::zip(x, y) | lib::views::transform([](auto &&e) {
             auto &&[a, b] = e;
             return a * b;
           });
  EXPECT_NEAR_REL(shp::reduce(shp::par_unseq, z, 0.0f, std::plus()), ref, 1e-5);
  EXPECT_NEAR_REL(shp::transform_reduce(shp::par_unseq, x, y, 0.0f), ref, 1e-5);
}

TEST(ShpExtra, InclusiveScanFloatLarge) {
  const std::size_t n = (1 << 21) + 5;
  std::vector<float> h(n);
  std::mt19937_64 g(3);
  std::uniform_real_distribution<float> u(0, 1);
  for (auto &x : h) x = u(g);
  shp::distributed_vector<float> v(n), o(n);
  shp::copy(h.begin(), h.end(), v.begin());
  shp::inclusive_scan(shp::par_unseq, v, o, std::plus<>(), 0.5f);
  auto got = to_host(o);
  double run = 0.5, worst = 0;
  for (std::size_t i = 0; i < n; i++) {
    run += h[i];
    worst = std::max(worst, std::fabs(got[i] - run) / run);
  }
  EXPECT_TRUE(worst <= 1e-5);
}

TEST(ShpExtra, ScanGenericAndExclusive) {
  const std::size_t n = 100003;
  std::vector<int> h(n);
  for (auto &x : h) x = (int)(lrand48() % 1000) - 500;
  shp::distributed_vector<int> v(n), o(n);
  shp::copy(h.begin(), h.end(), v.begin());
  // generic (lambda) max-scan: template kernels
  shp::inclusive_scan(shp::par_unseq, v, o, [](int a, int b) { return a < b ? b : a; });
  std::vector<int> ref(n);
  std::inclusive_scan(h.begin(), h.end(), ref.begin(), [](int a, int b) { return a < b ? b : a; });
  EXPECT_TRUE(to_host(o) == ref);
  shp::exclusive_scan(shp::par_unseq, v, o, 7);
  std::exclusive_scan(h.begin(), h.end(), ref.begin(), 7);
  EXPECT_TRUE(to_host(o) == ref);
}

template <typename K> static void sort_case(std::size_t n, std::uint64_t seed) {
  std::vector<K> h(n);
  std::mt19937_64 g(seed);
  for (auto &x : h) {
    if constexpr (std::is_floating_point_v<K>) x = (K)std::normal_distribution<double>(0, 1e3)(g);
    else x = (K)g();
    if constexpr (std::is_floating_point_v<K>)
      if (x == 0) x = 1;
  }
  shp::distributed_vector<K> dv(n);
  shp::copy(h.begin(), h.end(), dv.begin());
  shp::sort(shp::par_unseq, dv);
  std::sort(h.begin(), h.end());
  EXPECT_TRUE(to_host(dv) == h);
}

TEST(ShpExtra, Sort) {
  sort_case<std::uint32_t>(1000003, 1);
  sort_case<std::int32_t>(77777, 2);
  sort_case<float>(500001, 3);
  sort_case<std::int64_t>(65539, 4);
  sort_case<double>(33333, 5);
  // many duplicates across segment boundaries (exact splitting of ties)
  std::vector<int> h(200000);
  for (std::size_t i = 0; i < h.size(); i++) h[i] = (int)(i % 3);
  shp::distributed_vector<int> dv(h.size());
  shp::copy(h.begin(), h.end(), dv.begin());
  shp::sort(shp::par_unseq, dv, std::less<>());
  std::sort(h.begin(), h.end());
  EXPECT_TRUE(to_host(dv) == h);
}

template <typename K> static void sort_greater_case(std::size_t n, std::uint64_t seed, std::uint64_t mod) {
  std::vector<K> h(n);
  std::mt19937_64 g(seed);
  for (auto &x : h) {
    if constexpr (std::is_floating_point_v<K>) x = (K)std::normal_distribution<double>(0, 1e3)(g);
    else x = mod ? (K)(g() % mod) : (K)g();
    if constexpr (std::is_floating_point_v<K>)
      if (x == 0) x = 1;
  }
  shp::distributed_vector<K> dv(n);
  shp::copy(h.begin(), h.end(), dv.begin());
  shp::sort(shp::par_unseq, dv, std::greater<>());
  std::sort(h.begin(), h.end(), std::greater<>());
  EXPECT_TRUE(to_host(dv) == h);
}

TEST(ShpExtra, SortGreater) {
  // std::greater (descending) for every ABI key type, heavy duplicates, the
  // iterator form and a sub-range
  sort_greater_case<std::uint32_t>(1000003, 11, 0);
  sort_greater_case<std::int32_t>(77777, 12, 0);
  sort_greater_case<std::int32_t>(200001, 13, 5);
  sort_greater_case<float>(500001, 14, 0);
  sort_greater_case<std::uint64_t>(65539, 15, 0);
  sort_greater_case<std::int64_t>(65539, 16, 0);
  sort_greater_case<double>(33333, 17, 0);
  const std::size_t n = 300007;
  std::vector<std::int32_t> h(n);
  std::mt19937_64 g(18);
  for (auto &x : h) x = (std::int32_t)g();
  shp::distributed_vector<std::int32_t> dv(n);
  shp::copy(h.begin(), h.end(), dv.begin());
  shp::sort(shp::par_unseq, dv.begin() + 100, dv.end() - 200, std::greater<std::int32_t>());
  std::sort(h.begin() + 100, h.end() - 200, std::greater<std::int32_t>());
  EXPECT_TRUE(to_host(dv) == h);
  shp::sort(shp::par_unseq, dv, std::ranges::less{});
  std::sort(h.begin(), h.end());
  EXPECT_TRUE(to_host(dv) == h);
}

TEST(ShpExtra, SortSplitShapes) {
  // descending input (every boundary key lives in the last segment), a
  // sorted input sorted again (cached scratch reused across calls), a
  // sub-range (segments of unequal size) and all-equal keys
  const std::size_t n = 3 * (std::size_t(1) << 18) + 7;
  std::vector<std::uint32_t> h(n);
  for (std::size_t i = 0; i < n; i++) h[i] = static_cast<std::uint32_t>(n - i);
  shp::distributed_vector<std::uint32_t> dv(n);
  shp::copy(h.begin(), h.end(), dv.begin());
  shp::sort(shp::par_unseq, dv);
  std::sort(h.begin(), h.end());
  EXPECT_TRUE(to_host(dv) == h);
  shp::sort(shp::par_unseq, dv);
  EXPECT_TRUE(to_host(dv) == h);
  std::mt19937_64 g(9);
  for (auto &x : h) x = static_cast<std::uint32_t>(g() % 1000);
  shp::copy(h.begin(), h.end(), dv.begin());
  const std::size_t lo = 12345, hi = n - 54321;
  shp::sort(shp::par_unseq, std::ranges::subrange(dv.begin() + lo, dv.begin() + hi));
  std::sort(h.begin() + lo, h.begin() + hi);
  EXPECT_TRUE(to_host(dv) == h);
  std::fill(h.begin(), h.end(), 42u);
  shp::copy(h.begin(), h.end(), dv.begin());
  shp::sort(shp::par_unseq, dv);
  EXPECT_TRUE(to_host(dv) == h);
}

TEST(ShpExtra, SortSharedRankSegments) {
  // a distributed_span listing two segments of the SAME rank (every rank's
  // segment cut in two): shp::sort carves one scratch block per rank into
  // disjoint per-segment slices (sort.hpp) -- each piece's exchange buffer
  // must survive until its merge
  const std::size_t n = 4 * (std::size_t(1) << 16) + 321;
  std::vector<std::uint32_t> h(n);
  std::mt19937_64 g(21);
  for (auto &x : h) x = static_cast<std::uint32_t>(g());
  shp::distributed_vector<std::uint32_t> dv(n);
  shp::copy(h.begin(), h.end(), dv.begin());
  std::vector<shp::device_span<std::uint32_t>> parts;
  for (auto &&s : dv.segments()) {
    const std::size_t a = s.size() / 3;
    parts.emplace_back(s.data(), a, s.rank());
    parts.emplace_back(s.data() + a, s.size() - a, s.rank());
  }
  shp::distributed_span ds(parts);
  EXPECT_EQ(ds.size(), n);
  shp::sort(shp::par_unseq, ds);
  std::sort(h.begin(), h.end());
  EXPECT_TRUE(to_host(dv) == h);
}

// ---- the general comparator tier (dr/shp/merge_sort.hpp): stable, so the
// result must equal std::stable_sort's bit for bit
struct rec16 {
  std::uint32_t key, tag, pad0, pad1;
};
struct rec24 { // 2 items per thread, no LDS padding
  std::uint64_t key, a, b;
};
struct rec40 { // 1 item per thread
  std::int32_t key;
  std::uint32_t serial;
  std::uint8_t payload[32];
};
struct rec12 {
  std::int32_t key;
  float weight;
  std::uint32_t serial;
  __host__ __device__ bool operator<(const rec12 &o) const { return key < o.key; } // std::less<> on a non-ABI type
};
template <typename X> static bool same_bytes_v(const std::vector<X> &a, const std::vector<X> &b) {
  return a.size() == b.size() && std::memcmp(a.data(), b.data(), a.size() * sizeof(X)) == 0;
}
template <typename X, typename Comp> static void general_sort_case(std::vector<X> h, Comp comp, bool stable_api) {
  shp::distributed_vector<X> dv(h.size());
  shp::copy(h.begin(), h.end(), dv.begin());
  if (stable_api) shp::stable_sort(shp::par_unseq, dv, comp);
  else shp::sort(shp::par_unseq, dv, comp);
  std::stable_sort(h.begin(), h.end(), comp);
  EXPECT_TRUE(same_bytes_v(to_host(dv), h));
}

TEST(ShpExtra, SortGeneralComparator) {
  std::mt19937_64 g(31);
  // a struct ordered by one field, few distinct keys: stability decides the
  // order of every tie (tag = the original position)
  for (std::size_t n : {std::size_t(0), std::size_t(1), std::size_t(2), std::size_t(1000), std::size_t(300007)}) {
    std::vector<rec16> h(n);
    for (std::size_t i = 0; i < n; i++) h[i] = {static_cast<std::uint32_t>(g() % 97), static_cast<std::uint32_t>(i), 7u, 9u};
    general_sort_case(h, [](const rec16 &a, const rec16 &b) { return a.key < b.key; }, false);
  }
  // int keys ordered by abs(): -x and x are equivalent and keep their order
  {
    std::vector<std::int32_t> h(500001);
    for (auto &x : h) x = static_cast<std::int32_t>(g() % 2001) - 1000;
    general_sort_case(h, [](std::int32_t a, std::int32_t b) { return (a < 0 ? -a : a) < (b < 0 ? -b : b); }, false);
  }
  // a descending lambda over floats with -0.0 / +0.0 ties (not std::greater:
  // the general tier, stable)
  {
    std::vector<float> h(200003);
    for (auto &x : h) {
      const auto r = g() % 5;
      x = r == 0 ? 0.0f : r == 1 ? -0.0f : static_cast<float>(static_cast<std::int64_t>(g() % 2000) - 1000) * 0.5f;
    }
    general_sort_case(h, [](float a, float b) { return a > b; }, false);
    general_sort_case(h, std::less<>{}, true); // stable_sort of floats: the general tier too
  }
  // std::less<> on a non-ABI element type (operator<): sort(r) itself
  {
    std::vector<rec12> h(123457);
    for (std::size_t i = 0; i < h.size(); i++)
      h[i] = {static_cast<std::int32_t>(g() % 1000) - 500, 0.25f * static_cast<float>(i % 7), static_cast<std::uint32_t>(i)};
    shp::distributed_vector<rec12> dv(h.size());
    shp::copy(h.begin(), h.end(), dv.begin());
    shp::sort(shp::par_unseq, dv);
    std::stable_sort(h.begin(), h.end());
    EXPECT_TRUE(same_bytes_v(to_host(dv), h));
  }
  // wider elements: 24 B (2 items per thread) descending, 40 B (1 item per
  // thread) with few keys -- the unpadded LDS layouts of the tier
  {
    std::vector<rec24> h(100003);
    for (std::size_t i = 0; i < h.size(); i++) h[i] = {g() % 5003, i, ~i};
    general_sort_case(h, [](const rec24 &x, const rec24 &y) { return x.key > y.key; }, false);
  }
  {
    std::vector<rec40> h(50001);
    for (std::size_t i = 0; i < h.size(); i++) {
      h[i].key = static_cast<std::int32_t>(g() % 17) - 8;
      h[i].serial = static_cast<std::uint32_t>(i);
      for (int k = 0; k < 32; k++) h[i].payload[k] = static_cast<std::uint8_t>((i * 7 + k) & 0xFF);
    }
    general_sort_case(h, [](const rec40 &x, const rec40 &y) { return x.key < y.key; }, true);
  }
  // 64-bit keys by their low 20 bits, 2^24 elements (many merge passes)
  {
    std::vector<std::uint64_t> h(std::size_t(1) << 24);
    for (auto &x : h) x = g();
    general_sort_case(h, [](std::uint64_t a, std::uint64_t b) { return (a & 0xFFFFF) < (b & 0xFFFFF); }, true);
  }
  // a sub-range by iterators under a comparator
  {
    const std::size_t n = 250003;
    std::vector<std::uint32_t> h(n);
    for (auto &x : h) x = static_cast<std::uint32_t>(g());
    shp::distributed_vector<std::uint32_t> dv(n);
    shp::copy(h.begin(), h.end(), dv.begin());
    auto by_mod = [](std::uint32_t a, std::uint32_t b) { return a % 1000 < b % 1000; };
    shp::stable_sort(shp::par_unseq, dv.begin() + 17, dv.end() - 1001, by_mod);
    std::stable_sort(h.begin() + 17, h.end() - 1001, by_mod);
    EXPECT_TRUE(same_bytes_v(to_host(dv), h));
  }
}

TEST(ShpExtra, GemvColumnsChanged) {
  // the column-range cache (advisor round 4): after a gemv, rewrite every
  // tile's column indices on the device (mirror c -> n-1-c, so the windows
  // move), call columns_changed(), gemv again: the result must follow the
  // NEW columns (a stale window would read outside the copied part of b)
  const std::size_t m = 3001, n = 3001;
  shp::sparse_matrix<float, std::int32_t> a({m, n}, shp::csr_kind::banded, 10, 5);
  shp::distributed_vector<float> b(n), c(m, 0.0f);
  std::vector<float> hb(n);
  for (std::size_t i = 0; i < n; i++) hb[i] = (float)((i * 31) % 97) / 97.0f;
  shp::copy(hb.begin(), hb.end(), b.begin());
  shp::gemv(c, a, b);
  double worst = 0;
  std::vector<float> want(m, 0.0f);
  std::vector<std::vector<int>> rps, cis;
  std::vector<std::vector<float>> vas;
  for (auto &t : a.segments()) {
    const std::size_t rows = t.shape()[0], nnz = t.size();
    std::vector<int> rp(rows + 1), ci(nnz);
    std::vector<float> va(nnz);
    drhip_memcpy_d2h((int)t.rank(), rp.data(), t.rowptr_data(), rp.size() * 4);
    drhip_memcpy_d2h((int)t.rank(), ci.data(), t.colind_data(), ci.size() * 4);
    drhip_memcpy_d2h((int)t.rank(), va.data(), t.values_data(), va.size() * 4);
    shp::sync(t.rank());
    for (auto &x : ci) x = (int)(n - 1) - x; // mirrored columns
    drhip_memcpy_h2d((int)t.rank(), t.colind_data(), ci.data(), ci.size() * 4);
    shp::sync(t.rank());
    rps.push_back(rp);
    cis.push_back(ci);
    vas.push_back(va);
  }
  a.columns_changed();
  shp::fill(c, 0.0f);
  shp::gemv(c, a, b);
  auto got = to_host(c);
  auto segs = a.segments();
  for (std::size_t k = 0; k < segs.size(); k++) {
    const std::size_t row0 = segs[k].origin()[0];
    for (std::size_t r = 0; r + 1 < rps[k].size(); r++) {
      double acc = 0;
      for (int j = rps[k][r]; j < rps[k][r + 1]; j++) acc += (double)vas[k][j] * hb[cis[k][j]];
      worst = std::max(worst, std::fabs(got[row0 + r] - acc) / std::max(std::fabs(acc), 1e-30));
    }
  }
  EXPECT_TRUE(worst <= 1e-5);
}

TEST(ShpExtra, Gemv) {
  // intended c += A * b on a device-generated banded and random matrix,
  // checked against a host CSR SpMV in fp64 (rtol 1e-5 per row)
  for (auto kind : {shp::csr_kind::banded, shp::csr_kind::random}) {
    const std::size_t m = 5003, n = 4099;
    shp::sparse_matrix<float, std::int32_t> a({m, n}, kind, 10, 7);
    shp::distributed_vector<float> b(n), c(m, 1.0f);
    std::vector<float> hb(n);
    for (std::size_t i = 0; i < n; i++) hb[i] = (float)((i * 7919) % 1000) / 1000.0f;
    shp::copy(hb.begin(), hb.end(), b.begin());
    shp::gemv(c, a, b);
    auto got = to_host(c);
    // host CSR from the device tiles
    double worst = 0;
    for (auto &t : a.segments()) {
      const std::size_t rows = t.shape()[0], nnz = t.size(), row0 = t.origin()[0];
      std::vector<int> rp(rows + 1), ci(nnz);
      std::vector<float> va(nnz);
      drhip_memcpy_d2h((int)t.rank(), rp.data(), t.rowptr_data(), rp.size() * 4);
      if (nnz) {
        drhip_memcpy_d2h((int)t.rank(), ci.data(), t.colind_data(), ci.size() * 4);
        drhip_memcpy_d2h((int)t.rank(), va.data(), t.values_data(), va.size() * 4);
      }
      for (std::size_t r = 0; r < rows; r++) {
        double s = 1.0;
        for (int k = rp[r]; k < rp[r + 1]; k++) s += (double)va[k] * hb[ci[k]];
        worst = std::max(worst, std::fabs(got[row0 + r] - s) / std::max(std::fabs(s), 1e-30));
      }
    }
    EXPECT_TRUE(worst <= 1e-5);
    EXPECT_TRUE(a.size() > 0);
    // gemv ships each tile only its column window of b: the band around the
    // tile's rows (offsets -4..+5, clipped) for banded, [min, max] of the
    // random columns otherwise
    auto segs = a.segments();
    for (std::size_t k = 0; k < segs.size(); k++) {
      const std::size_t rows = segs[k].shape()[0], row0 = segs[k].origin()[0];
      if (!rows || !segs[k].size()) continue; // rows past n + 4 hold no band entries
      const auto [lo, hi] = a.column_range(k);
      if (kind == shp::csr_kind::banded) {
        EXPECT_TRUE(lo == (row0 >= 4 ? row0 - 4 : 0));
        EXPECT_TRUE(hi == std::min(n, row0 + rows + 5));
      } else {
        EXPECT_TRUE(lo < hi && hi <= n);
      }
    }
  }
}

// host reference c += A b from the matrix's own entries
template <typename T, typename I, typename BV>
static std::vector<double> host_gemv(const shp::sparse_matrix<T, I> &a, const std::vector<BV> &b, std::vector<double> c) {
  for (auto &&[idx, v] : a) c[idx[0]] += (double)v * (double)b[idx[1]];
  return c;
}

TEST(ShpSparse, DensityConstructor) {
  // sparse_test.cpp:13: sparse_matrix<float> x({100, 100}, 0.01)
  shp::sparse_matrix<float> x({100, 100}, 0.01);
  // row tiles: floor(0.01 * 100 * 100) in total; a 2-D default grid
  // (factor(nprocs())) generates each tile as its own tm x tn matrix
  std::size_t want = 0;
  for (auto &t : x.segments()) want += (std::size_t)(0.01 * (double)t.shape()[0] * (double)t.shape()[1]);
  if (x.grid_shape()[1] == 1) want = 100;
  EXPECT_EQ(x.size(), want);
  EXPECT_EQ(x.shape()[0], (std::size_t)100);
  std::size_t count = 0, last_i = 0, last_j = 0;
  bool ordered = true, inside = true;
  for (auto &&[idx, v] : x) {
    auto &&[i, j] = idx;
    inside &= i < 100 && j < 100 && v >= 0.0f && v < 1.0f;
    if (count) ordered &= (i > last_i) || (i == last_i && j > last_j);
    last_i = i, last_j = j;
    count++;
  }
  EXPECT_EQ(count, want);
  if (x.grid_shape()[1] == 1) EXPECT_TRUE(ordered); // tile order is row-major only for row tiles
  EXPECT_TRUE(inside);
  // same matrix for any row-tile count: compare with a one-tile partition
  shp::sparse_matrix<float> y({100, 100}, 0.01, shp::block_cyclic({shp::tile::div, shp::tile::div}, {1, 1}));
  std::vector<shp::matrix_entry<float>> ex(x.begin(), x.end()), ey(y.begin(), y.end());
  if (x.grid_shape()[1] == 1) EXPECT_TRUE(ex == ey); // the default grid is factor(nprocs()): 2 x 2 at 4
  EXPECT_EQ(ey.size(), (std::size_t)100);
}

TEST(ShpSparse, GemvExample) {
  // examples/shp/gemv_example.cpp:19-39 (int values, size_t indices)
  shp::distributed_vector<int, shp::device_allocator<int>> b(100);
  shp::for_each(shp::par_unseq, shp::enumerate(b), [](auto &&tuple) {
    auto &&[idx, value] = tuple;
    value = 1;
  });
  shp::distributed_vector<int, shp::device_allocator<int>> c(100);
  shp::for_each(shp::par_unseq, c, [](auto &&v) { v = 0; });
  shp::sparse_matrix<int> a({100, 100}, 0.01,
                            shp::block_cyclic({shp::tile::div, shp::tile::div}, {shp::nprocs(), 1}));
  EXPECT_EQ(a.grid_shape()[0], shp::nprocs());
  EXPECT_EQ(a.grid_shape()[1], (std::size_t)1);
  shp::gemv(c, a, b);
  auto ref = host_gemv(a, std::vector<int>(100, 1), std::vector<double>(100, 0.0));
  std::vector<int> got(100);
  shp::copy(c.begin(), c.end(), got.begin());
  bool ok = true;
  for (std::size_t i = 0; i < 100; i++) ok &= got[i] == (int)ref[i];
  EXPECT_TRUE(ok);
  shp::print_range(b, "b");
  shp::print_matrix(a, "a");
  shp::print_range(c, "c");
}

TEST(ShpSparse, GemvDoubleInt64AndGeneric) {
  const std::size_t m = 3001, n = 2777;
  const shp::block_cyclic rows_part({shp::tile::div, shp::tile::div}, {shp::nprocs(), 1});
  shp::sparse_matrix<double, std::int64_t> a({m, n}, 0.003, rows_part, 5);
  std::vector<double> hb(n);
  for (std::size_t i = 0; i < n; i++) hb[i] = 0.25 + (double)(i % 17);
  shp::distributed_vector<double> b(n), c(m, 2.0);
  shp::copy(hb.begin(), hb.end(), b.begin());
  shp::gemv(c, a, b);
  auto ref = host_gemv(a, hb, std::vector<double>(m, 2.0));
  auto got = to_host(c);
  double worst = 0;
  for (std::size_t i = 0; i < m; i++) worst = std::max(worst, std::fabs(got[i] - ref[i]) / std::fabs(ref[i]));
  EXPECT_TRUE(worst <= 1e-12);
  // float matrix times float vector into a double result: template kernel
  shp::sparse_matrix<float, std::int32_t> af({m, n}, 0.002, rows_part, 9);
  shp::distributed_vector<float> bf(n, 1.5f);
  shp::distributed_vector<double> cd(m, 0.0);
  shp::gemv(cd, af, bf);
  auto refd = host_gemv(af, std::vector<float>(n, 1.5f), std::vector<double>(m, 0.0));
  auto gotd = to_host(cd);
  worst = 0;
  for (std::size_t i = 0; i < m; i++) worst = std::max(worst, std::fabs(gotd[i] - refd[i]) / std::max(std::fabs(refd[i]), 1e-30));
  EXPECT_TRUE(worst <= 1e-6);
}

TEST(ShpSparse, BlockCyclicTiles) {
  // a 2 x 2 tile grid: tiles hold local column indices, segments() carry
  // their origin, entries come back with global indices; gemv refuses it
  shp::sparse_matrix<double> a({50, 60}, 0.1, shp::block_cyclic({shp::tile::div, shp::tile::div}, {2, 2}), 3);
  EXPECT_EQ(a.grid_shape()[0], (std::size_t)2);
  EXPECT_EQ(a.grid_shape()[1], (std::size_t)2);
  EXPECT_EQ(a.tile_shape()[0], (std::size_t)25);
  EXPECT_EQ(a.tile_shape()[1], (std::size_t)30);
  std::size_t total = 0;
  for (auto &t : a.segments()) total += t.size();
  EXPECT_EQ(total, a.size());
  auto t11 = a.tile({1, 1});
  EXPECT_EQ(t11.shape()[0], (std::size_t)25);
  bool inside = true;
  for (auto &&[idx, v] : a) inside &= idx[0] < 50 && idx[1] < 60;
  EXPECT_TRUE(inside);
  shp::distributed_vector<double> b(60, 1.0), c(50, 0.0);
  bool threw = false;
  try {
    shp::gemv(c, a, b);
  } catch (const std::runtime_error &) {
    threw = true;
  }
  EXPECT_TRUE(threw);
}

TEST(ShpSparse, MatrixMarket) {
  // symmetric real + general pattern coordinate files, 1-indexed
  const std::string p1 = "/tmp/drhip_mm_sym_" + std::to_string(::getpid()) + ".mtx";
  {
    FILE *f = std::fopen(p1.c_str(), "w");
    std::fprintf(f, "%%%%MatrixMarket matrix coordinate real symmetric\n%% comment\n4 4 5\n");
    std::fprintf(f, "1 1 2.0\n2 1 -1.5\n3 3 4.0\n4 2 0.5\n4 4 1.0\n");
    std::fclose(f);
  }
  auto a = shp::mmread<double, std::int32_t>(p1);
  std::remove(p1.c_str());
  EXPECT_EQ(a.size(), (std::size_t)7); // 5 entries + 2 mirrored off-diagonals
  std::vector<shp::matrix_entry<double>> e(a.begin(), a.end());
  std::vector<std::tuple<std::size_t, std::size_t, double>> want = {
      {0, 0, 2.0}, {0, 1, -1.5}, {1, 0, -1.5}, {1, 3, 0.5}, {2, 2, 4.0}, {3, 1, 0.5}, {3, 3, 1.0}};
  bool ok = e.size() == want.size();
  for (std::size_t k = 0; ok && k < e.size(); k++)
    ok = e[k].index()[0] == std::get<0>(want[k]) && e[k].index()[1] == std::get<1>(want[k]) &&
         e[k].value() == std::get<2>(want[k]);
  EXPECT_TRUE(ok);
  shp::distributed_vector<double> b(4, 1.0), c(4, 0.0);
  shp::gemv(c, a, b);
  auto got = to_host(c);
  EXPECT_TRUE(got == (std::vector<double>{0.5, -1.0, 4.0, 1.5}));
  const std::string p2 = "/tmp/drhip_mm_pat_" + std::to_string(::getpid()) + ".mtx";
  {
    FILE *f = std::fopen(p2.c_str(), "w");
    std::fprintf(f, "%%%%MatrixMarket matrix coordinate pattern general\n3 5 3\n1 5\n3 1\n1 2\n");
    std::fclose(f);
  }
  auto pm = shp::mmread<float>(p2);
  std::remove(p2.c_str());
  EXPECT_EQ(pm.size(), (std::size_t)3);
  EXPECT_EQ(pm.shape()[1], (std::size_t)5);
}


TEST(ShpExtra, ForEachStaged) {
  // the staged (register-copy) for_each path: odd lengths (in-place tail),
  // 1/2/4/8-byte types, misaligned drop() pieces (in-place path), and a
  // read-only functor (no write-back, every element seen exactly once)
  {
    const std::size_t n = 1000003;
    shp::distributed_vector<float> v(n, 1.5f);
    shp::for_each(shp::par_unseq, v, [](float &x) { x = x * 2.0f + 1.0f; });
    auto h = to_host(v);
    EXPECT_TRUE(std::all_of(h.begin(), h.end(), [](float x) { return x == 4.0f; }));
  }
  {
    const std::size_t n = 77;
    shp::distributed_vector<double> v(n);
    shp::iota(v, 1.0);
    shp::for_each(shp::par_unseq, v, [](auto &&x) { x = -x; });
    auto h = to_host(v);
    bool ok = true;
    for (std::size_t i = 0; i < n; i++) ok &= h[i] == -double(i + 1);
    EXPECT_TRUE(ok);
  }
  {
    const std::size_t n = 4099;
    shp::distributed_vector<std::uint8_t> v(n, 7);
    shp::for_each(shp::par_unseq, v, [](std::uint8_t &x) { x = static_cast<std::uint8_t>(x * 3); });
    shp::distributed_vector<std::int16_t> w(n, -2);
    shp::for_each(shp::par_unseq, w, [](auto &&x) { x += 5; });
    auto hv = to_host(v);
    auto hw = to_host(w);
    EXPECT_TRUE(std::all_of(hv.begin(), hv.end(), [](std::uint8_t x) { return x == 21; }));
    EXPECT_TRUE(std::all_of(hw.begin(), hw.end(), [](std::int16_t x) { return x == 3; }));
  }
  {
    const std::size_t n = 10007;
    shp::distributed_vector<std::int64_t> v(n);
    shp::iota(v, std::int64_t(0));
    auto dropped = v | rng::views::drop(3);
    shp::for_each(shp::par_unseq, dropped, [](auto &&x) { x += 1000000; });
    auto h = to_host(v);
    bool ok = true;
    for (std::size_t i = 0; i < n; i++) ok &= h[i] == std::int64_t(i) + (i >= 3 ? 1000000 : 0);
    EXPECT_TRUE(ok);
  }
  {
    // read-only: count elements with a device atomic; values stay intact
    const std::size_t n = (1 << 20) + 13;
    shp::distributed_vector<int> v(n);
    shp::iota(v, 0);
    void *cnt = nullptr;
    shp::detail::check(drhip_malloc(0, sizeof(unsigned long long), &cnt), "malloc");
    const unsigned long long zero = 0;
    shp::detail::check(drhip_memcpy_h2d(0, cnt, &zero, sizeof(zero)), "h2d");
    auto *c = static_cast<unsigned long long *>(cnt);
    shp::for_each(shp::par_unseq, v, [c](const int &x) { atomicAdd(c, (unsigned long long)(x & 1) + 1ull); });
    unsigned long long got = 0;
    shp::detail::check(drhip_memcpy_d2h(0, &got, cnt, sizeof(got)), "d2h");
    (void)drhip_free(0, cnt);
    EXPECT_EQ(got, (unsigned long long)(n + n / 2));
    auto h = to_host(v);
    bool ok = true;
    for (std::size_t i = 0; i < n; i++) ok &= h[i] == (int)i;
    EXPECT_TRUE(ok);
  }
}

TEST(ShpExtra, ReduceGeneric) {
  // user-lambda operators run the template reduce kernels: the staged
  // 16-byte path on aligned spans (odd lengths, 1/2/4/8-byte types), the
  // element path on misaligned drop() pieces and on zip | transform
  {
    const std::size_t n = 1000003;
    shp::distributed_vector<int> v(n);
    shp::iota(v, 0);
    const long long got = shp::reduce(shp::par_unseq, v, 5, [](int a, int b) { return a ^ b; });
    int want = 5;
    for (std::size_t i = 0; i < n; i++) want ^= (int)i;
    EXPECT_EQ(got, (long long)want);
  }
  {
    const std::size_t n = 4099;
    std::vector<std::uint8_t> h(n);
    for (std::size_t i = 0; i < n; i++) h[i] = static_cast<std::uint8_t>((i * 37) % 251);
    shp::distributed_vector<std::uint8_t> v(n);
    shp::copy(h.begin(), h.end(), v.begin());
    const int got = shp::reduce(shp::par_unseq, v, std::uint8_t(0),
                                [](std::uint8_t a, std::uint8_t b) { return a < b ? b : a; });
    EXPECT_EQ(got, (int)*std::max_element(h.begin(), h.end()));
    shp::distributed_vector<std::int16_t> w(n, 3);
    EXPECT_EQ((int)shp::reduce(shp::par_unseq, w, std::int16_t(1), [](std::int16_t a, std::int16_t b) {
                return static_cast<std::int16_t>(a + b);
              }),
              (int)static_cast<std::int16_t>(1 + 3 * n));
  }
  {
    const std::size_t n = 10007;
    shp::distributed_vector<std::int64_t> v(n);
    shp::iota(v, std::int64_t(-50));
    auto dropped = v | rng::views::drop(3);
    EXPECT_EQ(shp::reduce(shp::par_unseq, dropped, std::int64_t(1000), [](std::int64_t a, std::int64_t b) {
                return a < b ? a : b;
              }),
              (std::int64_t)-47);
    EXPECT_EQ(shp::reduce(shp::par_unseq, v, std::int64_t(0), [](std::int64_t a, std::int64_t b) { return a + b; }),
              (std::int64_t)((n * (n - 1)) / 2) - 50 * (std::int64_t)n);
  }
  {
    const std::size_t n = 300001;
    shp::distributed_vector<double> x(n, 0.5), y(n, 4.0);
    auto z = shp::views::zip(x, y) | lib::views::transform([](auto &&e) {
               auto &&[a, b] = e;
               return a * b;
             });
    EXPECT_NEAR_REL(shp::reduce(shp::par_unseq, z, 1.0, std::plus()), 1.0 + 2.0 * n, 1e-12);
  }
}

TEST(ShpExtra, ScanGenericManyTiles) {
  // template scan with hundreds of tiles per segment: a max-scan matches
  // std::inclusive_scan (the non-commutative cases are ScanNonCommutative)
  const std::size_t n = 5000011;
  std::vector<int> h(n);
  std::mt19937 g(7);
  for (auto &x : h) x = static_cast<int>(g() % 1000000) - 500000;
  shp::distributed_vector<int> v(n), o(n);
  shp::copy(h.begin(), h.end(), v.begin());
  shp::inclusive_scan(shp::par_unseq, v, o, [](int a, int b) { return a < b ? b : a; });
  std::vector<int> want(n);
  std::inclusive_scan(h.begin(), h.end(), want.begin(), [](int a, int b) { return a < b ? b : a; });
  EXPECT_TRUE(to_host(o) == want);
}

// ------------------------- non-commutative operators (template look-back scan)
// Affine maps x -> a*x + b (mod 2^32) composed left to right: associative,
// not commutative.  8 bytes: the 16-B vector path, value + status granules.
struct affine {
  std::uint32_t a, b;
};
struct affine_then {
  __host__ __device__ affine operator()(const affine &l, const affine &r) const { return {r.a * l.a, r.a * l.b + r.b}; }
};
// 12 bytes (not a vector type): accessor path, still one 16-B granule.
struct affine3 {
  std::uint32_t a, b, n;
};
struct affine3_then {
  __host__ __device__ affine3 operator()(const affine3 &l, const affine3 &r) const {
    return {r.a * l.a, r.a * l.b + r.b, l.n + r.n};
  }
};
// 2x2 matrices mod 2^32, 16 bytes: vector path with separate status words.
struct mat2 {
  std::uint32_t m[4];
};
struct mat2_mul {
  __host__ __device__ mat2 operator()(const mat2 &x, const mat2 &y) const {
    return {{x.m[0] * y.m[0] + x.m[1] * y.m[2], x.m[0] * y.m[1] + x.m[1] * y.m[3], x.m[2] * y.m[0] + x.m[3] * y.m[2],
             x.m[2] * y.m[1] + x.m[3] * y.m[3]}};
  }
};
template <typename X> static bool same_bytes(const std::vector<X> &a, const std::vector<X> &b) {
  return a.size() == b.size() && std::memcmp(a.data(), b.data(), a.size() * sizeof(X)) == 0;
}

// The reference's 3-phase algorithm (inclusive_scan.hpp:22-148) on the host:
// local scans of the zipped pieces (init on piece 0), the running fold of
// the piece totals, then x = op(x, S_{k-1}) on pieces k > 0.
template <typename X, typename Op>
static std::vector<X> ref_shp_scan(const std::vector<X> &x, std::size_t out_size, std::size_t P, Op op,
                                   const X *init) {
  const std::size_t n = x.size(), si = (n + P - 1) / P, so = (out_size + P - 1) / P;
  std::vector<std::size_t> b{0, n};
  for (std::size_t k = 1; k < P; k++) {
    if (k * si < n) b.push_back(k * si);
    if (k * so < n) b.push_back(k * so);
  }
  std::sort(b.begin(), b.end());
  b.erase(std::unique(b.begin(), b.end()), b.end());
  std::vector<X> out(n);
  std::vector<X> part;
  for (std::size_t k = 0; k + 1 < b.size(); k++) {
    X run = x[b[k]];
    if (k == 0 && init) run = op(*init, run);
    out[b[k]] = run;
    for (std::size_t i = b[k] + 1; i < b[k + 1]; i++) out[i] = run = op(run, x[i]);
    part.push_back(run);
  }
  for (std::size_t k = 1; k < part.size(); k++) part[k] = op(part[k - 1], part[k]);
  for (std::size_t k = 1; k + 1 < b.size(); k++)
    for (std::size_t i = b[k]; i < b[k + 1]; i++) out[i] = op(out[i], part[k - 1]);
  return out;
}

// Diagnosis (round 6): a hash of a range's bytes computed by a KERNEL, so a
// step check can tell whether the memory itself changed (the kernel sees it
// too) or only a device-to-host copy returned wrong bytes.  Word i of the
// range (global index) contributes w_i * (2 i + 1) mod 2^64: order-free.
__global__ void word_hash_kernel(const std::uint32_t *p, std::size_t nw, std::size_t base,
                                 unsigned long long *out) {
  unsigned long long acc = 0;
  for (std::size_t i = blockIdx.x * (std::size_t)blockDim.x + threadIdx.x; i < nw; i += (std::size_t)gridDim.x * blockDim.x)
    acc += (unsigned long long)p[i] * (2ull * (base + i) + 1ull);
  atomicAdd(out, acc);
}
static unsigned long long host_word_hash(const void *p, std::size_t bytes) {
  const auto *w = static_cast<const std::uint32_t *>(p);
  unsigned long long acc = 0;
  for (std::size_t i = 0; i < bytes / 4; i++) acc += (unsigned long long)w[i] * (2ull * i + 1ull);
  return acc;
}
template <typename X> static unsigned long long device_word_hash(const shp::distributed_vector<X> &dv) {
  static_assert(sizeof(X) % 4 == 0);
  unsigned long long total = 0;
  std::size_t base = 0;
  for (auto &&seg : dv.segments()) {
    const std::size_t rank = seg.rank();
    shp::sync(rank);
    // one word per device, allocated once (no hipFree: it would synchronise
    // the device between the steps being checked)
    static unsigned long long *words[64] = {};
    const int dev = shp::devices()[rank];
    (void)hipSetDevice(dev);
    unsigned long long *&d = words[dev & 63];
    if (!d) (void)hipMalloc(&d, 8);
    (void)hipMemset(d, 0, 8);
    const std::size_t nw = seg.size() * sizeof(X) / 4;
    hipLaunchKernelGGL(word_hash_kernel, dim3(1024), dim3(256), 0, 0, reinterpret_cast<const std::uint32_t *>(seg.data()),
                       nw, base, d);
    unsigned long long h = 0;
    (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
    total += h;
    base += nw;
  }
  return total;
}

template <typename X, typename Op, typename Gen> static void noncommutative_case(std::size_t n, Gen gen, Op op) {
  std::vector<X> h(n);
  std::mt19937 g(static_cast<unsigned>(n));
  for (auto &x : h) x = gen(g);
  const std::size_t P = shp::nprocs();
  shp::distributed_vector<X> v(n), o(n), o2(2 * n);
  shp::copy(h.begin(), h.end(), v.begin());
  const bool copied = same_bytes(to_host(v), h);
  EXPECT_TRUE(copied);
  if (!copied) std::printf("  (noncommutative_case: %zu-byte elements, n = %zu: the input differs right after the copy)\n", sizeof(X), n);
  // diagnosis (round 5 pool stress): allocation, fill and copy only
  if (std::getenv("SHP_TESTS_NO_SCAN")) return;
  // aligned pieces, no init
  // diagnosis (round 5 pool stress, SHP_TESTS_STEP_CHECK=1): the input after
  // every step, naming the first step after which it changed
  const bool step_check = std::getenv("SHP_TESTS_STEP_CHECK") != nullptr;
  const unsigned long long hh = step_check ? host_word_hash(h.data(), n * sizeof(X)) : 0;
  auto step = [&](const char *what) {
    if (!step_check) return;
    // the kernel's view first, then the copy's: which one sees a change
    const bool kernel_ok = device_word_hash(v) == hh;
    const bool copy_ok = same_bytes(to_host(v), h);
    if (!kernel_ok || !copy_ok)
      std::printf("  (noncommutative_case: %zu-byte elements, n = %zu: input changed after %s -- kernel view %s, "
                  "copy view %s)\n",
                  sizeof(X), n, what, kernel_ok ? "intact" : "CHANGED", copy_ok ? "intact" : "CHANGED");
  };
  step("the copy in");
  shp::inclusive_scan(shp::par_unseq, v, o, op);
  step("the inclusive scan into o");
  EXPECT_TRUE(same_bytes(to_host(o), ref_shp_scan(h, n, P, op, (const X *)nullptr)));
  step("reading o back");
  // misaligned output (algorithms.cpp:88-98 layout) with init
  const X init = gen(g);
  shp::inclusive_scan(shp::par_unseq, v, o2, op, init);
  step("the inclusive scan with init into o2");
  auto got = to_host(o2);
  got.resize(n);
  EXPECT_TRUE(same_bytes(got, ref_shp_scan(h, 2 * n, P, op, &init)));
  // std::exclusive_scan semantics (the carry is the fold of everything before)
  shp::exclusive_scan(shp::par_unseq, v, o, init, op);
  step("the exclusive scan into o");
  std::vector<X> want(n);
  std::exclusive_scan(h.begin(), h.end(), want.begin(), init, op);
  EXPECT_TRUE(same_bytes(to_host(o), want));
  if (!g_cur_failed) return;
  // failure context: element size, n, whether the input still holds h, and
  // where the last (exclusive) result first differs
  std::size_t first = n;
  const auto got_o = to_host(o);
  for (std::size_t i = 0; i < n && first == n; i++)
    if (std::memcmp(&got_o[i], &want[i], sizeof(X)) != 0) first = i;
  const auto hv = to_host(v);
  std::size_t c0 = n, c1 = 0;
  for (std::size_t i = 0; i < n; i++)
    if (std::memcmp(&hv[i], &h[i], sizeof(X)) != 0) {
      c0 = std::min(c0, i);
      c1 = i;
    }
  std::printf("  (noncommutative_case: %zu-byte elements, n = %zu, %zu segments; input intact: %d; exclusive "
              "result first differs at %zu)\n",
              sizeof(X), n, P, c0 == n ? 1 : 0, first);
  if (c0 < n) {
    unsigned w[4] = {0, 0, 0, 0}, e[4] = {0, 0, 0, 0};
    std::memcpy(w, &hv[c0], std::min<std::size_t>(sizeof(X), 16));
    std::memcpy(e, &h[c0], std::min<std::size_t>(sizeof(X), 16));
    std::printf("  input corrupted in [%zu, %zu]; at %zu: %08x %08x (want %08x %08x)\n", c0, c1, c0, w[0], w[1], e[0], e[1]);
  }
  auto &pool = shp::detail::lb_status_buffers();
  std::printf("  v %p o %p o2 %p; lb status buffer %p cap %zu\n", (void *)v.segments()[0].data(),
              (void *)o.segments()[0].data(), (void *)o2.segments()[0].data(),
              pool.per_rank.empty() ? nullptr : pool.per_rank[0].p, pool.per_rank.empty() ? 0 : pool.per_rank[0].cap);
}

TEST(ShpExtra, ScanNonCommutative) {
  auto gaff = [](std::mt19937 &g) { return affine{static_cast<std::uint32_t>(g()) | 1u, static_cast<std::uint32_t>(g())}; };
  auto gaff3 = [](std::mt19937 &g) {
    return affine3{static_cast<std::uint32_t>(g()) | 1u, static_cast<std::uint32_t>(g()), 1u};
  };
  auto gmat = [](std::mt19937 &g) {
    return mat2{{static_cast<std::uint32_t>(g()), static_cast<std::uint32_t>(g()), static_cast<std::uint32_t>(g()),
                 static_cast<std::uint32_t>(g())}};
  };
  {
    // keep-the-right-operand: the reference's op(x, S_{k-1}) makes every
    // element of pieces k > 0 equal the carry (inclusive_scan.hpp:132-134)
    const std::size_t n = 5000011;
    std::vector<int> h(n);
    std::mt19937 g(7);
    for (auto &x : h) x = static_cast<int>(g() % 1000000) - 500000;
    shp::distributed_vector<int> v(n), o(n);
    shp::copy(h.begin(), h.end(), v.begin());
    auto keep_right = [](int, int b) { return b; };
    shp::inclusive_scan(shp::par_unseq, v, o, keep_right);
    EXPECT_TRUE(to_host(o) == ref_shp_scan(h, n, shp::nprocs(), keep_right, (const int *)nullptr));
  }
  for (std::size_t n : {std::size_t(1), std::size_t(1000), std::size_t(300007), std::size_t(2000003)}) {
    noncommutative_case<affine>(n, gaff, affine_then{});
    noncommutative_case<affine3>(n, gaff3, affine3_then{});
    noncommutative_case<mat2>(n, gmat, mat2_mul{});
  }
}

TEST(ShpExtra, ScanStatusLayoutSwitch) {
  // Under DR_SHP_LB_EPOCH (a build knob, off by default) the template scan
  // keeps its status words between calls (epoch tags, dr/shp/runtime.hpp
  // lb_status_pool); without it this is a plain small / large / small
  // element-size alternation.  A small-T scan publishes {value,
  // tag} words exactly where a following large-T (mat2) scan reads its tag
  // words, so here the int scan's tile values are set to the tag the mat2
  // scan would carry if the buffer were not cleared on the layout switch
  // (exact on one segment, where the epochs are known): a mat2 tile then
  // reads a predecessor as INCL before it is published.  Every result is
  // checked whatever the segment count.
  const std::size_t P = shp::nprocs();
  const std::size_t ni = 100000, nm = 40000; // >= 2 tiles each (32 K ints, 5120 mat2 per tile)
  std::mt19937 g(11);
  auto keep_right = [](int, int b) { return b; };
  for (int rep = 0; rep < 6; rep++) {
    auto &pool = shp::detail::lb_status_buffers();
    const unsigned e0 = pool.per_rank.empty() ? 0u : pool.per_rank[0].epoch;
    const unsigned ea = e0 == 0 ? 1u : e0 + 1u; // the int scan's epoch without a layout clear
    const int c = static_cast<int>(((ea + 1u) << 2) | 2u); // ... and the mat2 scan's INCL tag
    shp::distributed_vector<int> vi(ni, P == 1 ? c : rep + 1), oi(ni);
    shp::inclusive_scan(shp::par_unseq, vi, oi, keep_right);
    EXPECT_TRUE(to_host(oi) == std::vector<int>(ni, P == 1 ? c : rep + 1));
    std::vector<mat2> h(nm);
    for (auto &x : h) x = mat2{{static_cast<std::uint32_t>(g()), static_cast<std::uint32_t>(g()),
                                static_cast<std::uint32_t>(g()), static_cast<std::uint32_t>(g())}};
    shp::distributed_vector<mat2> vm(nm), om(nm);
    shp::copy(h.begin(), h.end(), vm.begin());
    shp::inclusive_scan(shp::par_unseq, vm, om, mat2_mul{});
    EXPECT_TRUE(same_bytes(to_host(om), ref_shp_scan(h, nm, P, mat2_mul{}, (const mat2 *)nullptr)));
    // large -> small: the next int scan runs over a buffer the mat2 scan's
    // value arrays wrote into
    shp::distributed_vector<int> wi(ni), wo(ni);
    std::vector<int> hw(ni);
    for (auto &x : hw) x = static_cast<int>(g() % 2000) - 1000;
    shp::copy(hw.begin(), hw.end(), wi.begin());
    shp::inclusive_scan(shp::par_unseq, wi, wo, [](int a, int b) { return a + b; });
    std::vector<int> want(ni);
    std::inclusive_scan(hw.begin(), hw.end(), want.begin());
    EXPECT_TRUE(to_host(wo) == want);
  }
}

TEST(ShpExtra, ScanTransformView) {
  // a transform view as the input (accessor path, V = 1), int64 output
  const std::size_t n = 1000003;
  std::vector<int> h(n);
  std::mt19937 g(3);
  for (auto &x : h) x = static_cast<int>(g() % 2001) - 1000;
  shp::distributed_vector<int> v(n);
  shp::distributed_vector<long long> o(n);
  shp::copy(h.begin(), h.end(), v.begin());
  auto sq = lib::views::transform(v, [](int x) { return static_cast<long long>(x) * x; });
  shp::inclusive_scan(shp::par_unseq, sq, o, [](long long a, long long b) { return a + b; }, 5LL);
  std::vector<long long> want(n);
  long long run = 5;
  for (std::size_t i = 0; i < n; i++) want[i] = run += static_cast<long long>(h[i]) * h[i];
  EXPECT_TRUE(to_host(o) == want);
}

// ------------------------------------------- dense_matrix
TEST(ShpDense, MatrixExample) {
  // examples/shp/matrix_example.cpp: 10 x 10 block_cyclic, three host
  // writes, for_each adds 12 to every entry on the tiles' devices, then a
  // host walk in global row-major order
  auto partition = shp::block_cyclic();
  shp::dense_matrix<float> x({10, 10}, partition);
  x[{2, 3}] = 12;
  x[{5, 7}] = 42;
  x[{8, 9}] = 37;
  shp::for_each(shp::par_unseq, x, [](auto &&entry) {
    auto &&[idx, v] = entry;
    v = v + 12;
  });
  std::size_t k = 0;
  bool ok = true;
  for (auto iter = x.begin(); iter != x.end(); ++iter, ++k) {
    auto &&[idx, v] = *iter;
    auto &&[i, j] = idx;
    const float want = (i == 2 && j == 3) ? 24.f : (i == 5 && j == 7) ? 54.f : (i == 8 && j == 9) ? 49.f : 12.f;
    ok &= i == k / 10 && j == k % 10 && float(v) == want;
  }
  EXPECT_EQ(k, (std::size_t)100);
  EXPECT_TRUE(ok);
  EXPECT_EQ(std::ranges::distance(x.begin(), x.end()), (std::ptrdiff_t)100);
}

TEST(ShpDense, TilesAndSegments) {
  // dense_matrix.hpp:198-242: tiles trimmed at the edges, segments carry
  // their origin, every element covered once, ranks from block_cyclic
  const std::size_t m = 37, n = 23;
  shp::block_cyclic part({8, 5}, {2, 2});
  shp::dense_matrix<int> a({m, n}, part);
  EXPECT_EQ(a.tile_shape()[0], (std::size_t)8);
  EXPECT_EQ(a.grid_shape()[0], (std::size_t)5);
  EXPECT_EQ(a.grid_shape()[1], (std::size_t)5);
  std::vector<int> seen(m * n, 0);
  std::size_t total = 0;
  bool ranks_ok = true, shape_ok = true;
  auto segs = a.segments();
  auto tiles = a.tiles();
  for (std::size_t t = 0; t < segs.size(); t++) {
    auto &s = segs[t];
    const std::size_t ti = t / a.grid_shape()[1], tj = t % a.grid_shape()[1];
    ranks_ok &= s.rank() == part.tile_rank({m, n}, {ti, tj}) && s.rank() < shp::nprocs();
    shape_ok &= s.origin()[0] == ti * 8 && s.origin()[1] == tj * 5 && s.shape()[0] == std::min<std::size_t>(8, m - ti * 8) &&
                s.shape()[1] == std::min<std::size_t>(5, n - tj * 5) && s.ld() == 5 &&
                tiles[t].origin()[0] == 0 && tiles[t].shape() == s.shape();
    total += s.size();
  }
  EXPECT_TRUE(ranks_ok);
  EXPECT_TRUE(shape_ok);
  EXPECT_EQ(total, m * n);
  // every element written with its global linear index by its own device
  shp::for_each(shp::par_unseq, a, [=](auto &&e) {
    auto &&[idx, v] = e;
    v = static_cast<int>(idx[0] * n + idx[1]);
  });
  bool vals = true;
  for (auto &s : segs) {
    std::vector<int> h(s.shape()[0] * s.ld());
    shp::detail::check(drhip_memcpy_d2h(static_cast<int>(s.rank()), h.data(), s.data(), h.size() * sizeof(int)), "d2h");
    for (std::size_t i = 0; i < s.shape()[0]; i++)
      for (std::size_t j = 0; j < s.shape()[1]; j++) {
        const std::size_t g = (s.origin()[0] + i) * n + s.origin()[1] + j;
        vals &= h[i * s.ld() + j] == static_cast<int>(g);
        seen[g]++;
      }
  }
  EXPECT_TRUE(vals);
  EXPECT_TRUE(std::all_of(seen.begin(), seen.end(), [](int c) { return c == 1; }));
  // operator[] and the row-major host walk agree with the layout
  EXPECT_EQ(int(a[{36, 22}]), (int)(36 * n + 22));
  EXPECT_EQ(int(a[{9, 4}]), (int)(9 * n + 4));
  bool walk = true;
  std::size_t k = 0;
  for (auto &&[idx, v] : a) walk &= idx[0] * n + idx[1] == k && int(v) == (int)k, k++;
  EXPECT_TRUE(walk);
  // tile-local views: row / column / operator[] / entries of one tile
  auto t12 = a.tile({1, 2});
  EXPECT_EQ(int(t12[{3, 4}]), (int)((8 + 3) * n + 10 + 4));
  auto row = t12.row(3);
  bool rv = row.size() == 5;
  std::size_t j = 0;
  for (auto &&[idx, v] : row) rv &= idx[0] == 3 && idx[1] == j && int(v) == (int)((8 + 3) * n + 10 + j), j++;
  EXPECT_TRUE(rv);
  auto col = t12.column(2);
  bool cv = col.size() == 8;
  std::size_t i = 0;
  for (auto &&[idx, v] : col) cv &= idx[0] == i && idx[1] == 2 && int(v) == (int)((8 + i) * n + 12), i++;
  EXPECT_TRUE(cv);
  std::vector<shp::matrix_entry<int>> es(segs[6].begin(), segs[6].end());
  EXPECT_EQ(es.size(), segs[6].size());
  EXPECT_TRUE(es.front().index() == (shp::index<>{8, 5}) && es.front().value() == (int)(8 * n + 5));
}

TEST(ShpDense, ForEachLargeTiles) {
  // 2^11 x 3000 doubles on the default partition; for_each with the 32-bit
  // divider path and a per-tile view for_each
  const std::size_t m = 2048, n = 3000;
  shp::dense_matrix<double> a({m, n});
  shp::for_each(shp::par_unseq, a, [](auto &&e) {
    auto &&[idx, v] = e;
    v = double(idx[0]) * 4096.0 + double(idx[1]);
  });
  auto segs = a.segments();
  shp::for_each(shp::par_unseq, segs.back(), [](auto &&e) { e.value() += 0.5; });
  bool ok = true;
  for (std::size_t t = 0; t < segs.size(); t++) {
    auto &s = segs[t];
    std::vector<double> h(s.shape()[0] * s.ld());
    shp::detail::check(drhip_memcpy_d2h(static_cast<int>(s.rank()), h.data(), s.data(), h.size() * sizeof(double)), "d2h");
    const double add = t + 1 == segs.size() ? 0.5 : 0.0;
    for (std::size_t i = 0; i < s.shape()[0]; i++)
      for (std::size_t j = 0; j < s.shape()[1]; j++)
        ok &= h[i * s.ld() + j] == double(s.origin()[0] + i) * 4096.0 + double(s.origin()[1] + j) + add;
  }
  EXPECT_TRUE(ok);
}

TEST(ShpDense, RowDivider) {
  // the multiply-high divider matches / and % over every divisor class
  bool ok = true;
  for (std::uint64_t d : std::vector<std::uint64_t>{1, 2, 3, 5, 7, 10, 640, 1000, 3000, 65535, 65536,
                                                    (1ull << 20) + 7, (1ull << 30) + 3}) {
    shp::detail::row_divider dv(d, (1ull << 31) - 1);
    for (std::uint64_t nn : std::vector<std::uint64_t>{0, 1, d - 1, d, d + 1, 2 * d + 3, 123456789, (1ull << 31) - 2,
                                                       (1ull << 31) - 1}) {
      if (nn >= (1ull << 31)) continue;
      std::uint64_t q, r;
      dv.divmod(nn, q, r);
      ok &= q == nn / d && r == nn % d;
    }
  }
  EXPECT_TRUE(ok);
}

// --------------------------------------------------------------- main
// ------------------------------------------ examples/shp restated as tests
// Each body is the reference example with its printing replaced by checks;
// device selection is shp::init's (the runner's device list).

// examples/shp/zip_example.cpp
TEST(ShpExamples, ZipExample) {
  using DV = shp::distributed_vector<int, shp::device_allocator<int>>;
  DV v(100);
  DV v2(50);
  shp::for_each(shp::par_unseq, shp::enumerate(v), [](auto &&tuple) {
    auto &&[idx, value] = tuple;
    value = idx;
  });
  shp::for_each(shp::par_unseq, v, [](auto &&value) { value += 2; });
  std::size_t sum = shp::reduce(shp::par_unseq, v, int(0), std::plus{});
  EXPECT_EQ(sum, std::size_t(4950 + 200));
  shp::distributed_span dspan(v.segments());
  EXPECT_EQ(dspan.size(), v.size());
  EXPECT_TRUE(equal(dspan, v));
  auto i = rng::views::iota(int32_t(0), int32_t(rng::size(v)));
  shp::zip_view zip_v(i, v);
  auto segments = zip_v.segments();
  EXPECT_EQ(rng::size(segments), rng::size(v.segments()));
  shp::for_each(shp::par_unseq, zip_v, [](auto &&tuple) {
    auto &&[i, v] = tuple;
    v = i;
  });
  shp::zip_view zip_v2(i, v2);
  shp::for_each(shp::par_unseq, zip_v2, [](auto &&tuple) {
    auto &&[i, v2] = tuple;
    v2 = i;
  });
  shp::zip_view view2(v, v2);
  shp::for_each(shp::par_unseq, view2, [](auto &&tuple) {
    auto &&[v, v2] = tuple;
    v2 = 1;
  });
  std::vector<int> want_v(100), want_v2(50, 1);
  std::iota(want_v.begin(), want_v.end(), 0);
  EXPECT_TRUE(to_host(v) == want_v);
  EXPECT_TRUE(to_host(v2) == want_v2);
}

// examples/shp/take_example.cpp
TEST(ShpExamples, TakeExample) {
  shp::distributed_vector<int, shp::device_allocator<int>> v(100);
  shp::for_each(shp::par_unseq, shp::enumerate(v), [](auto &&tuple) {
    auto &&[idx, value] = tuple;
    value = idx;
  });
  shp::for_each(shp::par_unseq, v, [](auto &&value) { value += 2; });
  auto trimmed_view = shp::views::take(v, 53);
  EXPECT_EQ(std::size_t(rng::size(trimmed_view)), std::size_t(53));
  auto sum = shp::reduce(shp::par_unseq, v, 0, std::plus{});
  EXPECT_EQ(sum, 5150);
  auto tsum = shp::reduce(shp::par_unseq, trimmed_view, 0, std::plus{});
  EXPECT_EQ(tsum, 1378 + 106);
  auto sl = v | rng::views::drop(40) | shp::views::slice({5, 10});
  std::vector<int> want{47, 48, 49, 50, 51};
  EXPECT_TRUE(shp::detail::host_values(sl) == want);
}

// examples/shp/vector_example.cpp
TEST(ShpExamples, VectorExample) {
  shp::distributed_vector<int, shp::device_allocator<int>> v(100);
  shp::for_each(shp::par_unseq, shp::enumerate(v), [](auto &&tuple) {
    auto &&[idx, value] = tuple;
    value = idx;
  });
  shp::for_each(shp::par_unseq, v, [](auto &&value) { value += 2; });
  size_t sum = shp::reduce(shp::par_unseq, v, int(0), std::plus{});
  EXPECT_EQ(sum, std::size_t(5150));
  std::vector<int> local_vec(v.size());
  std::iota(local_vec.begin(), local_vec.end(), 0);
  shp::copy(local_vec.begin(), local_vec.end(), v.begin());
  shp::for_each(shp::par_unseq, v, [](auto &&value) { value += 2; });
  shp::copy(v.begin(), v.end(), local_vec.begin());
  for (std::size_t i = 0; i < local_vec.size(); i++) EXPECT_EQ(local_vec[i], int(i) + 2);
}

// examples/shp/inclusive_scan_example.cpp
TEST(ShpExamples, InclusiveScanExample) {
  shp::distributed_vector<int, shp::device_allocator<int>> v(100);
  std::vector<int> lv(100);
  std::iota(lv.begin(), lv.end(), 0);
  shp::copy(lv.begin(), lv.end(), v.begin());
  std::inclusive_scan(lv.begin(), lv.end(), lv.begin());
  shp::inclusive_scan(shp::par_unseq, v, v);
  for (size_t i = 0; i < lv.size(); i++) EXPECT_EQ(int(v[i]), lv[i]);
  std::iota(lv.begin(), lv.end(), 0);
  shp::copy(lv.begin(), lv.end(), v.begin());
  shp::distributed_vector<int, shp::device_allocator<int>> o(v.size() + 100);
  std::inclusive_scan(lv.begin(), lv.end(), lv.begin(), std::plus<>(), 12);
  shp::inclusive_scan(shp::par_unseq, v, o, std::plus<>(), 12);
  for (size_t i = 0; i < lv.size(); i++) EXPECT_EQ(int(o[i]), lv[i]);
}

// examples/shp/test_range.cpp: user-allocated device spans gathered into a
// distributed_span; the reference fills each segment with a SYCL kernel,
// here shp::for_each over the segment does the same.
std::vector<shp::device_ptr<int>> g_ptrs;
template <typename T> auto allocate_device_span(std::size_t size, std::size_t rank, shp::context_type context,
                                                auto &&devices) {
  auto data = shp::device_allocator<T>(context, devices[rank]).allocate(size);
  g_ptrs.push_back(data);
  return shp::device_span<T, decltype(data)>(data, size, rank);
}
template <typename T> auto allocate_device_spans(std::size_t size, shp::context_type context, auto &&devices) {
  std::vector<shp::device_span<T, shp::device_ptr<T>>> spans;
  for (size_t rank = 0; rank < devices.size(); rank++)
    spans.push_back(allocate_device_span<T>(size, rank, context, devices));
  return spans;
}
TEST(ShpExamples, TestRange) {
  auto devices = shp::devices();
  std::size_t size = 200;
  std::size_t size_per_segment = (size + devices.size() - 1) / devices.size();
  auto segments = allocate_device_spans<int>(size_per_segment, shp::context(), devices);
  shp::distributed_span dspan(segments);
  for (auto &&segment : dspan.segments()) {
    int *ptr = segment.begin().local();
    (void)ptr;
    shp::for_each(shp::par_unseq, shp::enumerate(shp::distributed_span(std::vector{segment})), [](auto &&t) {
      auto &&[id, x] = t;
      x = static_cast<int>(id);
    });
  }
  auto subspan = dspan.subspan(25, 70);
  EXPECT_EQ(subspan.size(), std::size_t(70));
  std::vector<int> h = shp::detail::host_values(dspan);
  double want_sub = 0;
  for (std::size_t i = 25; i < 95; i++) want_sub += h[i];
  auto policy = shp::par_unseq;
  auto r_sub = shp::reduce(policy, subspan, 0.0f, std::plus());
  EXPECT_NEAR_REL(r_sub, want_sub, 1e-6);
  shp::for_each(policy, dspan, [](auto &&elem) { elem = elem + 2; });
  auto r = shp::reduce(policy, dspan, 0.0f, std::plus());
  double want = 0;
  for (int x : h) want += x + 2;
  EXPECT_NEAR_REL(r, want, 1e-6);
  for (std::size_t k = 0; k < g_ptrs.size(); k++)
    shp::device_allocator<int>(k).deallocate(g_ptrs[k], size_per_segment);
  g_ptrs.clear();
}

// ------------------------------------------------- boundary API coverage
TEST(ShpExtra, CopyFillAsync) {
  // copy.hpp:19-168: the async forms return an event; work on several
  // segments is in flight until wait()
  const std::size_t n = 100003;
  shp::distributed_vector<float> dv(n);
  std::vector<float> h(n), back(n);
  for (std::size_t i = 0; i < n; i++) h[i] = float(i) * 0.5f;
  auto e1 = shp::copy_async(h.begin(), h.end(), dv.begin());
  e1.wait();
  auto e2 = shp::copy_async(dv.begin(), dv.end(), back.data());
  e2.wait();
  EXPECT_TRUE(back == h);
  auto e3 = shp::fill_async(dv, 3.0f);
  e3.wait();
  EXPECT_TRUE(to_host(dv) == std::vector<float>(n, 3.0f));
  auto seg = dv.segments()[0];
  shp::fill(seg.begin(), seg.begin() + 10, 7.0f);
  std::vector<float> first(10);
  shp::copy(seg.begin(), seg.begin() + 10, first.begin());
  EXPECT_TRUE(first == std::vector<float>(10, 7.0f));
  // device_ptr -> device_ptr
  shp::distributed_vector<float> dv2(n);
  auto s2 = dv2.segments()[0];
  shp::copy(seg.begin(), seg.begin() + 10, s2.begin());
  EXPECT_EQ(float(dv2[5]), 7.0f);
}

TEST(ShpExtra, DistributedSpan) {
  const std::size_t n = 1001;
  shp::distributed_vector<int> dv(n);
  std::iota(dv.begin(), dv.end(), 0);
  shp::distributed_span ds(dv);
  EXPECT_EQ(ds.size(), n);
  EXPECT_EQ(int(ds[500]), 500);
  EXPECT_EQ(int(ds.front()), 0);
  EXPECT_EQ(int(ds.back()), int(n - 1));
  auto sub = ds.subspan(123, 456);
  EXPECT_EQ(sub.size(), std::size_t(456));
  EXPECT_EQ(int(sub[0]), 123);
  EXPECT_EQ(int(sub.last(1)[0]), 123 + 455);
  EXPECT_EQ(shp::reduce(shp::par_unseq, sub, 0L, std::plus{}), long(456) * 123 + 455L * 456 / 2);
  // segments of a sub-span follow the original segment boundaries
  std::size_t tot = 0;
  for (auto &&s : lib::ranges::segments(sub)) tot += s.size();
  EXPECT_EQ(tot, std::size_t(456));
  // iterator-pair algorithms over a distributed_span
  shp::for_each(shp::par_unseq, sub.begin(), sub.begin() + 10, [](auto &&x) { x = -1; });
  EXPECT_EQ(int(dv[123]), -1);
  EXPECT_EQ(int(dv[133]), 133);
  shp::inclusive_scan(shp::par_unseq, ds.subspan(0, 5), ds.subspan(0, 5));
  EXPECT_EQ(int(dv[4]), 0 + 1 + 2 + 3 + 4);
}

namespace user_ns {
// A user range that is distributed only through ADL customization points
// (details/ranges.hpp:24-27,89-113): segments_ of the range, rank_ of a
// segment type that has no rank() member.
struct seg {
  int *p;
  std::size_t n, r;
  int *begin() const { return p; }
  int *end() const { return p + n; }
  std::size_t size() const { return n; }
};
inline std::size_t rank_(const seg &s) { return s.r; }
struct wrapped {
  shp::distributed_vector<int> *v;
  auto begin() const { return v->begin(); }
  auto end() const { return v->end(); }
  std::size_t size() const { return v->size(); }
};
inline auto segments_(const wrapped &w) { return w.v->segments(); }
} // namespace user_ns

TEST(ShpExtra, AdlCustomization) {
  const std::size_t n = 777;
  shp::distributed_vector<int> dv(n);
  std::iota(dv.begin(), dv.end(), 1);
  user_ns::wrapped w{&dv};
  static_assert(lib::distributed_range<user_ns::wrapped>);
  EXPECT_EQ(shp::reduce(shp::par_unseq, w, 0, std::plus{}), int(n * (n + 1) / 2));
  std::vector<user_ns::seg> segs;
  for (auto &&s : dv.segments()) segs.push_back({s.data(), s.size(), s.rank()});
  static_assert(lib::remote_range<user_ns::seg>);
  EXPECT_EQ(lib::ranges::rank(segs.back()), dv.segments().back().rank());
  shp::distributed_span ds(segs);
  EXPECT_EQ(shp::reduce(shp::par_unseq, ds, 0, std::plus{}), int(n * (n + 1) / 2));
  // iterator rank(): a device_ptr is a remote iterator
  auto it = dv.segments().back().begin();
  EXPECT_EQ(lib::ranges::rank(it), dv.segments().back().rank());
  static_assert(lib::remote_iterator<decltype(it)>);
  EXPECT_TRUE(lib::ranges::local(it) == dv.segments().back().data());
}

TEST(ShpExtra, Vector) {
  // vector.hpp:14-247 on device memory (device_allocator) and on the host
  shp::vector<int, shp::device_allocator<int>> dvv(10, 5, shp::device_allocator<int>(0));
  EXPECT_EQ(dvv.size(), std::size_t(10));
  EXPECT_EQ(int(dvv[3]), 5);
  for (int i = 0; i < 40; i++) dvv.push_back(i);
  EXPECT_EQ(dvv.size(), std::size_t(50));
  EXPECT_TRUE(dvv.capacity() >= 50);
  std::vector<int> h(50);
  shp::copy(dvv.begin(), dvv.end(), h.begin());
  for (int i = 0; i < 10; i++) EXPECT_EQ(h[i], 5);
  for (int i = 0; i < 40; i++) EXPECT_EQ(h[10 + i], i);
  auto copy = dvv;
  EXPECT_EQ(int(copy[49]), 39);
  copy.resize(60, -3);
  EXPECT_EQ(int(copy[59]), -3);
  EXPECT_EQ(int(copy[49]), 39);
  shp::vector<int, shp::device_allocator<int>> il({1, 2, 3}, shp::device_allocator<int>(0));
  EXPECT_EQ(int(il[2]), 3);
  shp::vector<double> hv(4, 1.5);
  hv.push_back(2.5);
  EXPECT_EQ(hv.size(), std::size_t(5));
  EXPECT_EQ(hv[4], 2.5);
}

int main(int argc, char **argv) {
  unsigned dev_num = 0;
  std::string filter, dev_list;
  for (int i = 1; i < argc; i++) {
    std::string a = argv[i];
    if ((a == "-d" || a == "--devicesCount") && i + 1 < argc) dev_num = (unsigned)std::atoi(argv[++i]);
    else if (a.rfind("--devicesCount=", 0) == 0) dev_num = (unsigned)std::atoi(a.c_str() + 15);
    else if (a == "--filter" && i + 1 < argc) filter = argv[++i];
    else if (a == "--devices" && i + 1 < argc) dev_list = argv[++i];
  }
  auto devices = shp::get_numa_devices();
  if (devices.empty()) {
    std::printf("no HIP device\n");
    return 2;
  }
  if (!dev_list.empty()) {
    // explicit, distinct device ids (--devices 0,1,2,...): the segments
    // live on different GPUs, so every cross-segment step crosses xGMI
    std::vector<int> ids;
    for (std::size_t p = 0; p < dev_list.size();) {
      std::size_t q = dev_list.find(',', p);
      if (q == std::string::npos) q = dev_list.size();
      ids.push_back(std::atoi(dev_list.substr(p, q - p).c_str()));
      p = q + 1;
    }
    devices = ids;
  } else if (dev_num > 0) {
    devices = shp::get_duplicated_devices(devices, dev_num); // shp-tests.cpp:34-39
  }
  shp::init(devices);
  std::printf("segments: %zu on devices:", shp::nprocs());
  for (int d : shp::devices()) std::printf(" %d", d);
  std::printf("\n");
  int run = 0;
  for (auto &t : registry()) {
    const std::string full = std::string(t.suite) + "." + t.name;
    if (!filter.empty() && full.find(filter) == std::string::npos) continue;
    g_cur_failed = false;
    try {
      t.fn();
    } catch (const std::exception &e) {
      std::printf("  exception: %s\n", e.what());
      g_cur_failed = true;
    }
    std::printf("[%s] %s\n", g_cur_failed ? "FAILED" : "    OK", full.c_str());
    g_fail += g_cur_failed;
    run++;
  }
  shp::finalize();
  std::printf("%d tests, %d failed\n", run, g_fail);
  return g_fail ? 1 : 0;
}
