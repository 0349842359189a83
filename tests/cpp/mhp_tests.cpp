// mhp_tests.cpp -- the reference's mhp gtests and stencil-1d example
// (test/gtest/mhp/{algorithms,views,distributed_vector,alignment,stencil}.cpp,
// examples/mhp/stencil-1d.cpp) restated against the one-process-per-GPU
// layer (distributed-ranges_amd/include/dr/mhp.hpp) on the RCCL C-ABI or
// MPI.  Checks run on rank 0 against std:: on host vectors, as the
// reference's do; the distributed side is read back with mhp::gather (the
// reference reads remote elements through its MPI window, which this layer
// does not have -- root-only element writes become the collective
// mhp::copy(root, ...) from root's host data, DistributedVector* below).
//
// bin/mhp_tests: one rank, or --rank r --nranks p --id-file F for a p-GPU
// job over RCCL (rank 0 writes the communicator id to F, the others wait
// for it).  bin/mhp_tests_mpi (this file with -DMHP_TESTS_MPI, linked
// against MPICH): every rank from mpiexec, `--transport mpi` (default; the
// reference's own MPI messages, several ranks may share ONE GPU, which
// RCCL refuses) or `--transport rccl` (one rank per GPU, id by MPI_Bcast).
// The reference runs its mhp suite on 1-4 ranks
// (test/gtest/mhp/CMakeLists.txt:27-33); tests/test_gpu_mhp.py does too.
// Known answers: tests/golden/shp_known_answers.json (mhp_reduce,
// mhp_stencil, stencil_1d), from the reference's own expected values.
#include <dr/mhp.hpp>
#ifdef MHP_TESTS_MPI
#include <dr/mhp_mpi.hpp>
#endif

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <numeric>
#include <random>
#include <string>
#include <thread>
#include <vector>

static int g_fail = 0;
#define EXPECT_TRUE(c)                                                       \
  do {                                                                       \
    if (!(c)) {                                                              \
      std::printf("  FAILED %s:%d: %s\n", __FILE__, __LINE__, #c);           \
      g_fail++;                                                              \
    }                                                                        \
  } while (0)

using T = int;

// MhpTests.Reduce: iota from 100 over n = 10, root 0 -> 1045
static void test_reduce() {
  mhp::distributed_vector<T> dv(10);
  mhp::iota(dv, 100);
  auto r = mhp::reduce(0, dv.begin(), dv.end(), 0, std::plus{});
  if (mhp::rank() == 0) EXPECT_TRUE(r == 1045);
  else EXPECT_TRUE(r == 0);
}

// MhpTests.Stencil: radius 4, s = v + sum_{i=0..4}(p[-i] + p[i])
static void test_stencil() {
  const std::size_t radius = 4, n = 10;
  mhp::distributed_vector<T> in(n, lib::halo_bounds(radius)), out(n, lib::halo_bounds(radius));
  mhp::iota(in, 10);
  in.halo().exchange();
  mhp::fill(out, 100);
  out.halo().exchange();
  auto sum = [](auto &&v) {
    T s = v;
    auto p = &v;
    for (std::size_t i = 0; i <= 4; i++) {
      s += p[-(std::ptrdiff_t)i];
      s += p[i];
    }
    return s;
  };
  mhp::transform(in.begin() + radius, in.end() - radius, out.begin() + radius, sum);
  auto got = mhp::gather(out);
  if (mhp::rank() == 0) EXPECT_TRUE((got == std::vector<T>{100, 100, 100, 100, 154, 165, 100, 100, 100, 100}));
}

// examples/mhp/stencil-1d.cpp: 3-point, halo 1, n = 10, 5 steps, ping-pong
static std::vector<T> stencil_1d(std::size_t n, std::size_t steps) {
  lib::halo_bounds hb(1);
  mhp::distributed_vector<T> a(n, hb), b(n, hb);
  mhp::iota(a, 100);
  mhp::fill(b, 0);
  auto op = [](auto &&v) {
    auto p = &v;
    return p[-1] + p[0] + p[+1];
  };
  auto in = mhp::subrange(a.begin() + 1, a.end() - 1);
  auto out = mhp::subrange(b.begin() + 1, b.end() - 1);
  for (std::size_t s = 0; s < steps; s++) {
    mhp::halo(in).exchange();
    mhp::transform(in, out.begin(), op);
    std::swap(in, out);
  }
  return mhp::gather(*in.first.dv);
}

static void test_stencil_1d_example() {
  auto got = stencil_1d(10, 5);
  if (mhp::rank() == 0) {
    std::vector<T> interior(got.begin() + 1, got.end() - 1);
    EXPECT_TRUE((interior == std::vector<T>{11043, 18986, 23329, 24972, 25188, 23905, 19679, 11529}));
  }
}

// larger sizes against the serial loop of the example's check()
static void test_stencil_1d_large() {
  for (std::size_t n : {1000ul, 1ul << 20}) {
    const std::size_t steps = 7;
    auto got = stencil_1d(n, steps);
    if (mhp::rank() != 0) continue;
    std::vector<T> a(n), b(n, 0);
    std::iota(a.begin(), a.end(), 100);
    std::vector<T> *in = &a, *out = &b;
    for (std::size_t s = 0; s < steps; s++) {
      for (std::size_t i = 1; i + 1 < n; i++) (*out)[i] = (*in)[i - 1] + (*in)[i] + (*in)[i + 1];
      std::swap(in, out);
    }
    bool ok = true;
    for (std::size_t i = 1; i + 1 < n; i++) ok &= got[i] == (*in)[i];
    EXPECT_TRUE(ok);
  }
}

// periodic halo: rank 0's prev halo wraps to the last rank's segment tail
static void test_periodic_halo() {
  const std::size_t n = 1000, r = 3;
  mhp::distributed_vector<T> dv(n, lib::halo_bounds(r, true));
  mhp::iota(dv, 7);
  dv.halo().exchange();
  auto h = mhp::local_buffer(dv);
  const std::size_t p = mhp::nprocs(), seg = dv.segment_size(), k = mhp::rank();
  auto g = [&](std::size_t i) { return i < n ? (T)(7 + i) : T(0); }; // cells past n stay zero
  bool ok = true;
  const std::size_t prev_rank = (k + p - 1) % p, next_rank = (k + 1) % p;
  for (std::size_t i = 0; i < r; i++) {
    ok &= h[i] == g(prev_rank * seg + seg - r + i);
    ok &= h[r + seg + i] == g(next_rank * seg + i);
  }
  EXPECT_TRUE(ok);
}

// mhp::reduce with a non-additive op keeps the reference's T(0) seeds
// (cpu_algorithms.hpp:109-120): max over positive values is unaffected
static void test_reduce_max_and_float() {
  mhp::distributed_vector<T> dv(12345);
  mhp::iota(dv, 3);
  auto m = mhp::reduce(0, dv.begin(), dv.end(), 0, [](T x, T y) { return x > y ? x : y; });
  if (mhp::rank() == 0) EXPECT_TRUE(m == 3 + 12344);
  mhp::distributed_vector<double> dd(1 << 20);
  mhp::fill(dd, 0.5);
  auto s = mhp::reduce(0, dd.begin() + 10, dd.end(), 1.0, std::plus{});
  if (mhp::rank() == 0) EXPECT_TRUE(s == 1.0 + 0.5 * ((1 << 20) - 10));
}


using V = std::vector<T>;
using DV = mhp::distributed_vector<T>;

static V iota_v(std::size_t n, T start) {
  V v(n);
  std::iota(v.begin(), v.end(), start);
  return v;
}
static bool equal(DV &dv, const V &v) {
  auto g = mhp::gather(dv);
  return mhp::rank() != 0 || g == v;
}
template <typename R> static bool equal_r(const R &r, const V &v) {
  auto g = mhp::gather(r);
  return mhp::rank() != 0 || V(g.begin(), g.end()) == v;
}

// MhpTests.Fill (algorithms.cpp:12-46): fill over an iterator pair and over
// a subrange, at [0, n) and [n/2 - 1, n/2 + 1)
static void check_fill(std::size_t n, std::size_t b, std::size_t size) {
  const std::size_t e = b + size;
  const T val = 33;
  DV dv1(n), dv3(n);
  mhp::iota(dv1, 10);
  mhp::iota(dv3, 10);
  mhp::fill(dv1.begin() + b, dv1.begin() + e, val);
  mhp::fill(mhp::subrange(dv3.begin() + b, dv3.begin() + e), val);
  mhp::fence();
  V v = iota_v(n, 10);
  std::fill(v.begin() + b, v.begin() + e, val);
  EXPECT_TRUE(equal(dv1, v));
  EXPECT_TRUE(equal(dv3, v));
}
static void test_fill() {
  const std::size_t n = 10;
  check_fill(n, 0, n);
  check_fill(n, n / 2 - 1, 2);
  check_fill(100003, 777, 50000); // segment boundaries inside the range
}

struct negate {
  __host__ __device__ void operator()(auto &&v) const { v = -v; }
};
struct increment {
  __host__ __device__ void operator()(auto &&v) const { v++; }
};

// MhpTests.ForEach (algorithms.cpp:48-66)
static void test_for_each() {
  const std::size_t n = 10;
  DV dv_a(n);
  mhp::iota(dv_a, 100);
  mhp::for_each(dv_a, negate{});
  V a = iota_v(n, 100);
  std::for_each(a.begin(), a.end(), negate{});
  EXPECT_TRUE(equal(dv_a, a));
  // the iterator-pair form over an interior subrange
  mhp::for_each(dv_a.begin() + 2, dv_a.end() - 3, increment{});
  std::for_each(a.begin() + 2, a.end() - 3, increment{});
  EXPECT_TRUE(equal(dv_a, a));
}

// MhpTests.Copy (algorithms.cpp:68-93): aligned copies and the misaligned
// copy(src + 1 .. end - 1 -> dst + 2), which is one collective alltoallv here
static void test_copy() {
  for (std::size_t n : {10ul, 1000ul, 65537ul}) {
    DV dv_src(n), dv_dst1(n), dv_dst2(n), dv_dst3(n);
    mhp::iota(dv_src, 100);
    mhp::iota(dv_dst1, 200);
    mhp::iota(dv_dst2, 200);
    mhp::iota(dv_dst3, 200);
    mhp::copy(dv_src, dv_dst1.begin());
    mhp::copy(dv_src.begin(), dv_src.end(), dv_dst2.begin());
    mhp::copy(dv_src.begin() + 1, dv_src.end() - 1, dv_dst3.begin() + 2);
    V v_src = iota_v(n, 100), v_dst = iota_v(n, 200), v_dst3 = iota_v(n, 200);
    std::copy(v_src.begin(), v_src.end(), v_dst.begin());
    EXPECT_TRUE(equal(dv_dst1, v_dst));
    EXPECT_TRUE(equal(dv_dst2, v_dst));
    std::copy(v_src.begin() + 1, v_src.end() - 1, v_dst3.begin() + 2);
    EXPECT_TRUE(equal(dv_dst3, v_dst3));
    // overlapping shift inside ONE vector (std::copy_backward semantics of a
    // whole-range move: the source is read before any element is written)
    V v_in = iota_v(n, 5);
    DV dv_in(n);
    mhp::iota(dv_in, 5);
    mhp::copy(dv_in.begin(), dv_in.end() - 3, dv_in.begin() + 3);
    V ref = v_in;
    std::copy(v_in.begin(), v_in.end() - 3, ref.begin() + 3);
    EXPECT_TRUE(equal(dv_in, ref));
  }
}

// MhpTests.Transform (algorithms.cpp:95-122)
static void test_transform() {
  auto copy = [](auto x) { return x; };
  auto twice = [](auto x) { return 2 * x + 1; };
  for (std::size_t n : {10ul, 4099ul}) {
    DV dv_src(n), dv_dst1(n), dv_dst2(n), dv_dst3(n);
    mhp::iota(dv_src, 100);
    mhp::iota(dv_dst1, 200);
    mhp::iota(dv_dst2, 200);
    mhp::iota(dv_dst3, 200);
    mhp::transform(dv_src, dv_dst1.begin(), copy);
    mhp::transform(dv_src.begin(), dv_src.end(), dv_dst2.begin(), copy);
    mhp::transform(dv_src.begin() + 1, dv_src.end() - 1, dv_dst3.begin() + 2, twice);
    V v_src = iota_v(n, 100), v_dst = iota_v(n, 200), v_dst3 = iota_v(n, 200);
    std::transform(v_src.begin(), v_src.end(), v_dst.begin(), copy);
    EXPECT_TRUE(equal(dv_dst1, v_dst));
    EXPECT_TRUE(equal(dv_dst2, v_dst));
    std::transform(v_src.begin() + 1, v_src.end() - 1, v_dst3.begin() + 2, twice);
    EXPECT_TRUE(equal(dv_dst3, v_dst3));
  }
}

// MhpTests.Subrange (views.cpp:16-21): a subrange is a distributed range --
// its segments tile it in rank order
static void test_subrange() {
  DV dv(10);
  auto r = mhp::subrange(dv.begin(), dv.end());
  auto segs = mhp::segments(r);
  std::size_t tot = 0, prev_end = 0;
  bool ok = !segs.empty();
  for (auto &s : segs) {
    ok &= s.global_begin() == prev_end && s.rank() < mhp::nprocs();
    prev_end = s.global_begin() + s.size();
    tot += s.size();
  }
  EXPECT_TRUE(ok && tot == 10);
  auto sub = mhp::subrange(dv.begin() + 3, dv.end() - 2);
  tot = 0;
  for (auto &s : mhp::segments(sub)) tot += s.size();
  EXPECT_TRUE(tot == 5 && mhp::segments(sub).front().global_begin() == 3);
}

// MhpTests.Zip (views.cpp:23-47): zip of two aligned vectors, for_each
// incrementing .first
static void test_zip() {
  DV dv1(10), dv2(10);
  mhp::iota(dv1, 10);
  mhp::iota(dv2, 20);
  auto dzv = mhp::views::zip(dv1, dv2);
  EXPECT_TRUE(mhp::aligned(dzv));
  mhp::barrier();
  auto incr_first = [](auto x) { x.first++; };
  mhp::for_each(dzv, incr_first);
  V v1 = iota_v(10, 10), v2 = iota_v(10, 20);
  for (auto &x : v1) x++;
  EXPECT_TRUE(equal(dv1, v1));
  EXPECT_TRUE(equal(dv2, v2));
  // a misaligned zip has no segments: for_each refuses it
  auto bad = mhp::views::zip(dv1, mhp::views::drop(dv2, 1));
  EXPECT_TRUE(mhp::nprocs() == 1 || !mhp::aligned(bad));
}

// MhpTests.Take / Drop (views.cpp:49-101)
static void test_take_drop() {
  const int n = 10;
  DV dv_a(n);
  mhp::iota(dv_a, 20);
  auto take = mhp::views::take(dv_a, 2);
  EXPECT_TRUE(equal_r(take, V{20, 21}));
  mhp::barrier();
  mhp::for_each(take, increment{});
  EXPECT_TRUE(equal_r(take, V{21, 22}));

  DV dv_b(n);
  mhp::iota(dv_b, 20);
  auto drop = mhp::views::drop(dv_b, 2);
  EXPECT_TRUE(equal_r(drop, iota_v(n - 2, 22)));
  mhp::barrier();
  mhp::for_each(drop, increment{});
  EXPECT_TRUE(equal_r(drop, iota_v(n - 2, 23)));
  std::size_t tot = 0;
  for (auto &s : mhp::segments(drop)) tot += s.size();
  EXPECT_TRUE(tot == (std::size_t)n - 2);
}

// MhpTests.TransformView (views.cpp:103-116)
static void test_transform_view() {
  const int n = 10;
  DV dv_a(n);
  mhp::iota(dv_a, 20);
  auto incr = [](auto x) { return x + 1; };
  auto view = mhp::views::transform(dv_a, incr);
  EXPECT_TRUE(equal_r(view, iota_v(n, 21)));
}

// MhpTests.DistributedVectorRequirements / Constructors / Query
// (distributed_vector.cpp:12-34), as this layer's concepts
static void test_dv_requirements() {
  static_assert(mhp::vector_range<DV &>);
  static_assert(mhp::vector_range<mhp::dv_range<T>>);
  DV a1(10);
  EXPECT_TRUE(a1.size() == 10);
  auto segs = a1.segments();
  std::size_t tot = 0;
  for (auto &s : segs) tot += s.size();
  EXPECT_TRUE(tot == 10 && segs.size() <= mhp::nprocs());
  // local_segments (mhp/views.hpp:9-21): this rank's span, sizes summing to n
  std::size_t mine = 0;
  for (auto &s : mhp::local_segments(a1)) mine += s.size();
  EXPECT_TRUE(mine == a1.local_size());
}

// MhpTests.DistributedVectorIndex / Algorithms (distributed_vector.cpp:
// 36-86): root writes through the vector, every rank sees the values --
// collective copy from root's host data here, gather for the reads
static void test_dv_index_algorithms() {
  const std::size_t n = 10;
  const int root = 0;
  DV dv(n);
  V ref(n);
  std::iota(ref.begin(), ref.end(), 10);
  mhp::copy(root, ref.data(), n, dv.begin()); // dv[i] = i + 10
  mhp::fence();
  EXPECT_TRUE(equal(dv, ref));
  std::iota(ref.begin(), ref.end(), 11);
  mhp::copy(root, ref.data(), n, dv.begin());
  EXPECT_TRUE(equal(dv, ref));
  // a partial write in the middle (dv2[3] = dv[3])
  DV dv2(n);
  T v3 = 0;
  mhp::copy(root, mhp::subrange(dv.begin() + 3, dv.begin() + 4), &v3);
  mhp::copy(root, &v3, 1, dv2.begin() + 3);
  V r2(n, 0);
  r2[3] = 14;
  EXPECT_TRUE(equal(dv2, r2));
  // rng::copy(dv, host) on root
  V back(n, -1);
  mhp::copy(root, mhp::range_of(dv), back.data());
  if (mhp::rank() == (std::size_t)root) EXPECT_TRUE(back == ref);
}

// MhpTests.IteratorConformance (alignment.cpp:12-38)
static void test_alignment() {
  DV dv1(10), dv2(10);
  EXPECT_TRUE(mhp::aligned(dv1.begin(), dv2.begin()));
  EXPECT_TRUE(mhp::aligned(dv1.begin(), dv2.begin(), dv1.begin()));
  if (mhp::nprocs() > 1) {
    EXPECT_TRUE(!mhp::aligned(dv1.begin() + 1, dv2.begin()));
    EXPECT_TRUE(!mhp::aligned(dv1.begin() + 1, dv2.begin(), dv2.begin()));
    EXPECT_TRUE(!mhp::aligned(dv2.begin(), dv1.begin() + 1, dv2.begin()));
  }
  auto aligned_z = mhp::views::zip(dv1, dv2);
  auto misaligned_z = mhp::views::zip(dv1, mhp::views::drop(dv2, 1));
  EXPECT_TRUE(mhp::aligned(aligned_z));
  EXPECT_TRUE(mhp::nprocs() == 1 || !mhp::aligned(misaligned_z));
}

// ---- C5 at its configured size through this layer (--c5 LOG2N STEPS):
// examples/mhp/stencil-1d.cpp:16-66 on mhp::distributed_vector<float>(2^LOG2N,
// halo_bounds(1)) -- `in` = [1, n-1), 3-point p[-1] + p[0] + p[1], STEPS
// ping-pong steps, each a span_halo exchange (details/halo.hpp:336-387) and
// an mhp::transform.  Input u01 floats from a hash of the global index,
// generated on every rank's device.  Every rank checks, bit-exact, the cells
// of its own segment within 4096 of either segment edge and of 64 global
// random windows against a serial fp32 simulation of the same slab (same
// left-to-right sums; boundary cells 0 and n-1 never written).  The counts
// go to rank 0 with mhp::reduce.
__host__ __device__ inline float c5_value(std::size_t g) {
  std::uint64_t z = 0xC5 + g + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}
__global__ void c5_gen(float *p, std::size_t n, std::size_t g0) {
  const std::size_t i = blockIdx.x * (std::size_t)blockDim.x + threadIdx.x;
  if (i < n) p[i] = c5_value(g0 + i);
}
// cells [lo, hi) after `steps` steps, exact where lo == 0 or i - lo > steps,
// and hi == n or hi - i > steps
static std::vector<float> c5_serial(std::size_t n, std::size_t lo, std::size_t hi, std::size_t steps) {
  std::vector<float> a(hi - lo), b(hi - lo, 0.0f);
  for (std::size_t i = lo; i < hi; i++) a[i - lo] = c5_value(i);
  std::vector<float> *in = &a, *out = &b;
  for (std::size_t s = 0; s < steps; s++) {
    for (std::size_t i = std::max<std::size_t>(lo + 1, 1); i + 1 < hi && i + 1 < n; i++)
      (*out)[i - lo] = (*in)[i - 1 - lo] + (*in)[i - lo] + (*in)[i + 1 - lo];
    std::swap(in, out);
  }
  return *in;
}
static int run_c5(std::size_t log2n, std::size_t steps) {
  const std::size_t n = std::size_t(1) << log2n;
  lib::halo_bounds hb(1);
  mhp::distributed_vector<float> a(n, hb), b(n, hb);
  if (a.local_size())
    hipLaunchKernelGGL(c5_gen, dim3((unsigned)((a.local_size() + 255) / 256)), dim3(256), 0, mhp::detail::stream(),
                       a.owned(), a.local_size(), a.first_index());
  mhp::fill(b, 0.0f); // barrier included
  auto op = [](auto &&v) {
    auto p = &v;
    return p[-1] + p[0] + p[+1];
  };
  auto in = mhp::subrange(a.begin() + 1, a.end() - 1);
  auto out = mhp::subrange(b.begin() + 1, b.end() - 1);
  const auto t0 = std::chrono::steady_clock::now();
  for (std::size_t s = 0; s < steps; s++) {
    mhp::halo(in).exchange();
    mhp::transform(in, out.begin(), op);
    std::swap(in, out);
  }
  mhp::barrier();
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  // this rank's check windows: both edges of its segment, the global ends,
  // and the parts of 64 global random windows inside its segment
  auto &res = *in.first.dv;
  const std::size_t f = res.first_index(), e = f + res.local_size(), W = 4096;
  std::vector<std::pair<std::size_t, std::size_t>> win;
  auto add = [&](std::size_t lo, std::size_t hi) {
    lo = std::max(lo, f), hi = std::min(hi, e);
    if (lo < hi) win.push_back({lo, hi});
  };
  add(f, f + W);
  add(e >= W ? e - W : 0, e);
  std::uint64_t z = 0xC5C5;
  for (int r = 0; r < 64; r++) {
    z = z * 6364136223846793005ull + 1442695040888963407ull;
    const std::size_t s0 = (std::size_t)((z >> 16) % (n - W));
    add(s0, s0 + W);
  }
  long bad = 0, checked = 0;
  std::vector<float> got;
  for (auto [lo, hi] : win) {
    got.resize(hi - lo);
    mhp::detail::check(drhip_memcpy_d2h(0, got.data(), res.owned() + (lo - f), (hi - lo) * sizeof(float)), "d2h");
    mhp::detail::sync();
    const std::size_t slo = lo >= steps ? lo - steps : 0, shi = std::min(n, hi + steps);
    const auto ref = c5_serial(n, slo, shi, steps);
    for (std::size_t i = lo; i < hi; i++) {
      bad += std::memcmp(&got[i - lo], &ref[i - slo], 4) != 0;
      checked++;
    }
  }
  // every rank's counts to rank 0 (mhp::reduce: locals seeded with T(0))
  mhp::distributed_vector<long> cnt(2 * mhp::nprocs());
  {
    const long mine[2] = {bad, checked};
    mhp::detail::check(drhip_memcpy_h2d(0, cnt.owned(), mine, sizeof mine), "h2d");
    mhp::detail::sync();
  }
  mhp::barrier();
  // segment of cnt per rank is 2 longs: bad at even, checked at odd
  auto all = mhp::gather(cnt);
  if (mhp::rank() == 0) {
    long tb = 0, tc = 0;
    for (std::size_t r = 0; r < mhp::nprocs(); r++) tb += all[2 * r], tc += all[2 * r + 1];
    std::printf("{\"config\": \"C5\", \"layer\": \"mhp\", \"transport\": \"%s\", \"cells\": %zu, \"ranks\": %zu, "
                "\"steps\": %zu, \"cells_checked\": %ld, \"cell_mismatches\": %ld, \"steps_ms\": %.2f, \"ok\": %s}\n",
                mhp::comm().name(), n, mhp::nprocs(), steps, tc, tb, ms, tb == 0 && tc > 0 ? "true" : "false");
    return tb == 0 && tc > 0 ? 0 : 1;
  }
  return 0;
}

int main(int argc, char **argv) {
  int rank = 0, nranks = 1, device = 0;
  const char *id_file = nullptr;
  const char *tr = "mpi";
  for (int i = 1; i + 1 < argc; i += 2) {
    if (!std::strcmp(argv[i], "--rank")) rank = std::atoi(argv[i + 1]);
    else if (!std::strcmp(argv[i], "--nranks")) nranks = std::atoi(argv[i + 1]);
    else if (!std::strcmp(argv[i], "--device")) device = std::atoi(argv[i + 1]);
    else if (!std::strcmp(argv[i], "--id-file")) id_file = argv[i + 1];
    else if (!std::strcmp(argv[i], "--transport")) tr = argv[i + 1];
  }
#ifdef MHP_TESTS_MPI
  MPI_Init(&argc, &argv);
  bool dev_given = false;
  for (int i = 1; i < argc; i++) dev_given |= !std::strcmp(argv[i], "--device");
  mhp::init_mpi(dev_given ? device : -1, !std::strcmp(tr, "rccl"));
  rank = (int)mhp::rank();
  nranks = (int)mhp::nprocs();
#else
  (void)tr;
  if (nranks == 1) {
    mhp::init(device);
  } else {
    if (!id_file) {
      std::printf("--id-file is required with --nranks > 1\n");
      return 2;
    }
    mhp::comm_id id{};
    if (rank == 0) {
      id = mhp::make_comm_id();
      std::string tmp = std::string(id_file) + ".tmp";
      std::ofstream(tmp, std::ios::binary).write(id.data(), id.size());
      std::rename(tmp.c_str(), id_file);
    } else {
      for (int t = 0; t < 6000; t++) { // up to 60 s
        std::ifstream f(id_file, std::ios::binary);
        if (f && f.read(id.data(), id.size())) break;
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
      }
    }
    mhp::init(rank, nranks, device, id);
  }
#endif
  for (int i = 1; i + 2 < argc; i++)
    if (!std::strcmp(argv[i], "--c5")) {
      int rc = 1;
      try {
        rc = run_c5((std::size_t)std::atoi(argv[i + 1]), (std::size_t)std::atoi(argv[i + 2]));
      } catch (const std::exception &e) {
        std::printf("{\"config\": \"C5\", \"ok\": false, \"error\": \"%s\"}\n", e.what());
      }
      mhp::finalize();
#ifdef MHP_TESTS_MPI
      MPI_Finalize();
#endif
      return rc;
    }
  struct {
    const char *name;
    void (*fn)();
  } tests[] = {{"MhpTests.Reduce", test_reduce},
               {"MhpTests.Stencil", test_stencil},
               {"MhpExamples.Stencil1d", test_stencil_1d_example},
               {"MhpTests.Stencil1dLarge", test_stencil_1d_large},
               {"MhpTests.PeriodicHalo", test_periodic_halo},
               {"MhpTests.ReduceMaxFloat", test_reduce_max_and_float},
               {"MhpTests.Fill", test_fill},
               {"MhpTests.ForEach", test_for_each},
               {"MhpTests.Copy", test_copy},
               {"MhpTests.Transform", test_transform},
               {"MhpTests.Subrange", test_subrange},
               {"MhpTests.Zip", test_zip},
               {"MhpTests.TakeDrop", test_take_drop},
               {"MhpTests.TransformView", test_transform_view},
               {"MhpTests.DistributedVectorRequirements", test_dv_requirements},
               {"MhpTests.DistributedVectorIndexAlgorithms", test_dv_index_algorithms},
               {"MhpTests.IteratorConformance", test_alignment}};
  for (auto &t : tests) {
    const int before = g_fail;
    try {
      t.fn();
    } catch (const std::exception &e) {
      std::printf("  EXCEPTION %s\n", e.what());
      g_fail++;
    }
    std::printf("[%s] %s (rank %d of %d, %s)\n", g_fail == before ? "  OK  " : "FAILED", t.name, rank, nranks,
                mhp::comm().name());
  }
  mhp::finalize();
#ifdef MHP_TESTS_MPI
  MPI_Finalize();
#endif
  std::printf("%s: %d failure(s)\n", g_fail ? "FAILED" : "PASSED", g_fail);
  return g_fail ? 1 : 0;
}
