// mhp_tests.cpp -- the reference's mhp gtests and stencil-1d example
// (test/gtest/mhp/algorithms.cpp:124-135, test/gtest/mhp/stencil.cpp:12-55,
// examples/mhp/stencil-1d.cpp) restated against the one-process-per-GPU
// layer (distributed-ranges_amd/include/dr/mhp.hpp) on the RCCL C-ABI.
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
  struct {
    const char *name;
    void (*fn)();
  } tests[] = {{"MhpTests.Reduce", test_reduce},
               {"MhpTests.Stencil", test_stencil},
               {"MhpExamples.Stencil1d", test_stencil_1d_example},
               {"MhpTests.Stencil1dLarge", test_stencil_1d_large},
               {"MhpTests.PeriodicHalo", test_periodic_halo},
               {"MhpTests.ReduceMaxFloat", test_reduce_max_and_float}};
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
