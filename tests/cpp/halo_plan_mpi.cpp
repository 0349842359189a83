// halo_plan_mpi.cpp -- CPU test of the mhp message sequence
// (distributed-ranges_amd/include/dr/details/halo_plan.hpp) on 1..N MPICH
// ranks with host buffers: the same message list libdrhip's RCCL halo
// exchange (csrc/comm.hip) and dr/mhp_mpi.hpp's MPI transport issue.
//
// Test infrastructure only: the cell arithmetic below is the checker's
// restatement of the reference tests' transforms, not a product path.
//   MhpTests.Reduce    test/gtest/mhp/algorithms.cpp:124-135      -> 1045
//   MhpTests.Stencil   test/gtest/mhp/stencil.cpp:12-55           -> [100 x4, 154, 165, 100 x4]
//   stencil-1d         examples/mhp/stencil-1d.cpp (n 10, 5 steps) -> interior
//   plus: large 1-D stencils against a serial loop, periodic halos, and
//   the in-order pairing RCCL relies on (every rank count 1..8).
#include <dr/details/halo_plan.hpp>
#include <mpi.h>

#include <cstdio>
#include <cstring>
#include <functional>
#include <numeric>
#include <vector>

static int g_fail = 0;
static int g_rank = 0, g_size = 1;
#define CHECK(c)                                                                        \
  do {                                                                                  \
    if (!(c)) {                                                                         \
      std::printf("  rank %d FAILED %s:%d: %s\n", g_rank, __FILE__, __LINE__, #c);      \
      g_fail++;                                                                         \
    }                                                                                   \
  } while (0)

// one rank's block of a halo'd vector: host buffer [prev | segment | next]
struct hvec {
  std::size_t n, prev, next;
  bool periodic;
  dr_plan::block b;
  std::vector<int> buf;
  hvec(std::size_t n_, std::size_t r, bool per = false)
      : n(n_), prev(r), next(r), periodic(per), b(dr_plan::block_of(n_, g_size, g_rank, r, r)),
        buf(r + b.segment + r, 0) {}
  int *owned() { return buf.data() + prev; }
  void iota(int s) {
    for (std::size_t i = 0; i < b.local; i++) owned()[i] = s + (int)(b.first + i);
  }
  void fill(int v) {
    for (std::size_t i = 0; i < b.local; i++) owned()[i] = v;
  }
  // halo.hpp:55-70 exchange() through the shared message list
  void exchange() {
    const auto msgs = dr_plan::halo_messages(g_rank, g_size, b.segment, prev, next, periodic);
    std::vector<MPI_Request> req(msgs.size(), MPI_REQUEST_NULL);
    for (std::size_t i = 0; i < msgs.size(); i++)
      if (!msgs[i].send)
        MPI_Irecv(buf.data() + msgs[i].cell_off, (int)msgs[i].cells, MPI_INT, msgs[i].peer, msgs[i].tag,
                  MPI_COMM_WORLD, &req[i]);
    // sends from a copy: a send and a receive may not share cells
    std::vector<std::vector<int>> out(msgs.size());
    for (std::size_t i = 0; i < msgs.size(); i++)
      if (msgs[i].send) {
        out[i].assign(buf.begin() + msgs[i].cell_off, buf.begin() + msgs[i].cell_off + msgs[i].cells);
        MPI_Isend(out[i].data(), (int)msgs[i].cells, MPI_INT, msgs[i].peer, msgs[i].tag, MPI_COMM_WORLD, &req[i]);
      }
    MPI_Waitall((int)req.size(), req.data(), MPI_STATUSES_IGNORE);
  }
  // the whole vector on rank 0
  std::vector<int> gather() {
    std::vector<int> all(g_rank == 0 ? b.segment * g_size : 0);
    MPI_Gather(owned(), (int)b.segment, MPI_INT, all.data(), (int)b.segment, MPI_INT, 0, MPI_COMM_WORLD);
    all.resize(g_rank == 0 ? n : 0);
    return all;
  }
};

// mhp::transform over global [g0, g1) of aligned vectors
static void transform(hvec &in, hvec &out, std::size_t g0, std::size_t g1, const std::function<int(const int *)> &op) {
  for (std::size_t i = 0; i < in.b.local; i++) {
    const std::size_t g = in.b.first + i;
    if (g >= g0 && g < g1) out.owned()[i] = op(in.owned() + i);
  }
  MPI_Barrier(MPI_COMM_WORLD);
}

static void test_reduce() {
  hvec v(10, 0);
  v.iota(100);
  int local = 0; // std::reduce(seg, T(0), op) per rank
  for (std::size_t i = 0; i < v.b.local; i++) local += v.owned()[i];
  std::vector<int> all(g_size);
  MPI_Gather(&local, 1, MPI_INT, all.data(), 1, MPI_INT, 0, MPI_COMM_WORLD);
  if (g_rank == 0) CHECK(dr_plan::fold_locals(0, all.begin(), all.end(), std::plus<int>{}) == 1045);
}

static void test_stencil() {
  const std::size_t radius = 4, n = 10;
  hvec in(n, radius), out(n, radius);
  in.iota(10);
  in.exchange();
  out.fill(100);
  out.exchange();
  transform(in, out, radius, n - radius, [](const int *p) {
    int s = p[0];
    for (int i = 0; i <= 4; i++) s += p[-i] + p[i];
    return s;
  });
  auto got = out.gather();
  if (g_rank == 0) CHECK((got == std::vector<int>{100, 100, 100, 100, 154, 165, 100, 100, 100, 100}));
}

static std::vector<int> stencil_1d(std::size_t n, std::size_t steps) {
  hvec a(n, 1), b(n, 1);
  a.iota(100);
  b.fill(0);
  hvec *in = &a, *out = &b;
  for (std::size_t s = 0; s < steps; s++) {
    in->exchange();
    transform(*in, *out, 1, n - 1, [](const int *p) { return p[-1] + p[0] + p[1]; });
    std::swap(in, out);
  }
  return in->gather();
}

static void test_stencil_1d() {
  auto got = stencil_1d(10, 5);
  if (g_rank == 0)
    CHECK((std::vector<int>(got.begin() + 1, got.end() - 1) ==
           std::vector<int>{11043, 18986, 23329, 24972, 25188, 23905, 19679, 11529}));
  for (std::size_t n : {7ul, 1000ul, 12345ul}) {
    const std::size_t steps = 6;
    auto g = stencil_1d(n, steps);
    if (g_rank) continue;
    std::vector<int> x(n), y(n, 0);
    std::iota(x.begin(), x.end(), 100);
    std::vector<int> *i0 = &x, *o0 = &y;
    for (std::size_t s = 0; s < steps; s++) {
      for (std::size_t i = 1; i + 1 < n; i++) (*o0)[i] = (*i0)[i - 1] + (*i0)[i] + (*i0)[i + 1];
      std::swap(i0, o0);
    }
    CHECK(g == *i0);
  }
}

static void test_periodic() {
  for (std::size_t r : {1ul, 3ul}) {
    const std::size_t n = 1000;
    hvec v(n, r, true);
    v.iota(7);
    v.exchange();
    const std::size_t p = g_size, seg = v.b.segment, k = g_rank;
    const std::size_t pr = (k + p - 1) % p, nx = (k + 1) % p;
    auto g = [&](std::size_t i) { return i < n ? (int)(7 + i) : 0; }; // cells past n stay 0
    bool ok = true;
    for (std::size_t i = 0; i < r; i++) {
      ok &= v.buf[i] == g(pr * seg + seg - r + i);
      ok &= v.buf[r + seg + i] == g(nx * seg + i);
    }
    CHECK(ok);
  }
}

// RCCL pairs a peer's sends with our receives in issue order, untagged:
// for every rank count and both end conditions, the k-th send from a to b
// must have the size of the k-th receive at b from a, and land where the
// tagged (MPI) pairing puts it.
static void test_inorder_pairing() {
  if (g_rank) return;
  for (int p = 1; p <= 8; p++)
    for (int per = 0; per < 2; per++) {
      const std::size_t r = 2, seg = 5;
      std::vector<std::vector<dr_plan::halo_msg>> m(p);
      for (int k = 0; k < p; k++) m[k] = dr_plan::halo_messages(k, p, seg, r, r, per);
      for (int a = 0; a < p; a++)
        for (int b = 0; b < p; b++) {
          std::vector<dr_plan::halo_msg> s, v;
          for (auto &x : m[a])
            if (x.send && x.peer == b) s.push_back(x);
          for (auto &x : m[b])
            if (!x.send && x.peer == a) v.push_back(x);
          CHECK(s.size() == v.size());
          for (std::size_t i = 0; i < s.size() && i < v.size(); i++) {
            CHECK(s[i].cells == v[i].cells);
            CHECK(s[i].tag == v[i].tag);
          }
        }
    }
}

// dr_plan::exchange_plan (the misaligned mhp::copy / transform exchange) on
// host buffers: every rank holds its owned input block of global values,
// MPI_Alltoallv moves the pieces the plan lists, and the gathered output
// must equal a serial std::copy of [a, b) to o -- over many shapes,
// including different segment sizes (halo'd layouts) and n_in != n_out.
static void test_exchange_plan() {
  unsigned long long seed = 12345;
  auto rnd = [&](std::size_t m) {
    seed = seed * 6364136223846793005ull + 1442695040888963407ull;
    return m ? (std::size_t)((seed >> 33) % m) : 0;
  };
  for (int trial = 0; trial < 300; trial++) {
    const std::size_t n_in = 1 + rnd(200), n_out = 1 + rnd(200);
    const std::size_t hin = rnd(4) == 0 ? rnd(40) : 0, hout = rnd(4) == 0 ? rnd(40) : 0; // halo'd segment sizes
    const auto bi = dr_plan::block_of(n_in, g_size, g_rank, hin, hin);
    const auto bo = dr_plan::block_of(n_out, g_size, g_rank, hout, hout);
    const std::size_t a = rnd(n_in), b = a + rnd(n_in - a + 1);
    const std::size_t len = std::min(b - a, n_out);
    const std::size_t o = rnd(n_out - len + 1);
    const std::size_t bb = a + len;
    std::vector<int> in(bi.segment), out(bo.segment, -1);
    for (std::size_t i = 0; i < bi.local; i++) in[i] = (int)(bi.first + i) * 7 + 1;
    const auto e = dr_plan::exchange_plan(n_in, bi.segment, a, bb, n_out, bo.segment, o, g_size, g_rank);
    std::vector<int> sc(g_size), sd(g_size), rc(g_size), rd(g_size);
    std::size_t tot = 0;
    for (int r = 0; r < g_size; r++) {
      sc[r] = (int)e.send_cnt[r];
      sd[r] = (int)e.send_off[r];
      rc[r] = (int)e.recv_cnt[r];
      rd[r] = (int)e.recv_off[r];
      tot += e.recv_cnt[r];
      CHECK(e.send_off[r] + e.send_cnt[r] <= bi.local || !e.send_cnt[r]);
      CHECK(e.recv_off[r] + e.recv_cnt[r] <= bo.local || !e.recv_cnt[r]);
    }
    CHECK(tot == e.recv_total);
    MPI_Alltoallv(in.data(), sc.data(), sd.data(), MPI_INT, out.data(), rc.data(), rd.data(), MPI_INT,
                  MPI_COMM_WORLD);
    // gather every rank's owned output part on rank 0
    std::vector<int> all(g_rank == 0 ? (std::size_t)g_size * bo.segment : 0);
    MPI_Gather(out.data(), (int)bo.segment, MPI_INT, all.data(), (int)bo.segment, MPI_INT, 0, MPI_COMM_WORLD);
    if (g_rank == 0) {
      bool ok = true;
      for (std::size_t k = 0; k < len; k++) ok &= all[o + k] == (int)(a + k) * 7 + 1;
      for (std::size_t g = 0; g < n_out; g++)
        if (g < o || g >= o + len) ok &= all[g] == -1; // untouched
      CHECK(ok);
    }
  }
}

int main(int argc, char **argv) {
  MPI_Init(&argc, &argv);
  MPI_Comm_rank(MPI_COMM_WORLD, &g_rank);
  MPI_Comm_size(MPI_COMM_WORLD, &g_size);
  struct {
    const char *name;
    void (*fn)();
  } tests[] = {{"MhpTests.Reduce", test_reduce},     {"MhpTests.Stencil", test_stencil},
               {"MhpExamples.Stencil1d", test_stencil_1d}, {"HaloPlan.Periodic", test_periodic},
               {"HaloPlan.InOrderPairing", test_inorder_pairing}, {"ExchangePlan.MisalignedCopy", test_exchange_plan}};
  for (auto &t : tests) {
    const int before = g_fail;
    t.fn();
    int mine = g_fail - before, any = 0;
    MPI_Allreduce(&mine, &any, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD);
    if (g_rank == 0) std::printf("[%s] %s (%d ranks)\n", any ? "FAILED" : "  OK  ", t.name, g_size);
  }
  int total = 0;
  MPI_Allreduce(&g_fail, &total, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD);
  if (g_rank == 0) std::printf("%s: %d failure(s)\n", total ? "FAILED" : "PASSED", total);
  MPI_Finalize();
  return total ? 1 : 0;
}
