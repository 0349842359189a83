// cpu_bench.cpp -- the CPU baseline of bench.py (TEST/MEASUREMENT
// INFRASTRUCTURE, never the product path): the reference's mhp-style CPU
// execution of each BASELINE config, restated on OpenMP threads playing the
// MPI ranks (one block of ceil(n/P) per rank, mhp/containers/
// distributed_vector.hpp:190-207), timed on the host cores.
//
//   C2  mhp::reduce (mhp/algorithms/cpu_algorithms.hpp:102-140: per-rank
//       std::reduce, gather of one T to the root, root fold) + the 3-phase
//       scan of shp/algorithms/inclusive_scan.hpp:22-148 on rank blocks
//       (oracle.c orc_mhp_reduce_f32 / orc_mhp_scan_f32)
//   C3  sort (absent from the reference): per-rank std::sort, then pairwise
//       std::inplace_merge rounds (a CPU sample-sort stand-in)
//   C4  CSR gemv, the intended c += A*b of shp/algorithms/gemv.hpp:13-71,
//       rows split over ranks, the oracle's banded / random generators
//   C5  1-D 3-point and 2-D 5-point stencils (examples/mhp/stencil-1d.cpp,
//       halo cells copied from the neighbouring rank blocks each step)
//
// Every config: one untimed warm-up, then the median of `reps` timed runs
// (steady_clock).  One JSON line per config on stdout.
//   usage: cpu_bench <threads> <reps>
#include <omp.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <random>
#include <string>
#include <vector>

extern "C" {
#include "oracle.h"
}

static double median_seconds(int reps, const std::function<void()> &f) {
  f(); // warm-up
  std::vector<double> t;
  for (int r = 0; r < reps; r++) {
    const auto a = std::chrono::steady_clock::now();
    f();
    t.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count());
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

static void emit(const char *config, const char *workload, double units, const char *unit, double sec, int threads,
                 int reps, double check) {
  std::printf("{\"config\": \"%s\", \"workload\": \"%s\", \"value\": %.6g, \"unit\": \"%s\", \"median_s\": %.6g, "
              "\"threads\": %d, \"runs\": %d, \"check\": %.17g}\n",
              config, workload, units / sec, unit, sec, threads, reps, check);
  std::fflush(stdout);
}

int main(int argc, char **argv) {
  const int P = argc > 1 ? std::atoi(argv[1]) : 16;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 7;
  omp_set_num_threads(P);
  std::mt19937_64 g(1);

  // ---------------------------------------------------------------- C2
  {
    const std::size_t n = std::size_t(1) << 27;
    std::vector<float> x(n), out(n);
    std::uniform_real_distribution<float> u(0.f, 1.f);
    for (auto &v : x) v = u(g);
    double red = 0;
    const double s = median_seconds(reps, [&] {
      red = orc_mhp_reduce_f32(x.data(), n, P, 0.0, P);
      orc_mhp_scan_f32(x.data(), out.data(), n, P, P);
    });
    emit("C2", "mhp reduce + 3-phase inclusive_scan, 2^27 f32", (double)n, "elements/s", s, P, reps, red);
  }
  // ---------------------------------------------------------------- C3
  {
    const std::size_t n = std::size_t(1) << 24;
    std::vector<std::uint32_t> src(n), k(n);
    for (auto &v : src) v = (std::uint32_t)g();
    const double s = median_seconds(reps, [&] {
      k = src;
      const std::size_t blk = (n + P - 1) / P;
#pragma omp parallel for schedule(static, 1)
      for (int r = 0; r < P; r++) {
        const std::size_t lo = std::min(n, r * blk), hi = std::min(n, lo + blk);
        std::sort(k.begin() + lo, k.begin() + hi);
      }
      for (std::size_t w = blk; w < n; w *= 2) {
        const long pairs = (long)((n + 2 * w - 1) / (2 * w));
#pragma omp parallel for schedule(dynamic, 1)
        for (long p = 0; p < pairs; p++) {
          const std::size_t lo = p * 2 * w, mid = std::min(n, lo + w), hi = std::min(n, lo + 2 * w);
          std::inplace_merge(k.begin() + lo, k.begin() + mid, k.begin() + hi);
        }
      }
    });
    emit("C3", "sort 2^24 uint32 (per-rank std::sort + merge rounds)", (double)n, "keys/s", s, P, reps,
         std::is_sorted(k.begin(), k.end()) ? 1.0 : 0.0);
  }
  // ---------------------------------------------------------------- C4
  for (int kind = 0; kind < 2; kind++) {
    const std::size_t m = std::size_t(1) << 22;
    const std::size_t nnz = kind == 0 ? orc_csr_banded_nnz(m, m) : m * 10;
    std::vector<std::int32_t> rp(m + 1), ci(nnz);
    std::vector<float> va(nnz), xv(m), y(m);
    if (kind == 0)
      orc_csr_gen_banded_f32(0, m, m, 1, rp.data(), ci.data(), va.data());
    else
      orc_csr_gen_random_f32(0, m, m, 10, 1, rp.data(), ci.data(), va.data());
    std::uniform_real_distribution<float> u(0.f, 1.f);
    for (auto &v : xv) v = u(g);
    const double s = median_seconds(reps, [&] {
      const std::size_t blk = (m + P - 1) / P;
#pragma omp parallel for schedule(static, 1)
      for (int r = 0; r < P; r++)
        for (std::size_t i = std::min(m, r * blk); i < std::min(m, (r + 1) * blk); i++) {
          float acc = 0.f;
          for (std::int32_t e = rp[i]; e < rp[i + 1]; e++) acc += va[e] * xv[ci[e]];
          y[i] = acc;
        }
    });
    emit(kind == 0 ? "C4-banded" : "C4-random",
         kind == 0 ? "CSR gemv 2^22 rows banded (10 diagonals)" : "CSR gemv 2^22 rows random (10 columns/row)",
         (double)nnz, "nnz/s", s, P, reps, (double)y[m / 2]);
  }
  // ---------------------------------------------------------------- C5
  {
    const std::size_t n = std::size_t(1) << 27;
    const std::size_t blk = (n + P - 1) / P;
    // per-rank buffers [halo | block | halo], as the mhp distributed_vector
    std::vector<std::vector<float>> a(P), b(P);
    std::uniform_real_distribution<float> u(0.f, 1.f);
    for (int r = 0; r < P; r++) {
      a[r].resize(blk + 2);
      b[r].resize(blk + 2);
      for (auto &v : a[r]) v = u(g);
    }
    const double s = median_seconds(reps, [&] {
      for (int r = 0; r < P; r++) { // span_halo exchange (details/halo.hpp:336-387)
        if (r > 0) a[r][0] = a[r - 1][blk];
        if (r + 1 < P) a[r][blk + 1] = a[r + 1][1];
      }
#pragma omp parallel for schedule(static, 1)
      for (int r = 0; r < P; r++) {
        const float *p = a[r].data();
        float *q = b[r].data();
        const std::size_t lo = r == 0 ? 2 : 1, hi = r == P - 1 ? blk : blk + 1;
        for (std::size_t i = lo; i < hi; i++) q[i] = p[i - 1] + p[i] + p[i + 1];
      }
    });
    emit("C5-1d", "3-point stencil step, 2^27 cells", (double)n, "cells/s", s, P, reps, (double)b[0][5]);
  }
  {
    const std::size_t nx = 16384, ny = 8192; // 2^27 cells
    const std::size_t rows = (ny + P - 1) / P;
    std::vector<std::vector<float>> a(P), b(P);
    std::uniform_real_distribution<float> u(0.f, 1.f);
    for (int r = 0; r < P; r++) {
      a[r].resize((rows + 2) * nx);
      b[r].resize((rows + 2) * nx);
      for (auto &v : a[r]) v = u(g);
    }
    const double s = median_seconds(reps, [&] {
      for (int r = 0; r < P; r++) { // one halo row per side
        if (r > 0) std::copy_n(a[r - 1].begin() + rows * nx, nx, a[r].begin());
        if (r + 1 < P) std::copy_n(a[r + 1].begin() + nx, nx, a[r].begin() + (rows + 1) * nx);
      }
#pragma omp parallel for schedule(static, 1)
      for (int r = 0; r < P; r++) {
        const float *p = a[r].data();
        float *q = b[r].data();
        for (std::size_t y = (r == 0 ? 2 : 1); y < (r == P - 1 ? rows : rows + 1); y++)
          for (std::size_t x = 1; x + 1 < nx; x++) {
            const std::size_t i = y * nx + x;
            q[i] = p[i] + p[i - 1] + p[i + 1] + p[i - nx] + p[i + nx];
          }
      }
    });
    emit("C5-2d", "5-point stencil step, 8192 x 16384 cells", (double)(nx * ny), "cells/s", s, P, reps,
         (double)b[0][2 * nx + 7]);
  }
  return 0;
}
