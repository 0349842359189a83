// dense_matrix for_each throughput: v = v + f(index) over a
// row-major fp32 dense_matrix on one device, HIP events on the segment
// stream.  Algorithmic bytes: 8 B per element (read + write).
//   dense_bench [log2 rows] [log2 cols] [reps]
#include <dr/shp.hpp>

#include <cmath>
#include <cstdio>
#include <new>
#include <cstdlib>

// a failed HIP call ends the benchmark with its error (no silent timings)
static void hchk(hipError_t e, const char *what) {
  if (e != hipSuccess) {
    std::fprintf(stderr, "dense_bench: %s: %s\n", what, hipGetErrorString(e));
    std::exit(3);
  }
}

int main(int argc, char **argv) {
  const int lr = argc > 1 ? std::atoi(argv[1]) : 15, lc = argc > 2 ? std::atoi(argv[2]) : 15;
  const int reps = argc > 3 ? std::atoi(argv[3]) : 10;
  auto devices = shp::get_numa_devices();
  if (devices.empty()) return 2;
  shp::init(std::vector<int>{devices[0]});
  const std::size_t m = std::size_t(1) << lr, n = std::size_t(1) << lc;
  shp::dense_matrix<float> a({m, n});
  auto body = [](auto &&e) {
    auto &&[idx, v] = e;
    v = v + float(idx[1] & 7);
  };
  shp::for_each(shp::par_unseq, a, body); // warm-up
  hipEvent_t e0, e1;
  hchk(hipEventCreate(&e0), "hipEventCreate");
  hchk(hipEventCreate(&e1), "hipEventCreate");
  hchk(hipEventRecord(e0, shp::stream(0)), "hipEventRecord");
  for (int r = 0; r < reps; r++) shp::for_each(shp::par_unseq, a, body);
  hchk(hipEventRecord(e1, shp::stream(0)), "hipEventRecord");
  hchk(hipEventSynchronize(e1), "hipEventSynchronize");
  float ms = 0;
  hchk(hipEventElapsedTime(&ms, e0, e1), "hipEventElapsedTime");
  ms /= reps;
  const double gbs = 8.0 * double(m * n) / (ms * 1e-3) / 1e9;
  // spot check: element (i, j) was incremented (reps + 1) times by j & 7
  const float got = a[{m - 1, n - 3}];
  const float want = float(reps + 1) * float((n - 3) & 7);
  // the same body over a distributed_vector of m*n floats (generic
  // for_each through the contiguous span accessor)
  shp::distributed_vector<float> dv(m * n);
  auto vbody = [](float &v) { v = v + 1.0f; };
  shp::for_each(shp::par_unseq, dv, vbody);
  hchk(hipEventRecord(e0, shp::stream(0)), "hipEventRecord");
  for (int r = 0; r < reps; r++) shp::for_each(shp::par_unseq, dv, vbody);
  hchk(hipEventRecord(e1, shp::stream(0)), "hipEventRecord");
  hchk(hipEventSynchronize(e1), "hipEventSynchronize");
  float vms = 0;
  hchk(hipEventElapsedTime(&vms, e0, e1), "hipEventElapsedTime");
  vms /= reps;
  const float vgot = dv[m * n - 5];
  std::printf("{\"op\": \"vector_for_each\", \"n\": %zu, \"ms\": %.4f, \"GBps\": %.1f, \"frac\": %.4f, \"check\": %s}\n",
              m * n, vms, 8.0 * double(m * n) / (vms * 1e-3) / 1e9, 8.0 * double(m * n) / (vms * 1e-3) / 1e9 / 8000.0,
              vgot == float(reps + 1) ? "true" : "false");
  // views: enumerate (write idx, 4 B/elem written + 0 read) and zip
  // (a = a + b: 12 B/elem) over distributed_vectors, generic kernel
  auto timeit = [&](auto &&fn) {
    fn();
    hchk(hipEventRecord(e0, shp::stream(0)), "hipEventRecord");
    for (int r = 0; r < reps; r++) fn();
    hchk(hipEventRecord(e1, shp::stream(0)), "hipEventRecord");
    hchk(hipEventSynchronize(e1), "hipEventSynchronize");
    float t = 0;
    hchk(hipEventElapsedTime(&t, e0, e1), "hipEventElapsedTime");
    return t / reps;
  };
  const std::size_t nz = m * n / 2;
  shp::distributed_vector<float> za(nz), zb(nz, 1.0f);
  const float ems = timeit([&] {
    shp::for_each(shp::par_unseq, shp::views::enumerate(za), [](auto &&t) {
      auto &&[idx, value] = t;
      value = float(idx & 1023);
    });
  });
  const float zms = timeit([&] {
    shp::for_each(shp::par_unseq, shp::views::zip(za, zb), [](auto &&t) {
      auto &&[x, y] = t;
      x = x + y;
    });
  });
  std::printf("{\"op\": \"enumerate_for_each\", \"n\": %zu, \"ms\": %.4f, \"GBps\": %.1f, \"frac\": %.4f}\n", nz, ems,
              4.0 * nz / (ems * 1e-3) / 1e9, 4.0 * nz / (ems * 1e-3) / 1e9 / 8000.0);
  std::printf("{\"op\": \"zip_for_each\", \"n\": %zu, \"ms\": %.4f, \"GBps\": %.1f, \"frac\": %.4f}\n", nz, zms,
              12.0 * nz / (zms * 1e-3) / 1e9, 12.0 * nz / (zms * 1e-3) / 1e9 / 8000.0);
  // generic reduce: the reference's dot composition reduce(zip | transform)
  // (examples/shp/dot_product.cpp:11-18; 8 B/pair) and a user-lambda op
  // (4 B/elem), both through the template reduce kernel
  zb.~distributed_vector();
  new (&zb) shp::distributed_vector<float>(nz, 0.5f);
  shp::fill(za, 0.25f);
  auto prod = shp::views::zip(za, zb) | lib::views::transform([](auto &&e) {
                auto &&[x, y] = e;
                return x * y;
              });
  float dot = 0;
  const float dms = timeit([&] { dot = shp::reduce(shp::par_unseq, prod, 0.0f, std::plus()); });
  float gsum = 0;
  const float gms = timeit([&] { gsum = shp::reduce(shp::par_unseq, za, 0.0f, [](float x, float y) { return x + y; }); });
  std::printf("{\"op\": \"reduce_zip_transform\", \"n\": %zu, \"ms\": %.4f, \"GBps\": %.1f, \"frac\": %.4f, "
              "\"check\": %s}\n", nz, dms, 8.0 * nz / (dms * 1e-3) / 1e9, 8.0 * nz / (dms * 1e-3) / 1e9 / 8000.0,
              std::fabs(dot - 0.125f * nz) <= 1e-4f * 0.125f * nz ? "true" : "false");
  std::printf("{\"op\": \"reduce_lambda_op\", \"n\": %zu, \"ms\": %.4f, \"GBps\": %.1f, \"frac\": %.4f, "
              "\"check\": %s}\n", nz, gms, 4.0 * nz / (gms * 1e-3) / 1e9, 4.0 * nz / (gms * 1e-3) / 1e9 / 8000.0,
              std::fabs(gsum - 0.25f * nz) <= 1e-4f * 0.25f * nz ? "true" : "false");
  // generic inclusive_scan with a user-lambda operator (template 3-kernel
  // reduce-then-scan: 12 B/elem moved, 8 B/elem algorithmic)
  const float sms = timeit([&] { shp::inclusive_scan(shp::par_unseq, za, zb, [](float x, float y) { return x + y; }); });
  const float slast = zb[nz - 1];
  std::printf("{\"op\": \"scan_lambda_op\", \"n\": %zu, \"ms\": %.4f, \"GBps\": %.1f, \"frac\": %.4f, "
              "\"check\": %s}\n", nz, sms, 8.0 * nz / (sms * 1e-3) / 1e9, 8.0 * nz / (sms * 1e-3) / 1e9 / 8000.0,
              std::fabs(slast - 0.25f * nz) <= 1e-3f * 0.25f * nz ? "true" : "false");
  std::printf("{\"op\": \"dense_for_each\", \"shape\": [%zu, %zu], \"ms\": %.4f, \"GBps\": %.1f, \"frac\": %.4f, "
              "\"check\": %s}\n",
              m, n, ms, gbs, gbs / 8000.0, got == want ? "true" : "false");
  shp::finalize();
  return got == want ? 0 : 1;
}
