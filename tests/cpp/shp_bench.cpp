// The reference's own execution model, timed: ONE process driving P devices
// through the C++ drop-in (shp::init(devices), include/dr/shp/init.hpp:40-50
// in the reference), one segment per device, every algorithm call blocking
// as the reference's do.  bench.py runs it on rank 0 at N > 1 so that the
// driver's multi-GPU box exercises the single-process peer paths:
//   * shp::reduce (per-device partials, host fold in segment order,
//     reduce.hpp:40-88);
//   * shp::inclusive_scan (P > 1: piece totals, exclusive prefix, carry-in
//     single-pass scans on every device, inclusive_scan.hpp:22-148);
//   * shp::sort (local radix sorts, exact splitting, piece copies across
//     devices over xGMI, merge of the received runs; sort.hpp).
// Weak scaling: 2^log2n floats and 2^sort_log2n uint32 keys PER DEVICE.
//
//   shp_bench --devices 0,1,.. [--log2n 30] [--sort-log2n 28] [--reps 5]
// Prints one JSON line (wall-clock median per call, elements/s, checks).
#include <dr/shp.hpp>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

__device__ std::uint64_t mix64(std::uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__global__ void fill_u01(float *x, std::size_t n, std::uint64_t start) {
  const std::size_t i = blockIdx.x * (std::size_t)blockDim.x + threadIdx.x;
  if (i < n) x[i] = (float)(mix64(start + i) >> 40) * (1.0f / 16777216.0f);
}
__global__ void fill_keys(std::uint32_t *x, std::size_t n, std::uint64_t start) {
  const std::size_t i = blockIdx.x * (std::size_t)blockDim.x + threadIdx.x;
  if (i < n) x[i] = (std::uint32_t)(mix64(0xC3 + start + i) >> 32);
}

// Independent fp64 checker kernels (not the product's reduce / scan): the
// fp64 sum of every B-element chunk of a segment, one plain block per chunk,
// and the chunk-end elements of the scanned output.
__global__ void chunk_sums_f64(const float *x, std::size_t n, std::size_t B, double *out) {
  __shared__ double s[256];
  const std::size_t c = blockIdx.x, b = c * B, e = b + B < n ? b + B : n;
  double acc = 0;
  for (std::size_t i = b + threadIdx.x; i < e; i += blockDim.x) acc += (double)x[i];
  s[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) s[threadIdx.x] += s[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[c] = s[0];
}
__global__ void chunk_ends(const float *y, std::size_t n, std::size_t B, std::size_t nch, float *out) {
  const std::size_t c = blockIdx.x * (std::size_t)blockDim.x + threadIdx.x;
  if (c < nch) out[c] = y[(c + 1) * B < n ? (c + 1) * B - 1 : n - 1];
}

template <typename T, typename K> void fill_segments(shp::distributed_vector<T> &dv, K kernel, std::uint64_t salt) {
  std::size_t off = 0;
  for (auto &&s : dv.segments()) {
    hipLaunchKernelGGL(kernel, dim3((unsigned)((s.size() + 255) / 256)), dim3(256), 0, shp::stream(s.rank()),
                       s.data(), s.size(), (std::uint64_t)off + salt);
    shp::detail::hip_check(hipGetLastError(), "fill");
    off += s.size();
  }
  shp::sync_all();
}

template <typename F> double median_ms(int reps, F &&f) {
  std::vector<double> t;
  for (int r = 0; r < reps; r++) t.push_back(f());
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

} // namespace

// Per-call overhead of the blocking C++ drop-in on ONE device: a blocking
// shp::reduce on a tiny vector (pure overhead), its pieces (drhip_reduce +
// drhip_sync, drhip_sync of an idle stream, the kernel alone by events), and
// a 2^27 reduce (the per-GPU share of strong-scaled C2 at 8 GPUs) wall vs
// kernel.  Medians of 200 (tiny) / 20 calls, microseconds.
static void overhead(int dev) {
  shp::init(std::vector<int>{dev});
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  auto us_of = [](auto &&f, int reps) {
    std::vector<double> t;
    for (int r = 0; r < reps; r++) {
      auto t0 = std::chrono::steady_clock::now();
      f();
      t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    return t;
  };
  double o_red, o_abi, o_sync, k_small, w27, k27;
  {
    shp::distributed_vector<float> x(1024);
    fill_segments(x, fill_u01, 0);
    float r = 0;
    for (int i = 0; i < 20; i++) r += shp::reduce(shp::par_unseq, x, 0.0f, std::plus<>());
    o_red = med(us_of([&] { r += shp::reduce(shp::par_unseq, x, 0.0f, std::plus<>()); }, 200));
    double *part = nullptr;
    shp::detail::check(drhip_host_alloc(sizeof(double), (void **)&part), "host alloc");
    auto seg = *x.segments().begin();
    o_abi = med(us_of([&] {
      shp::detail::check(drhip_reduce(0, DRHIP_F32, DRHIP_PLUS, seg.data(), seg.size(), part), "reduce");
      shp::detail::check(drhip_sync(0), "sync");
    }, 200));
    o_sync = med(us_of([&] { shp::detail::check(drhip_sync(0), "sync"); }, 200));
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    std::vector<double> ks;
    for (int i = 0; i < 50; i++) {
      (void)hipEventRecord(e0, shp::stream(0));
      shp::detail::check(drhip_reduce(0, DRHIP_F32, DRHIP_PLUS, seg.data(), seg.size(), part), "reduce");
      (void)hipEventRecord(e1, shp::stream(0));
      shp::sync(0);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      ks.push_back(ms * 1e3);
    }
    k_small = med(ks);
    shp::distributed_vector<float> y(std::size_t(1) << 27);
    fill_segments(y, fill_u01, 7);
    w27 = med(us_of([&] { r += shp::reduce(shp::par_unseq, y, 0.0f, std::plus<>()); }, 20));
    auto ys = *y.segments().begin();
    ks.clear();
    for (int i = 0; i < 20; i++) {
      (void)hipEventRecord(e0, shp::stream(0));
      shp::detail::check(drhip_reduce(0, DRHIP_F32, DRHIP_PLUS, ys.data(), ys.size(), part), "reduce");
      (void)hipEventRecord(e1, shp::stream(0));
      shp::sync(0);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      ks.push_back(ms * 1e3);
    }
    k27 = med(ks);
    (void)drhip_host_free(part);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (r < 0) std::printf("# %f\n", r);
  }
  // The allocator's price: a distributed_vector<float>(2^27)
  // created and destroyed in a loop (construction = allocation + the zero
  // fill of distributed_vector.hpp:153, blocking; destruction = drhip_free),
  // and the same while a 2^27 reduce is queued on the segment's stream (a
  // device-synchronising free waits for it)
  double cd_us, cd_busy_us;
  {
    const std::size_t n27 = std::size_t(1) << 27;
    for (int i = 0; i < 3; i++) shp::distributed_vector<float> v(n27);
    cd_us = med(us_of([&] { shp::distributed_vector<float> v(n27); }, 30));
    shp::distributed_vector<float> y(n27);
    fill_segments(y, fill_u01, 9);
    auto ys = *y.segments().begin();
    double *part = nullptr;
    shp::detail::check(drhip_host_alloc(sizeof(double), (void **)&part), "host alloc");
    cd_busy_us = med(us_of([&] {
      shp::detail::check(drhip_reduce(0, DRHIP_F32, DRHIP_PLUS, ys.data(), ys.size(), part), "reduce");
      { shp::distributed_vector<float> v(n27); }
      shp::sync(0);
    }, 30));
    (void)drhip_host_free(part);
  }
  const char *al = std::getenv("DRHIP_ALLOC");
  std::printf("{\"op\": \"alloc_price\", \"allocator\": \"%s\", \"create_destroy_2p27_f32_us\": %.1f, "
              "\"create_destroy_behind_2p27_reduce_us\": %.1f, \"reduce_2p27_kernel_us\": %.1f}\n",
              al ? al : "hipmalloc", cd_us, cd_busy_us, k27);
  const char *sm = std::getenv("DRHIP_SYNC");
  std::printf("{\"op\": \"shp_call_overhead\", \"sync_mode\": \"%s\", \"reduce_1k_us\": %.2f, "
              "\"abi_reduce_plus_sync_1k_us\": %.2f, \"sync_idle_us\": %.2f, \"kernel_1k_us\": %.2f, "
              "\"reduce_2p27_wall_us\": %.2f, \"reduce_2p27_kernel_us\": %.2f, "
              "\"blocking_overhead_2p27_us\": %.2f}\n",
              sm ? sm : "spin", o_red, o_abi, o_sync, k_small, w27, k27, w27 - k27);
  shp::finalize();
}

int main(int argc, char **argv) {
  for (int i = 1; i < argc; i++)
    if (!std::strcmp(argv[i], "--overhead")) {
      overhead(i + 1 < argc ? std::atoi(argv[i + 1]) : 0);
      return 0;
    }
  int log2n = 30, sort_log2n = 28, reps = 5;
  std::string dev_list = "0";
  for (int i = 1; i + 1 < argc; i++) {
    std::string a = argv[i];
    if (a == "--devices") dev_list = argv[++i];
    else if (a == "--log2n") log2n = std::atoi(argv[++i]);
    else if (a == "--sort-log2n") sort_log2n = std::atoi(argv[++i]);
    else if (a == "--reps") reps = std::atoi(argv[++i]);
  }
  std::vector<int> devices;
  for (std::size_t p = 0; p < dev_list.size();) {
    std::size_t q = dev_list.find(',', p);
    if (q == std::string::npos) q = dev_list.size();
    devices.push_back(std::atoi(dev_list.substr(p, q - p).c_str()));
    p = q + 1;
  }
  shp::init(devices);
  const std::size_t P = devices.size();
  const std::size_t n = P << log2n, ns = P << sort_log2n;
  bool ok = true;
  double red_ms, scan_ms, sort_ms, red_err, scan_err, red_kernel_ms = -1;
  std::size_t sort_bad = 0;
  {
    shp::distributed_vector<float> x(n), y(n);
    fill_segments(x, fill_u01, 0);
    float red = 0;
    shp::reduce(shp::par_unseq, x, 0.0f, std::plus<>()); // warm-up (pinned partials)
    red_ms = median_ms(reps, [&] {
      auto t0 = std::chrono::steady_clock::now();
      red = shp::reduce(shp::par_unseq, x, 0.0f, std::plus<>());
      return ms_since(t0);
    });
    // the same reduce's kernel alone (HIP events on segment 0's stream around
    // the C-ABI launch), so the line separates blocking overhead from kernel
    // time at 2^30
    if (P == 1) {
      shp::detail::pinned<double> part(1);
      hipEvent_t e0, e1;
      (void)hipEventCreate(&e0);
      (void)hipEventCreate(&e1);
      auto seg = *x.segments().begin();
      red_kernel_ms = median_ms(reps, [&] {
        (void)hipEventRecord(e0, shp::stream(0));
        shp::detail::check(drhip_reduce(0, DRHIP_F32, DRHIP_PLUS, seg.data(), seg.size(), &part[0]), "reduce");
        (void)hipEventRecord(e1, shp::stream(0));
        shp::sync(0);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        return (double)ms;
      });
      (void)hipEventDestroy(e0);
      (void)hipEventDestroy(e1);
    }
    shp::inclusive_scan(shp::par_unseq, x, y); // warm-up (workspaces)
    scan_ms = median_ms(reps, [&] {
      auto t0 = std::chrono::steady_clock::now();
      shp::inclusive_scan(shp::par_unseq, x, y);
      return ms_since(t0);
    });
    // checks against an independent fp64 reference (the checker kernels
    // above, not the product's reduce / scan): the fp64 sum of every 2^16-
    // element chunk of every device, prefix-summed on the host in segment
    // order; the reduce vs the fp64 total, and the scan's element at the end
    // of EVERY chunk (2^14 per 2^30 elements, carries across devices
    // included) vs the fp64 prefix there -- rel <= 1e-5
    constexpr std::size_t B = std::size_t(1) << 16;
    double run = 0;
    red_err = 0;
    scan_err = 0;
    auto xsegs = x.segments();
    auto ysegs = y.segments();
    for (std::size_t k = 0; k < xsegs.size(); k++) {
      auto &&xs = xsegs[k];
      auto &&ys = ysegs[k];
      const std::size_t m = xs.size(), nch = (m + B - 1) / B;
      double *cs = nullptr;
      float *ce = nullptr;
      shp::detail::check(drhip_malloc((int)xs.rank(), nch * sizeof(double), (void **)&cs), "malloc");
      shp::detail::check(drhip_malloc((int)xs.rank(), nch * sizeof(float), (void **)&ce), "malloc");
      hipLaunchKernelGGL(chunk_sums_f64, dim3((unsigned)nch), dim3(256), 0, shp::stream(xs.rank()), xs.data(), m, B, cs);
      hipLaunchKernelGGL(chunk_ends, dim3((unsigned)((nch + 255) / 256)), dim3(256), 0, shp::stream(xs.rank()),
                         ys.data(), m, B, nch, ce);
      std::vector<double> hcs(nch);
      std::vector<float> hce(nch);
      shp::detail::check(drhip_memcpy_d2h((int)xs.rank(), hcs.data(), cs, nch * sizeof(double)), "d2h");
      shp::detail::check(drhip_memcpy_d2h((int)xs.rank(), hce.data(), ce, nch * sizeof(float)), "d2h");
      shp::sync(xs.rank());
      for (std::size_t c = 0; c < nch; c++) {
        run += hcs[c];
        scan_err = std::max(scan_err, std::fabs((double)hce[c] - run) / std::fabs(run));
      }
      shp::detail::check(drhip_free((int)xs.rank(), cs), "free");
      shp::detail::check(drhip_free((int)xs.rank(), ce), "free");
    }
    red_err = std::fabs((double)red - run) / std::fabs(run);
    ok = ok && red_err <= 1e-5 && scan_err <= 1e-5;
  }
  {
    shp::distributed_vector<std::uint32_t> k(ns);
    fill_segments(k, fill_keys, 0);
    shp::sort(shp::par_unseq, k); // warm-up (scratch)
    sort_ms = median_ms(reps, [&] {
      fill_segments(k, fill_keys, 0);
      auto t0 = std::chrono::steady_clock::now();
      shp::sort(shp::par_unseq, k);
      return ms_since(t0);
    });
    // check: each device's first and last 2^20 keys ascending, ordered across
    // device boundaries, every segment keeps ceil(ns/P) keys
    std::uint32_t prev_last = 0;
    std::size_t idx = 0;
    for (auto &&s : k.segments()) {
      if (s.size() != (ns + P - 1) / P) sort_bad++;
      const std::size_t m = std::min<std::size_t>(s.size(), std::size_t(1) << 20);
      std::vector<std::uint32_t> a(m), b(m);
      shp::detail::check(drhip_memcpy_d2h((int)s.rank(), a.data(), s.data(), m * 4), "d2h");
      shp::detail::check(drhip_memcpy_d2h((int)s.rank(), b.data(), s.data() + (s.size() - m), m * 4), "d2h");
      shp::sync(s.rank());
      if (idx && a[0] < prev_last) sort_bad++;
      for (std::size_t i = 1; i < m; i++) sort_bad += (a[i] < a[i - 1]) + (b[i] < b[i - 1]);
      prev_last = b[m - 1];
      idx++;
    }
    ok = ok && sort_bad == 0;
  }
  // the general-comparator tier (dr/shp/merge_sort.hpp): the same keys under
  // a lambda ordering on their high 24 bits, which the radix path does not
  // take (a stable merge sort in this TU); checked by the comparator on each
  // device's first and last 2^20 keys and across device boundaries
  double sort_cmp_ms;
  std::size_t sort_cmp_bad = 0;
  {
    auto cmp = [](std::uint32_t a, std::uint32_t b) { return (a >> 8) < (b >> 8); };
    shp::distributed_vector<std::uint32_t> k(ns);
    fill_segments(k, fill_keys, 0);
    shp::sort(shp::par_unseq, k, cmp); // warm-up (scratch)
    sort_cmp_ms = median_ms(reps, [&] {
      fill_segments(k, fill_keys, 0);
      auto t0 = std::chrono::steady_clock::now();
      shp::sort(shp::par_unseq, k, cmp);
      return ms_since(t0);
    });
    std::uint32_t prev_last = 0;
    std::size_t idx = 0;
    for (auto &&s : k.segments()) {
      const std::size_t m = std::min<std::size_t>(s.size(), std::size_t(1) << 20);
      std::vector<std::uint32_t> a(m), b(m);
      shp::detail::check(drhip_memcpy_d2h((int)s.rank(), a.data(), s.data(), m * 4), "d2h");
      shp::detail::check(drhip_memcpy_d2h((int)s.rank(), b.data(), s.data() + (s.size() - m), m * 4), "d2h");
      shp::sync(s.rank());
      if (idx && cmp(a[0], prev_last)) sort_cmp_bad++;
      for (std::size_t i = 1; i < m; i++) sort_cmp_bad += cmp(a[i], a[i - 1]) + cmp(b[i], b[i - 1]);
      prev_last = b[m - 1];
      idx++;
    }
    ok = ok && sort_cmp_bad == 0;
  }
  std::printf("{\"op\": \"shp_one_process\", \"devices\": \"%s\", \"segments\": %zu, "
              "\"model\": \"one process, shp::init(devices), one segment per device, blocking C++ calls\", "
              "\"reduce\": {\"elements\": %zu, \"ms\": %.4f, \"elements_per_s\": %.6g, \"kernel_ms\": %.4f}, "
              "\"inclusive_scan\": {\"elements\": %zu, \"ms\": %.4f, \"elements_per_s\": %.6g}, "
              "\"sort\": {\"keys\": %zu, \"ms\": %.4f, \"keys_per_s\": %.6g}, "
              "\"sort_lambda_cmp\": {\"keys\": %zu, \"ms\": %.4f, \"keys_per_s\": %.6g, \"bad\": %zu, "
              "\"path\": \"stable merge sort (dr/shp/merge_sort.hpp), comparator (a >> 8) < (b >> 8)\"}, "
              "\"check\": {\"reduce_vs_fp64_rel\": %.3g, \"scan_chunk_ends_vs_fp64_rel\": %.3g, \"sort_bad\": %zu, "
              "\"ref\": \"independent fp64 chunk sums (2^16-element chunks), every chunk end\", "
              "\"ok\": %s}, \"timing\": \"wall-clock median of %d blocking calls\"}\n",
              dev_list.c_str(), P, n, red_ms, n / (red_ms * 1e-3), red_kernel_ms, n, scan_ms, n / (scan_ms * 1e-3), ns, sort_ms,
              ns / (sort_ms * 1e-3), ns, sort_cmp_ms, ns / (sort_cmp_ms * 1e-3), sort_cmp_bad, red_err, scan_err,
              sort_bad, ok ? "true" : "false", reps);
  shp::finalize();
  return ok ? 0 : 1;
}
