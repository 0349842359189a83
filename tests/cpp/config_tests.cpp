// BASELINE configs at their configured GLOBAL sizes, in their distributed
// forms, through the C++ drop-in (include/dr/shp.hpp).  On a one-GPU box the
// P segments are duplicated on device 0 -- the reference's own method
// (test/gtest/shp/shp-tests.cpp:34-39); with --devices they sit on distinct
// GPUs.  Test infrastructure: links the CPU oracle (oracle/liboracle.so) as
// the checker only.
//
// C3 (default mode): shp::sort of a distributed_vector<uint32_t> of 2^31 keys
// over P = 8 segments (include/dr/shp/sort.hpp: local radix sorts, exact
// splitting, one piece copy per (source, destination), drhip_merge_runs of 8
// runs of 2^28 keys per destination, copy back).  Checks:
//   * every segment keeps ceil(n/P) keys (shp/distributed_vector.hpp:142);
//   * every key equals orc_radix_sort_u32_par of the same input (the std::less
//     order of uint32, pinned to qsort in tests/test_oracle.py): bit-exact.
// Keys: high word of splitmix64(seed + i), generated on the device by the
// kernel below and on the host by orc_fill_hash_u32 (same function).
//
// C2 (`c2` mode): the reference's C2 call sequence (shp-tests.cpp:34-39 +
// algorithms.cpp:61-149 at config size) -- shp::reduce(par_unseq, dv, 0) then
// shp::inclusive_scan(par_unseq, dv, out) on distributed_vector<float|int32_t>
// of 2^log2n elements over P segments.  With `out` the same size the pieces
// sit on distinct segments, so the scan runs the pinned-totals tile path
// (drhip_reduce_tiles per piece, totals folded on the device:
// algorithms.hpp inclusive_scan_impl); with --misaligned K `out` has n + P*K
// elements, its segment boundaries fall inside the input's segments, pieces
// share segments and the host-fold path runs.  Checks:
//   * f32: reduce rel <= 1e-5 vs the fp64 (compensated) sum; every scan
//     element rel <= 1e-5 vs the fp64 sequential prefix (orc_scan_exact_f32);
//   * i32: reduce == orc_shp_reduce_i32 and every element ==
//     orc_shp_scan_i32 over the zipped pieces (orc_zip_pieces): bit-exact.
// Input: u01 floats / integers in [0, 2^16) from splitmix64, generated on
// the device, copied back for the oracle.
//
//   config_tests [log2n=31] [P=8] [--greater] [--lambda] [--devices 0,1,...] [--threads T]
//   config_tests c2 [log2n=30] [P=8] [--dtype f32|i32] [--misaligned K] [--devices ...]
//   config_tests c4 [log2n=26] [P=8] [--kind banded|random] [--index i64|i32] [--devices ...]
// Prints one JSON line; exit 0 iff every check passed.
#include <dr/shp.hpp>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <type_traits>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

extern "C" {
#include "../../oracle/oracle.h"
}

__global__ void hash_keys(std::uint32_t *x, std::size_t n, std::uint64_t seed, std::uint64_t start) {
  const std::size_t i = blockIdx.x * (std::size_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  std::uint64_t z = seed + start + i + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  x[i] = (std::uint32_t)((z ^ (z >> 31)) >> 32);
}

struct args {
  int log2n = -1, P = 8, threads = 16;
  std::size_t misaligned = 0;
  bool greater = false; // C3: std::greater (descending)
  bool lambda = false;  // C3: the same order as a lambda (the general-comparator merge tier)
  std::string dtype = "f32";
  std::string kind = "banded", index = "i64"; // C4
  std::vector<int> devices;
};

// --devices wins; otherwise P segments duplicated on the first device
static bool open_devices(args &a, const std::string &dev_list) {
  if (!dev_list.empty()) {
    for (std::size_t p = 0; p < dev_list.size();) {
      std::size_t q = dev_list.find(',', p);
      if (q == std::string::npos) q = dev_list.size();
      a.devices.push_back(std::atoi(dev_list.substr(p, q - p).c_str()));
      p = q + 1;
    }
    a.P = (int)a.devices.size();
  } else {
    auto all = shp::get_numa_devices();
    if (all.empty()) return false;
    a.devices = shp::get_duplicated_devices({all[0]}, (std::size_t)a.P);
  }
  shp::init(a.devices);
  return true;
}

static std::string device_string(const args &a) {
  std::string s;
  for (std::size_t i = 0; i < a.devices.size(); i++) s += (i ? "," : "") + std::to_string(a.devices[i]);
  return s;
}

static int run_c3(const args &a) {
  const int P = a.P, threads = a.threads;
  const std::vector<int> &devices = a.devices;
  const std::uint64_t seed = 0xC3;
  const std::size_t n = std::size_t(1) << a.log2n;
  bool ok = true;
  {
    shp::distributed_vector<std::uint32_t> dv(n);
    std::size_t off = 0;
    for (auto &&s : dv.segments()) {
      const unsigned blocks = (unsigned)((s.size() + 255) / 256);
      hipLaunchKernelGGL(hash_keys, dim3(blocks), dim3(256), 0, shp::stream(s.rank()), s.data(), s.size(), seed,
                         (std::uint64_t)off);
      shp::detail::hip_check(hipGetLastError(), "hash_keys");
      off += s.size();
    }
    shp::sync_all();

    // the oracle's answer, computed while nothing else runs
    auto h0 = std::chrono::steady_clock::now();
    std::vector<std::uint32_t> ref(n);
    orc_fill_hash_u32(ref.data(), n, seed, 0, threads);
    if (orc_radix_sort_u32_par(ref.data(), n, threads) != 0) {
      std::printf("{\"ok\": false, \"error\": \"oracle sort out of memory\"}\n");
      return 1;
    }
    if (a.greater) std::reverse(ref.begin(), ref.end()); // std::greater: the ascending order reversed
    const double oracle_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - h0).count();

    // one sort of the real input, timed end to end (first call: scratch grown)
    auto sort_call = [&] {
      if (a.lambda && a.greater) shp::sort(shp::par_unseq, dv, [](std::uint32_t x, std::uint32_t y) { return x > y; });
      else if (a.lambda) shp::sort(shp::par_unseq, dv, [](std::uint32_t x, std::uint32_t y) { return x < y; });
      else if (a.greater) shp::sort(shp::par_unseq, dv, std::greater<>());
      else shp::sort(shp::par_unseq, dv);
    };
    auto t0 = std::chrono::steady_clock::now();
    sort_call();
    const double sort_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();

    // the same input again with the scratch warm: the distributed C3 step
    // time (regenerate, drain, sort); checked below
    off = 0;
    for (auto &&s : dv.segments()) {
      hipLaunchKernelGGL(hash_keys, dim3((unsigned)((s.size() + 255) / 256)), dim3(256), 0, shp::stream(s.rank()),
                         s.data(), s.size(), seed, (std::uint64_t)off);
      off += s.size();
    }
    shp::sync_all();
    t0 = std::chrono::steady_clock::now();
    sort_call();
    const double sort_ms_warm = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();

    const std::size_t seg = (n + (std::size_t)P - 1) / (std::size_t)P;
    std::size_t k = 0, base = 0, bad = 0, bad_sizes = 0;
    std::vector<std::uint32_t> host;
    std::string sizes;
    for (auto &&s : dv.segments()) {
      const std::size_t want = std::min(seg, n - base);
      if (s.size() != want) bad_sizes++;
      sizes += (k ? "," : "") + std::to_string(s.size());
      host.resize(s.size());
      shp::detail::check(drhip_memcpy_d2h((int)s.rank(), host.data(), s.data(), s.size() * 4), "d2h");
      shp::sync(s.rank());
      for (std::size_t i = 0; i < s.size(); i++) bad += host[i] != ref[base + i];
      base += s.size();
      k++;
    }
    ok = bad == 0 && bad_sizes == 0 && base == n;
    std::printf("{\"config\": \"C3\", \"order\": \"%s\", \"comparator\": \"%s\", \"keys\": %zu, \"segments\": %d, "
                "\"devices\": \"%s",
                a.greater ? "greater" : "less", a.lambda ? "lambda (merge tier)" : "std (radix)", n, P,
                device_string(a).c_str());
    std::printf("\", \"segment_sizes\": [%s], \"size_mismatches\": %zu, \"key_mismatches\": %zu, "
                "\"sort_ms_first_call\": %.3f, \"sort_ms\": %.3f, \"oracle_s\": %.2f, \"oracle_threads\": %d, \"ok\": %s}\n",
                sizes.c_str(), bad_sizes, bad, sort_ms, sort_ms_warm, oracle_s, threads, ok ? "true" : "false");
  }
  return ok ? 0 : 1;
}

// ------------------------------------------------------------------ C2
__device__ std::uint64_t mix64(std::uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
template <typename T> __global__ void gen_c2(T *x, std::size_t n, std::uint64_t start) {
  const std::size_t i = blockIdx.x * (std::size_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const std::uint64_t z = mix64(0xC2 + start + i);
  if constexpr (std::is_same_v<T, float>) x[i] = (float)(z >> 40) * (1.0f / 16777216.0f);
  else x[i] = (T)(z >> 48);
}

template <typename T> static void d2h_prefix(shp::distributed_vector<T> &dv, T *host, std::size_t count) {
  std::size_t off = 0;
  for (auto &&s : dv.segments()) {
    if (off >= count) break;
    const std::size_t m = std::min(s.size(), count - off);
    shp::detail::check(drhip_memcpy_d2h((int)s.rank(), host + off, s.data(), m * sizeof(T)), "d2h");
    shp::sync(s.rank());
    off += m;
  }
}

template <typename T> static int run_c2(const args &a) {
  const int P = a.P;
  const std::size_t n = std::size_t(1) << a.log2n, no = n + (std::size_t)P * a.misaligned;
  constexpr bool F32 = std::is_same_v<T, float>;

  // the zipped pieces of (dv, out) and the path inclusive_scan_impl takes:
  // the tile path iff pieces 0..P-2 sit on distinct input segments
  std::vector<std::size_t> lr(P), lo(P), pl(2 * P + 2);
  std::vector<int> prr(2 * P + 2), pro(2 * P + 2);
  const int nr = orc_dv_segments(n, P, lr.data()), nout = orc_dv_segments(no, P, lo.data());
  const int np = orc_zip_pieces(lr.data(), nr, lo.data(), nout, pl.data(), prr.data(), pro.data(), 2 * P + 2);
  bool distinct = true;
  for (int k = 0; k + 1 < np; k++)
    for (int j = 0; j < k; j++) distinct = distinct && prr[j] != prr[k];
  const char *path = np == 1 ? "single" : distinct ? "tiles_pinned_totals" : "host_fold";

  bool ok = true;
  double red_err = 0, scan_err[2] = {0, 0}, red_ms = 0, scan_ms[2] = {0, 0}, oracle_s = 0;
  std::size_t bad[2] = {0, 0}, bad_sizes = 0;
  bool red_exact = true;
  std::string sizes;
  {
    shp::distributed_vector<T> dv(n), out(no);
    std::size_t off = 0;
    for (auto &&s : dv.segments()) {
      hipLaunchKernelGGL(gen_c2<T>, dim3((unsigned)((s.size() + 255) / 256)), dim3(256), 0, shp::stream(s.rank()),
                         s.data(), s.size(), (std::uint64_t)off);
      shp::detail::hip_check(hipGetLastError(), "gen_c2");
      off += s.size();
    }
    shp::sync_all();
    const std::size_t seg = (n + (std::size_t)P - 1) / (std::size_t)P;
    std::size_t k = 0, base = 0;
    for (auto &&s : dv.segments()) {
      if (s.size() != std::min(seg, n - base)) bad_sizes++;
      sizes += (k++ ? "," : "") + std::to_string(s.size());
      base += s.size();
    }
    std::vector<T> x(n), got(n);
    d2h_prefix(dv, x.data(), n);

    // the oracle's answers
    auto h0 = std::chrono::steady_clock::now();
    std::vector<double> ref_f;
    std::vector<T> ref_i;
    double ref_red = 0;
    std::int32_t ref_red_i = 0;
    if constexpr (F32) {
      ref_red = orc_reduce_exact_f32(x.data(), n, 0.0, ORC_PLUS);
      ref_f.resize(n);
      orc_scan_exact_f32(x.data(), ref_f.data(), n, ORC_PLUS, 0, 0.0);
    } else {
      ref_red_i = orc_shp_reduce_i32(x.data(), lr.data(), nr, 0, ORC_PLUS);
      ref_i.resize(n);
      orc_shp_scan_i32(x.data(), ref_i.data(), pl.data(), np, ORC_PLUS, 0, 0);
    }
    oracle_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - h0).count();

    // the reference's call sequence, twice (first call grows the workspaces;
    // the output is cleared in between so the second scan must rewrite it all)
    for (int rep = 0; rep < 2; rep++) {
      for (auto &&s : out.segments())
        shp::detail::hip_check(hipMemsetAsync(s.data(), 0xff, s.size() * sizeof(T), shp::stream(s.rank())), "memset");
      shp::sync_all();
      auto t0 = std::chrono::steady_clock::now();
      const T red = shp::reduce(shp::par_unseq, dv, T(0));
      red_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      t0 = std::chrono::steady_clock::now();
      shp::inclusive_scan(shp::par_unseq, dv, out);
      scan_ms[rep] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if constexpr (F32) red_err = std::max(red_err, std::fabs((double)red - ref_red) / ref_red);
      else red_exact = red_exact && red == ref_red_i;
      d2h_prefix(out, got.data(), n);
      for (std::size_t i = 0; i < n; i++) {
        if constexpr (F32) {
          const double e = std::fabs((double)got[i] - ref_f[i]) / std::max(std::fabs(ref_f[i]), 1e-30);
          if (!(e <= 1e-5)) bad[rep]++;
          if (e > scan_err[rep] || e != e) scan_err[rep] = e;
        } else {
          bad[rep] += got[i] != ref_i[i];
        }
      }
    }
  }
  ok = bad_sizes == 0 && bad[0] == 0 && bad[1] == 0 && red_exact && red_err <= 1e-5;
  std::printf("{\"config\": \"C2\", \"dtype\": \"%s\", \"elements\": %zu, \"segments\": %d, \"devices\": \"%s\", "
              "\"out_elements\": %zu, \"pieces\": %d, \"path\": \"%s\", \"segment_sizes\": [%s], "
              "\"size_mismatches\": %zu, \"reduce_rel_err\": %.3g, \"reduce_exact\": %s, "
              "\"scan_mismatches\": [%zu, %zu], \"scan_max_rel_err\": [%.3g, %.3g], \"reduce_ms\": %.3f, "
              "\"scan_ms\": [%.3f, %.3f], \"oracle_s\": %.2f, \"ok\": %s}\n",
              F32 ? "f32" : "i32", n, P, device_string(a).c_str(), no, np, path, sizes.c_str(), bad_sizes, red_err,
              red_exact ? "true" : "false", bad[0], bad[1], scan_err[0], scan_err[1], red_ms, scan_ms[0], scan_ms[1],
              oracle_s, ok ? "true" : "false");
  return ok ? 0 : 1;
}

// ------------------------------------------------------------------ C4
// shp::gemv(c, a, b) through the drop-in (include/dr/shp/sparse.hpp: every
// row tile's window of b gathered by device-to-device copies of b's
// segments, then the tile SpMV) on a sparse_matrix<float, I> of 2^log2n x
// 2^log2n over P {P, 1} row tiles, I = std::size_t by default (the
// reference's sparse_matrix<T, I = std::size_t>, containers/
// sparse_matrix.hpp:126).  b ~ U[0,1) generated on the device, c starts at
// zero (gemv accumulates: gemv_example.cpp:25-27).  Checks c on windows of
// `W` rows around every row-tile edge (and both ends) plus `R` random
// windows, against the oracle's row-addressable generator + fp64 CSR rows:
// rel <= 1e-5 per row.
template <typename I> static int run_c4(const args &a, bool random_kind) {
  const int P = a.P;
  const std::size_t m = std::size_t(1) << a.log2n;
  constexpr std::size_t W = 4096;
  constexpr int R = 64;
  const int k = 10;
  const std::uint64_t seed = 1;
  bool ok = true;
  std::size_t bad = 0, rows_checked = 0;
  double max_err = 0, gemv_ms[2] = {0, 0}, gen_s = 0;
  std::size_t nnz = 0;
  {
    auto g0 = std::chrono::steady_clock::now();
    shp::sparse_matrix<float, I> A({m, m}, random_kind ? shp::csr_kind::random : shp::csr_kind::banded, k, seed);
    shp::distributed_vector<float> b(m), c(m);
    std::size_t off = 0;
    for (auto &&s : b.segments()) {
      hipLaunchKernelGGL(gen_c2<float>, dim3((unsigned)((s.size() + 255) / 256)), dim3(256), 0, shp::stream(s.rank()),
                         s.data(), s.size(), (std::uint64_t)off);
      shp::detail::hip_check(hipGetLastError(), "gen b");
      off += s.size();
    }
    shp::sync_all();
    gen_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - g0).count();
    nnz = A.size();
    // gemv twice: c = A b, then c = 2 A b (accumulation); the check uses the
    // second result against 2 * the fp64 rows
    for (int rep = 0; rep < 2; rep++) {
      auto t0 = std::chrono::steady_clock::now();
      shp::gemv(c, A, b);
      gemv_ms[rep] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    std::vector<float> hb(m), hc(m);
    d2h_prefix(b, hb.data(), m);
    d2h_prefix(c, hc.data(), m);
    // windows: both ends, every tile edge, R random
    const std::size_t tile_rows = (m + (std::size_t)P - 1) / (std::size_t)P;
    std::vector<std::size_t> starts{0, m - W};
    for (int t = 1; t < P; t++) starts.push_back(std::min(m - W, t * tile_rows - W / 2));
    std::uint64_t z = 0xC4;
    for (int r = 0; r < R; r++) {
      z = z * 6364136223846793005ull + 1442695040888963407ull;
      starts.push_back((std::size_t)((z >> 20) % (m - W)));
    }
    std::vector<std::int32_t> rp(W + 1), ci(W * 32);
    std::vector<float> va(W * 32), y0(W, 0.0f);
    std::vector<double> ref(W);
    for (std::size_t r0 : starts) {
      if (random_kind) orc_csr_gen_random_f32(r0, W, m, k, seed, rp.data(), ci.data(), va.data());
      else orc_csr_gen_banded_f32(r0, W, m, seed, rp.data(), ci.data(), va.data());
      orc_csr_spmv_f32_i32(W, rp.data(), ci.data(), va.data(), hb.data(), y0.data(), ref.data());
      for (std::size_t i = 0; i < W; i++) {
        const double want = 2.0 * ref[i];
        const double e = std::fabs((double)hc[r0 + i] - want) / std::max(std::fabs(want), 1e-30);
        if (!(e <= 1e-5)) bad++;
        if (e > max_err || e != e) max_err = e;
      }
      rows_checked += W;
    }
  }
  ok = bad == 0;
  std::printf("{\"config\": \"C4\", \"kind\": \"%s\", \"index_bytes\": %zu, \"rows\": %zu, \"nnz\": %zu, "
              "\"segments\": %d, \"devices\": \"%s\", \"rows_checked\": %zu, \"row_mismatches\": %zu, "
              "\"max_rel_err\": %.3g, \"gemv_ms\": [%.3f, %.3f], \"generate_s\": %.2f, \"ok\": %s}\n",
              random_kind ? "random" : "banded", sizeof(I), m, nnz, P, device_string(a).c_str(), rows_checked, bad,
              max_err, gemv_ms[0], gemv_ms[1], gen_s, ok ? "true" : "false");
  return ok ? 0 : 1;
}

int main(int argc, char **argv) {
  args a;
  std::string dev_list, mode = "c3";
  std::vector<std::string> pos;
  for (int i = 1; i < argc; i++) {
    std::string s = argv[i];
    if (s == "--devices" && i + 1 < argc) dev_list = argv[++i];
    else if (s == "--threads" && i + 1 < argc) a.threads = std::atoi(argv[++i]);
    else if (s == "--dtype" && i + 1 < argc) a.dtype = argv[++i];
    else if (s == "--misaligned" && i + 1 < argc) a.misaligned = std::strtoull(argv[++i], nullptr, 10);
    else if (s == "--greater") a.greater = true;
    else if (s == "--lambda") a.lambda = true;
    else if (s == "--kind" && i + 1 < argc) a.kind = argv[++i];
    else if (s == "--index" && i + 1 < argc) a.index = argv[++i];
    else if (s == "c2" || s == "c3" || s == "c4") mode = s;
    else pos.push_back(s);
  }
  a.log2n = mode == "c2" ? 30 : mode == "c4" ? 26 : 31;
  if (pos.size() > 0) a.log2n = std::atoi(pos[0].c_str());
  if (pos.size() > 1) a.P = std::atoi(pos[1].c_str());
  if (a.P < 1 || a.log2n < 1 || a.log2n > 34 || (mode == "c2" && a.dtype != "f32" && a.dtype != "i32")) {
    std::printf("{\"ok\": false, \"error\": \"bad arguments\"}\n");
    return 2;
  }
  if (!open_devices(a, dev_list)) {
    std::printf("{\"ok\": false, \"error\": \"no HIP device\"}\n");
    return 2;
  }
  int rc;
  try {
    if (mode == "c3") rc = run_c3(a);
    else if (mode == "c4")
      rc = a.index == "i32" ? run_c4<std::int32_t>(a, a.kind == "random") : run_c4<std::size_t>(a, a.kind == "random");
    else if (a.dtype == "f32") rc = run_c2<float>(a);
    else rc = run_c2<std::int32_t>(a);
  } catch (const std::exception &e) {
    std::printf("{\"ok\": false, \"error\": \"%s\"}\n", e.what());
    rc = 1;
  }
  shp::finalize();
  return rc;
}
