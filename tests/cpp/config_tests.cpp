// BASELINE config C3 at its configured GLOBAL size, in its distributed form,
// through the C++ drop-in: shp::sort of a distributed_vector<uint32_t> of
// 2^31 keys over P = 8 segments (include/dr/shp/sort.hpp: local radix sorts,
// exact splitting, one piece copy per (source, destination), drhip_merge_runs
// of 8 runs of 2^28 keys per destination, copy back).  On a one-GPU box the 8
// segments are duplicated on device 0 -- the reference's own method
// (test/gtest/shp/shp-tests.cpp:34-39); with --devices they sit on distinct
// GPUs.
//
// Checks (test infrastructure: links the CPU oracle, oracle/liboracle.so):
//   * every segment keeps ceil(n/P) keys (shp/distributed_vector.hpp:142);
//   * every key equals orc_radix_sort_u32_par of the same input (the std::less
//     order of uint32, pinned to qsort in tests/test_oracle.py): bit-exact.
// Keys: high word of splitmix64(seed + i), generated on the device by the
// kernel below and on the host by orc_fill_hash_u32 (same function).
//
//   config_tests [log2n=31] [P=8] [--devices 0,1,...] [--threads T]
// Prints one JSON line; exit 0 iff every check passed.
#include <dr/shp.hpp>

#include <chrono>
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

int main(int argc, char **argv) {
  int log2n = 31, P = 8, threads = 16;
  std::string dev_list;
  std::vector<std::string> pos;
  for (int i = 1; i < argc; i++) {
    std::string a = argv[i];
    if (a == "--devices" && i + 1 < argc) dev_list = argv[++i];
    else if (a == "--threads" && i + 1 < argc) threads = std::atoi(argv[++i]);
    else pos.push_back(a);
  }
  if (pos.size() > 0) log2n = std::atoi(pos[0].c_str());
  if (pos.size() > 1) P = std::atoi(pos[1].c_str());
  const std::uint64_t seed = 0xC3;
  const std::size_t n = std::size_t(1) << log2n;

  std::vector<int> devices;
  if (!dev_list.empty()) {
    for (std::size_t p = 0; p < dev_list.size();) {
      std::size_t q = dev_list.find(',', p);
      if (q == std::string::npos) q = dev_list.size();
      devices.push_back(std::atoi(dev_list.substr(p, q - p).c_str()));
      p = q + 1;
    }
    P = (int)devices.size();
  } else {
    auto all = shp::get_numa_devices();
    if (all.empty()) {
      std::printf("{\"ok\": false, \"error\": \"no HIP device\"}\n");
      return 2;
    }
    devices = shp::get_duplicated_devices({all[0]}, (std::size_t)P);
  }
  shp::init(devices);
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
    const double oracle_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - h0).count();

    // one sort of the real input, timed end to end (first call: scratch grown)
    auto t0 = std::chrono::steady_clock::now();
    shp::sort(shp::par_unseq, dv);
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
    shp::sort(shp::par_unseq, dv);
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
    std::printf("{\"config\": \"C3\", \"keys\": %zu, \"segments\": %d, \"devices\": \"", n, P);
    for (std::size_t i = 0; i < devices.size(); i++) std::printf("%s%d", i ? "," : "", devices[i]);
    std::printf("\", \"segment_sizes\": [%s], \"size_mismatches\": %zu, \"key_mismatches\": %zu, "
                "\"sort_ms_first_call\": %.3f, \"sort_ms\": %.3f, \"oracle_s\": %.2f, \"oracle_threads\": %d, \"ok\": %s}\n",
                sizes.c_str(), bad_sizes, bad, sort_ms, sort_ms_warm, oracle_s, threads, ok ? "true" : "false");
  }
  shp::finalize();
  return ok ? 0 : 1;
}
