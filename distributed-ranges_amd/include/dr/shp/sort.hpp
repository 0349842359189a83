// dr/shp/sort.hpp -- shp::sort over a distributed range.
//
// The reference has no sort.  Semantics are
// std::ranges::sort: ascending under std::less, in place, the result keeps
// the range's segmentation.  Algorithm (single process, P segments):
//   1. every segment sorts locally (drhip_sort, LSD radix, in parallel) and
//      takes regular samples (drhip_sort_sample);
//   2. exact splitting (csrc/split.hip): from the samples, a value bracket
//      per segment boundary g_k = sum of the sizes of segments < k and each
//      segment's slice of sorted keys that holds it; from those slices the
//      key v_k of global rank g_k, with keys equal to v_k split in segment
//      order, so every destination gets exactly its segment's size -- two
//      small host exchanges instead of a device round trip per bisection
//      step (the same code dr_dist.exact_splits runs over two allgathers);
//   3. every (source, destination) piece moves with one device-to-device
//      copy (xGMI peer copy across GPUs) into a per-destination buffer;
//   4. every destination merges its P sorted runs (drhip_merge_runs) and
//      copies them back into its segment.
// All device scratch comes from the cached per-segment pool.  With P == 1
// only step 1's sort runs.
#pragma once

#include <cstring>
#include <functional>
#include <map>

#include "algorithms.hpp"
#include "merge_sort.hpp"
#include "../details/split_plan.hpp"

namespace shp {

namespace detail {

template <typename T> struct key_bits;
template <> struct key_bits<std::uint32_t> {
  using U = std::uint32_t;
  static U in(std::uint32_t x) { return x; }
  static std::uint32_t out(U u) { return u; }
};
template <> struct key_bits<std::int32_t> {
  using U = std::uint32_t;
  static U in(std::int32_t x) { return static_cast<U>(x) ^ 0x80000000u; }
  static std::int32_t out(U u) { return static_cast<std::int32_t>(u ^ 0x80000000u); }
};
template <> struct key_bits<float> {
  using U = std::uint32_t;
  static U in(float x) {
    U u;
    std::memcpy(&u, &x, 4);
    return u ^ ((u & 0x80000000u) ? 0xFFFFFFFFu : 0x80000000u);
  }
  static float out(U u) {
    u ^= (u & 0x80000000u) ? 0x80000000u : 0xFFFFFFFFu;
    float x;
    std::memcpy(&x, &u, 4);
    return x;
  }
};
template <> struct key_bits<std::uint64_t> {
  using U = std::uint64_t;
  static U in(std::uint64_t x) { return x; }
  static std::uint64_t out(U u) { return u; }
};
template <> struct key_bits<std::int64_t> {
  using U = std::uint64_t;
  static U in(std::int64_t x) { return static_cast<U>(x) ^ 0x8000000000000000ull; }
  static std::int64_t out(U u) { return static_cast<std::int64_t>(u ^ 0x8000000000000000ull); }
};
template <> struct key_bits<double> {
  using U = std::uint64_t;
  static U in(double x) {
    U u;
    std::memcpy(&u, &x, 8);
    return u ^ ((u & 0x8000000000000000ull) ? ~0ull : 0x8000000000000000ull);
  }
  static double out(U u) {
    u ^= (u & 0x8000000000000000ull) ? 0x8000000000000000ull : ~0ull;
    double x;
    std::memcpy(&x, &u, 8);
    return x;
  }
};

// Per-segment scratch of one sort call, carved from the cached per-rank
// device scratch (runtime.hpp device_scratch: grown once, reused by later
// calls, released by finalize) -- the sort allocates nothing per call once
// warm.  Layout per segment: [radix workspace | n-key exchange buffer |
// merge workspace | regular samples].  Segments that share a rank (a
// distributed_span may list several segments of one rank) get disjoint
// slices of that rank's ONE scratch block, sized for all of them.
struct sort_scratch {
  void *ws = nullptr, *buf = nullptr, *mws = nullptr, *smp = nullptr;
  std::size_t wsb = 0, mwsb = 0, bytes = 0;
};

inline std::size_t align_up(std::size_t x) { return (x + 255) & ~std::size_t(255); }

template <typename T>
sort_scratch size_sort_scratch(std::size_t rank, std::size_t n, std::size_t P, std::size_t nsamples) {
  const int r = static_cast<int>(rank);
  sort_scratch sc;
  check(drhip_sort_workspace(r, dtype_code<T>(), n, &sc.wsb), "drhip_sort_workspace");
  if (P > 1) check(drhip_merge_workspace(r, dtype_code<T>(), n, static_cast<int>(P), &sc.mwsb), "drhip_merge_workspace");
  const std::size_t bufb = P > 1 ? align_up(n * sizeof(T)) : 0;
  const std::size_t smpb = P > 1 ? align_up(nsamples * sizeof(T)) : 0;
  sc.bytes = align_up(sc.wsb) + bufb + align_up(sc.mwsb) + smpb;
  return sc;
}

template <typename T> void carve_sort_scratch(sort_scratch &sc, char *base, std::size_t n, std::size_t P) {
  const std::size_t bufb = P > 1 ? align_up(n * sizeof(T)) : 0;
  sc.ws = base;
  sc.buf = base + align_up(sc.wsb);
  sc.mws = base + align_up(sc.wsb) + bufb;
  sc.smp = base + align_up(sc.wsb) + bufb + align_up(sc.mwsb);
}

// Regular samples per segment for the exact splitting (split.hip): a stride
// of ceil(n / kSortSamples) keys keeps every boundary's bracket to a few
// strides of keys per segment.
constexpr std::size_t kSortSamples = std::size_t(1) << 16;

} // namespace detail

namespace detail {
template <typename T, typename Comp> void sort_general(auto &segs, Comp comp);
}

// std::ranges::sort(r): ascending under std::less.  int32/uint32/int64/
// uint64/float/double keys take the LSD radix path of libdrhip below; any
// other trivially-copyable T the general merge tier (merge_sort.hpp).
template <typename ExecutionPolicy, typename R>
  requires lib::distributed_contiguous_range<R>
void sort(ExecutionPolicy &&, R &&r) {
  using T = std::remove_cv_t<std::ranges::range_value_t<R>>;
  auto segs = lib::ranges::segments(r);
  if constexpr (!detail::abi_type<T>) {
    detail::sort_general<T>(segs, std::less<>{});
    return;
  } else {
  using KB = detail::key_bits<T>;
  std::vector<device_span<T>> parts;
  for (auto &s : segs)
    if (s.size()) parts.push_back(s);
  const std::size_t P = parts.size();
  if (P == 0) return;
  std::vector<std::uint64_t> n(P), stride(P), ns(P);
  for (std::size_t k = 0; k < P; k++) {
    n[k] = parts[k].size();
    stride[k] = std::max<std::uint64_t>(1, (n[k] + detail::kSortSamples - 1) / detail::kSortSamples);
    ns[k] = (n[k] + stride[k] - 1) / stride[k];
  }
  std::vector<detail::sort_scratch> sc(P);
  {
    std::map<std::size_t, std::size_t> rank_bytes; // one scratch block per rank, carved per segment
    for (std::size_t k = 0; k < P; k++) {
      sc[k] = detail::size_sort_scratch<T>(parts[k].rank(), n[k], P, ns[k]);
      rank_bytes[parts[k].rank()] += sc[k].bytes;
    }
    std::map<std::size_t, char *> rank_next;
    for (auto &[rk, b] : rank_bytes) rank_next[rk] = static_cast<char *>(detail::device_scratch().get(rk, b));
    for (std::size_t k = 0; k < P; k++) {
      char *&next = rank_next[parts[k].rank()];
      detail::carve_sort_scratch<T>(sc[k], next, n[k], P);
      next += sc[k].bytes;
    }
  }

  // 1. local sorts (every segment in flight), then the regular samples
  for (std::size_t k = 0; k < P; k++) {
    const int rk = static_cast<int>(parts[k].rank());
    if (n[k] > 1)
      detail::check(drhip_sort(rk, detail::dtype_code<T>(), parts[k].data(), n[k], sc[k].ws, sc[k].wsb), "drhip_sort");
    if (P > 1)
      detail::check(drhip_sort_sample(rk, detail::dtype_code<T>(), parts[k].data(), n[k], stride[k], sc[k].smp),
                    "drhip_sort_sample");
  }
  if (P == 1) {
    sync(parts[0].rank());
    return;
  }
  std::size_t tot_smp = 0;
  for (auto v : ns) tot_smp += v;
  detail::pinned<T> hs(tot_smp);
  for (std::size_t k = 0, off = 0; k < P; off += ns[k], k++)
    detail::check(drhip_memcpy_d2h(static_cast<int>(parts[k].rank()), hs.data() + off, sc[k].smp, ns[k] * sizeof(T)),
                  "sort samples d2h");
  for (std::size_t k = 0; k < P; k++) sync(parts[k].rank());

  // 2. exact splitting at the segment boundaries (csrc/split.hip): value
  //    brackets from the samples, then each boundary key on the slices of
  //    every sorted segment that hold its bracket
  const std::size_t nb = P - 1;
  std::vector<std::uint64_t> g(nb), lo(nb), hi(nb), win(2 * P * nb), split(P * (nb + 1));
  for (std::size_t k = 0, acc = 0; k < nb; k++) g[k] = acc += n[k];
  {
    std::vector<std::uint64_t> bits(tot_smp);
    for (std::size_t i = 0; i < tot_smp; i++) bits[i] = static_cast<std::uint64_t>(KB::in(hs[i]));
    detail::check(drhip_split_windows(static_cast<int>(P), n.data(), stride.data(), ns.data(), bits.data(),
                                      static_cast<int>(nb), g.data(), lo.data(), hi.data(), win.data()),
                  "drhip_split_windows");
  }
  std::size_t tot_win = 0;
  for (std::size_t i = 0; i < P * nb; i++) tot_win += win[2 * i + 1] - win[2 * i];
  {
    detail::pinned<T> hw(tot_win);
    std::size_t off = 0;
    for (std::size_t s = 0; s < P; s++)
      for (std::size_t k = 0; k < nb; k++) {
        const std::size_t a = win[2 * (s * nb + k)], b = win[2 * (s * nb + k) + 1];
        if (b > a)
          detail::check(drhip_memcpy_d2h(static_cast<int>(parts[s].rank()), hw.data() + off, parts[s].data() + a,
                                         (b - a) * sizeof(T)),
                        "sort slices d2h");
        off += b - a;
      }
    for (std::size_t s = 0; s < P; s++) sync(parts[s].rank());
    std::vector<std::uint64_t> wbits(tot_win);
    for (std::size_t i = 0; i < tot_win; i++) wbits[i] = static_cast<std::uint64_t>(KB::in(hw[i]));
    detail::check(drhip_split_exact(static_cast<int>(P), n.data(), static_cast<int>(nb), g.data(), lo.data(),
                                    hi.data(), win.data(), wbits.data(), split.data()),
                  "drhip_split_exact");
  }
  auto sp = [&](std::size_t s, std::size_t k) -> std::size_t { return split[s * (nb + 1) + k]; };

  // 3. move pieces: source s range [split[s][k-1], split[s][k]) -> dest k
  //    (xGMI peer copies across GPUs)
  for (std::size_t k = 0; k < P; k++) {
    std::size_t off = 0;
    for (std::size_t s = 0; s < P; s++) {
      const std::size_t a = k == 0 ? 0 : sp(s, k - 1), b = sp(s, k);
      if (b > a)
        detail::check(drhip_memcpy_d2d(static_cast<int>(parts[k].rank()), static_cast<T *>(sc[k].buf) + off,
                                       parts[s].data() + a, (b - a) * sizeof(T)),
                      "sort piece copy");
      off += b - a;
    }
    if (off != n[k]) throw std::runtime_error("shp::sort: splitting did not balance");
  }
  sync_all();
  // 4. destination merge of the P sorted runs straight into the segment
  //    (drhip_merge_runs_to: ceil(log2 P) merge-path passes instead of a
  //    second radix sort, the last pass writing the segment -- no copy back;
  //    every piece copy of step 3 has finished reading the segments)
  for (std::size_t k = 0; k < P; k++) {
    const int rk = static_cast<int>(parts[k].rank());
    std::vector<std::size_t> offs(P + 1, 0);
    for (std::size_t s = 0; s < P; s++) offs[s + 1] = offs[s] + (sp(s, k) - (k == 0 ? 0 : sp(s, k - 1)));
    detail::check(drhip_merge_runs_to(rk, detail::dtype_code<T>(), sc[k].buf, parts[k].data(), n[k], offs.data(),
                                      static_cast<int>(P), sc[k].mws, sc[k].mwsb),
                  "drhip_merge_runs_to");
  }
  sync_all();
  }
}

namespace detail {

// An order-reversing involution of the key's bits: ~x for integers (for
// two's complement ~x = -1 - x), the sign bit for IEEE floats (-x).  std::
// greater sorts as std::less on flipped keys, flipped back: two elementwise
// passes around the ascending radix sort (8 B/key each).
template <typename T> struct flip_order {
  __host__ __device__ void operator()(T &x) const {
    if constexpr (std::is_same_v<T, float>)
      x = __builtin_bit_cast(float, __builtin_bit_cast(std::uint32_t, x) ^ 0x80000000u);
    else if constexpr (std::is_same_v<T, double>)
      x = __builtin_bit_cast(double, __builtin_bit_cast(std::uint64_t, x) ^ 0x8000000000000000ull);
    else
      x = static_cast<T>(~x);
  }
};

template <typename C, typename T>
constexpr bool is_less_v = std::is_same_v<C, std::less<>> || std::is_same_v<C, std::less<T>> ||
                           std::is_same_v<C, std::ranges::less>;
template <typename C, typename T>
constexpr bool is_greater_v = std::is_same_v<C, std::greater<>> || std::is_same_v<C, std::greater<T>> ||
                              std::is_same_v<C, std::ranges::greater>;

} // namespace detail

namespace detail {

// The general tier (dr/shp/merge_sort.hpp): any trivially-copyable T, any
// strict weak ordering `comp` callable on host and device.  Stable: the
// result is std::stable_sort's over the whole range (equivalent elements keep
// their order -- segment order, then index order within a segment).
//   1. every segment: stable local merge sort, then its regular samples;
//   2. exact splitting under comp (dr_plan::split_windows_cmp /
//      split_exact_cmp, the general form of csrc/split.hip): windows from the
//      samples, then the key of every boundary rank from the windows, with
//      equivalent keys given out in segment order;
//   3. every (source, destination) piece moves with one device-to-device copy;
//   4. every destination merges its P runs pairwise (ceil(log2 P) rounds of
//      merge_kernel, the earlier run first on ties) into its segment.
template <typename T, typename Comp> void sort_general(auto &segs, Comp comp) {
  static_assert(std::is_trivially_copyable_v<T>, "shp::sort: the element type must be trivially copyable");
  static_assert(sizeof(T) <= 256, "shp::sort: elements above 256 bytes are not supported");
  std::vector<device_span<T>> parts;
  for (auto &s : segs)
    if (s.size()) parts.push_back(s);
  const std::size_t P = parts.size();
  if (P == 0) return;
  std::vector<std::uint64_t> n(P), stride(P), ns(P);
  for (std::size_t k = 0; k < P; k++) {
    n[k] = parts[k].size();
    stride[k] = std::max<std::uint64_t>(1, (n[k] + kSortSamples - 1) / kSortSamples);
    ns[k] = P > 1 ? (n[k] + stride[k] - 1) / stride[k] : 0;
  }
  // per segment: [local-sort scratch (doubles as the piece buffer) | samples]
  auto seg_bytes = [&](std::size_t k) { return align_up(msort::scratch_bytes<T>(n[k])) + align_up(ns[k] * sizeof(T)); };
  std::vector<char *> base(P);
  {
    std::map<std::size_t, std::size_t> rank_bytes;
    for (std::size_t k = 0; k < P; k++) rank_bytes[parts[k].rank()] += seg_bytes(k);
    std::map<std::size_t, char *> next;
    for (auto &[rk, b] : rank_bytes) next[rk] = static_cast<char *>(device_scratch().get(rk, b));
    for (std::size_t k = 0; k < P; k++) {
      base[k] = next[parts[k].rank()];
      next[parts[k].rank()] += seg_bytes(k);
    }
  }
  auto smp = [&](std::size_t k) { return reinterpret_cast<T *>(base[k] + align_up(msort::scratch_bytes<T>(n[k]))); };
  auto st = [&](std::size_t k) {
    hip_check(hipSetDevice(device_list().at(parts[k].rank())), "hipSetDevice");
    return stream(parts[k].rank());
  };
  // 1. local sorts and samples
  for (std::size_t k = 0; k < P; k++) {
    hipStream_t s = st(k);
    msort::local_sort(parts[k].data(), n[k], base[k], comp, s);
    if (P > 1)
      hipLaunchKernelGGL((msort::gather_samples_kernel<T>), dim3(msort::blocks_of(ns[k], 256)), dim3(256), 0, s,
                         parts[k].data(), stride[k], ns[k], smp(k));
    hip_check(hipGetLastError(), "shp::sort launch");
  }
  if (P == 1) {
    sync(parts[0].rank());
    return;
  }
  std::size_t tot_smp = 0;
  for (auto v : ns) tot_smp += v;
  std::vector<T> hs(tot_smp);
  for (std::size_t k = 0, off = 0; k < P; off += ns[k], k++)
    check(drhip_memcpy_d2h(static_cast<int>(parts[k].rank()), hs.data() + off, smp(k), ns[k] * sizeof(T)),
          "sort samples d2h");
  for (std::size_t k = 0; k < P; k++) sync(parts[k].rank());
  // 2. exact splitting under comp
  const std::size_t nb = P - 1;
  std::vector<std::uint64_t> g(nb), win(2 * P * nb), split(P * (nb + 1));
  for (std::size_t k = 0, acc = 0; k < nb; k++) g[k] = acc += n[k];
  if (const char *why = dr_plan::split_windows_cmp(static_cast<int>(P), n.data(), stride.data(), ns.data(), hs.data(),
                                                   static_cast<int>(nb), g.data(), comp, win.data()))
    throw std::runtime_error(std::string("shp::sort: ") + why);
  std::size_t tot_win = 0;
  for (std::size_t i = 0; i < P * nb; i++) tot_win += win[2 * i + 1] - win[2 * i];
  std::vector<T> hw(tot_win);
  for (std::size_t s = 0, off = 0; s < P; s++)
    for (std::size_t k = 0; k < nb; k++) {
      const std::size_t a = win[2 * (s * nb + k)], b = win[2 * (s * nb + k) + 1];
      if (b > a)
        check(drhip_memcpy_d2h(static_cast<int>(parts[s].rank()), hw.data() + off, parts[s].data() + a,
                               (b - a) * sizeof(T)),
              "sort slices d2h");
      off += b - a;
    }
  for (std::size_t s = 0; s < P; s++) sync(parts[s].rank());
  if (const char *why = dr_plan::split_exact_cmp(static_cast<int>(P), n.data(), static_cast<int>(nb), g.data(),
                                                 win.data(), hw.data(), comp, split.data()))
    throw std::runtime_error(std::string("shp::sort: ") + why);
  auto sp = [&](std::size_t s, std::size_t k) -> std::size_t { return split[s * (nb + 1) + k]; };
  // 3. pieces into every destination's buffer, in source order
  std::vector<std::vector<std::size_t>> offs(P, std::vector<std::size_t>(P + 1, 0));
  for (std::size_t k = 0; k < P; k++) {
    T *buf = reinterpret_cast<T *>(base[k]);
    for (std::size_t s = 0; s < P; s++) {
      const std::size_t a = k == 0 ? 0 : sp(s, k - 1), b = sp(s, k);
      if (b > a)
        check(drhip_memcpy_d2d(static_cast<int>(parts[k].rank()), buf + offs[k][s], parts[s].data() + a,
                               (b - a) * sizeof(T)),
              "sort piece copy");
      offs[k][s + 1] = offs[k][s] + (b - a);
    }
    if (offs[k][P] != n[k]) throw std::runtime_error("shp::sort: splitting did not balance");
  }
  sync_all();
  // 4. pairwise run merges, the last round into the segment: with R rounds
  //    and two buffers, the runs start in the segment when R is even
  std::size_t R = 0;
  while ((std::size_t(1) << R) < P) R++;
  for (std::size_t k = 0; k < P; k++) {
    hipStream_t s = st(k);
    T *buf = reinterpret_cast<T *>(base[k]), *seg = parts[k].data();
    T *src = buf, *dst = seg;
    if (R % 2 == 0) {
      hip_check(hipMemcpyAsync(seg, buf, n[k] * sizeof(T), hipMemcpyDeviceToDevice, s), "sort run copy");
      std::swap(src, dst);
    }
    // the tile splits: where the local sort kept its own, past the piece buffer
    std::vector<std::size_t> run = offs[k];
    auto *part = reinterpret_cast<std::size_t *>(base[k] + align_up(n[k] * sizeof(T)));
    while (run.size() > 2) {
      std::vector<std::size_t> next{0};
      for (std::size_t r = 0; r + 1 < run.size(); r += 2) {
        const std::size_t a = run[r], m = run[r + 1], e = r + 2 < run.size() ? run[r + 2] : m;
        if (e > a) {
          if (e > m && m > a)
            msort::merge_pass<T>(src + a, dst + a, msort::pass_geom{e - a, m - a, true}, part, comp, s);
          else
            hip_check(hipMemcpyAsync(dst + a, src + a, (e - a) * sizeof(T), hipMemcpyDeviceToDevice, s), "sort run copy");
        }
        next.push_back(e);
      }
      run.swap(next);
      std::swap(src, dst);
      hip_check(hipGetLastError(), "shp::sort merge launch");
    }
  }
  sync_all();
}

} // namespace detail

// std::ranges::sort(r, comp) for comp in {std::less, std::greater} (any of
// their spellings).  Descending keys: equal keys are indistinguishable, so
// the result is bit-identical to any correct descending sort (for floats,
// as with std::less: inputs without NaN, and -0.0 / +0.0 compare equal).
// Any other comparator or element type: the stable general tier.
template <typename ExecutionPolicy, typename R, typename Compare>
  requires lib::distributed_contiguous_range<R>
void sort(ExecutionPolicy &&policy, R &&r, Compare comp) {
  using C = std::remove_cvref_t<Compare>;
  using T = std::remove_cv_t<std::ranges::range_value_t<R>>;
  if constexpr (detail::abi_type<T> && detail::is_less_v<C, T>) {
    shp::sort(std::forward<ExecutionPolicy>(policy), std::forward<R>(r));
  } else if constexpr (detail::abi_type<T> && detail::is_greater_v<C, T>) {
    shp::for_each(policy, r, detail::flip_order<T>{});
    shp::sort(policy, r);
    shp::for_each(policy, r, detail::flip_order<T>{});
  } else {
    auto segs = lib::ranges::segments(r);
    detail::sort_general<T>(segs, comp);
  }
}

// std::ranges::stable_sort(r[, comp]): equivalent elements keep their order.
// Integer keys under std::less / std::greater are indistinguishable when
// equivalent, so they keep the radix path; everything else (floats included:
// -0.0 and +0.0 are equivalent but not identical) takes the general tier.
template <typename ExecutionPolicy, typename R, typename Compare = std::ranges::less>
  requires lib::distributed_contiguous_range<R>
void stable_sort(ExecutionPolicy &&policy, R &&r, Compare comp = {}) {
  using C = std::remove_cvref_t<Compare>;
  using T = std::remove_cv_t<std::ranges::range_value_t<R>>;
  if constexpr (detail::abi_type<T> && std::is_integral_v<T> && (detail::is_less_v<C, T> || detail::is_greater_v<C, T>)) {
    shp::sort(std::forward<ExecutionPolicy>(policy), std::forward<R>(r), comp);
  } else {
    auto segs = lib::ranges::segments(r);
    detail::sort_general<T>(segs, comp);
  }
}

template <typename ExecutionPolicy, lib::distributed_iterator Iter, typename Compare = std::ranges::less>
void stable_sort(ExecutionPolicy &&policy, Iter first, Iter last, Compare comp = {}) {
  shp::stable_sort(std::forward<ExecutionPolicy>(policy), std::ranges::subrange(first, last), comp);
}

template <typename ExecutionPolicy, lib::distributed_iterator Iter>
void sort(ExecutionPolicy &&policy, Iter first, Iter last) {
  shp::sort(std::forward<ExecutionPolicy>(policy), std::ranges::subrange(first, last));
}

template <typename ExecutionPolicy, lib::distributed_iterator Iter, typename Compare>
void sort(ExecutionPolicy &&policy, Iter first, Iter last, Compare comp) {
  shp::sort(std::forward<ExecutionPolicy>(policy), std::ranges::subrange(first, last), comp);
}

} // namespace shp
