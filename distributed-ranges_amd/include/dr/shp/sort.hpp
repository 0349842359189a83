// dr/shp/sort.hpp -- shp::sort over a distributed range.
//
// The reference has no sort.  Semantics are
// std::ranges::sort: ascending under std::less, in place, the result keeps
// the range's segmentation.  Algorithm (single process, P segments):
//   1. every segment sorts locally (drhip_sort, LSD radix, in parallel);
//   2. exact splitting: for every segment boundary g_k = sum of the sizes of
//      segments < k, the value v_k of global rank g_k is found by bisection
//      over the order-preserving key bits, counting keys below a candidate in
//      every sorted segment (drhip_sort_bucket_counts, radix order); keys
//      equal to v_k are split in segment order, so every destination gets
//      exactly its segment's size;
//   3. every (source, destination) piece moves with one device-to-device
//      copy (xGMI peer copy across GPUs) into a per-destination buffer;
//   4. every destination sorts its buffer (P sorted runs) and copies it back
//      into its segment.
// With P == 1 only step 1 runs.
#pragma once

#include <cstring>
#include <functional>

#include "algorithms.hpp"

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

template <typename T> void sort_segment(const device_span<T> &s) {
  if (s.size() < 2) return;
  const int r = static_cast<int>(s.rank());
  std::size_t wsb = 0;
  check(drhip_sort_workspace(r, dtype_code<T>(), s.size(), &wsb), "drhip_sort_workspace");
  void *ws = nullptr;
  check(drhip_malloc(r, wsb, &ws), "drhip_malloc");
  check(drhip_sort(r, dtype_code<T>(), s.data(), s.size(), ws, wsb), "drhip_sort");
  sync(s.rank());
  check(drhip_free(r, ws), "drhip_free");
}

} // namespace detail

template <typename ExecutionPolicy, typename R>
  requires lib::distributed_contiguous_range<R>
void sort(ExecutionPolicy &&, R &&r) {
  using T = std::remove_cv_t<std::ranges::range_value_t<R>>;
  static_assert(detail::abi_type<T>, "shp::sort: key type must be int32/uint32/int64/uint64/float/double");
  using KB = detail::key_bits<T>;
  using U = typename KB::U;
  auto segs = lib::ranges::segments(r);
  std::vector<device_span<T>> parts;
  for (auto &s : segs)
    if (s.size()) parts.push_back(s);
  const std::size_t P = parts.size();
  if (P == 0) return;
  // 1. local sorts (all segments in flight, then wait)
  std::vector<void *> ws(P, nullptr);
  for (std::size_t k = 0; k < P; k++) {
    if (parts[k].size() < 2) continue;
    const int rk = static_cast<int>(parts[k].rank());
    std::size_t wsb = 0;
    detail::check(drhip_sort_workspace(rk, detail::dtype_code<T>(), parts[k].size(), &wsb), "drhip_sort_workspace");
    detail::check(drhip_malloc(rk, wsb, &ws[k]), "drhip_malloc");
    detail::check(drhip_sort(rk, detail::dtype_code<T>(), parts[k].data(), parts[k].size(), ws[k], wsb), "drhip_sort");
  }
  for (std::size_t k = 0; k < P; k++) {
    sync(parts[k].rank());
    if (ws[k]) detail::check(drhip_free(static_cast<int>(parts[k].rank()), ws[k]), "drhip_free");
  }
  if (P == 1) return;

  // 2. exact splitting at the segment boundaries
  const std::size_t nb = P - 1;
  std::vector<std::size_t> g(nb);
  {
    std::size_t acc = 0;
    for (std::size_t k = 0; k < nb; k++) g[k] = acc += parts[k].size();
  }
  detail::pinned<T> spl(nb);
  detail::pinned<std::uint64_t> cnt(P * (nb + 1));
  // count_below[s][k] = # keys of sorted segment s below spl[k] (radix order)
  auto count_below = [&](std::vector<std::vector<std::uint64_t>> &out) {
    for (std::size_t s = 0; s < P; s++)
      detail::check(drhip_sort_bucket_counts(static_cast<int>(parts[s].rank()), detail::dtype_code<T>(),
                                             parts[s].data(), parts[s].size(), spl.data(),
                                             static_cast<int>(nb), cnt.data() + s * (nb + 1)),
                    "drhip_sort_bucket_counts");
    for (std::size_t s = 0; s < P; s++) sync(parts[s].rank());
    for (std::size_t s = 0; s < P; s++) {
      std::uint64_t run = 0;
      for (std::size_t k = 0; k < nb; k++) {
        run += cnt[s * (nb + 1) + k];
        out[s][k] = run;
      }
    }
  };
  // bisection per boundary (all boundaries advance together): find the
  // smallest v with count(< v) > g_k; then v - 1 (in bits) is the key of
  // global rank g_k, i.e. lo ends at that key.
  std::vector<U> lo(nb, U(0)), hi(nb, ~U(0));
  std::vector<std::vector<std::uint64_t>> below(P, std::vector<std::uint64_t>(nb));
  for (int it = 0; it < 8 * (int)sizeof(U); it++) {
    // candidate c = lo + (hi - lo + 1) / 2: is count(< c) <= g ?  then lo = c
    std::vector<U> c(nb);
    for (std::size_t k = 0; k < nb; k++) {
      c[k] = lo[k] + static_cast<U>((hi[k] - lo[k]) / 2 + ((hi[k] - lo[k]) & 1));
      spl[k] = KB::out(c[k]);
    }
    count_below(below);
    for (std::size_t k = 0; k < nb; k++) {
      std::uint64_t tot = 0;
      for (std::size_t s = 0; s < P; s++) tot += below[s][k];
      if (hi[k] == lo[k]) continue;
      if (tot <= g[k]) lo[k] = c[k];
      else hi[k] = c[k] - 1;
    }
  }
  // v_k = lo: count(< v_k) <= g_k < count(<= v_k).  Per-source split points:
  // all keys below v_k, then keys equal to v_k in segment order.
  std::vector<std::vector<std::uint64_t>> split(P, std::vector<std::uint64_t>(nb + 1));
  {
    std::vector<std::vector<std::uint64_t>> lt(P, std::vector<std::uint64_t>(nb)), le(P, std::vector<std::uint64_t>(nb));
    for (std::size_t k = 0; k < nb; k++) spl[k] = KB::out(lo[k]);
    count_below(lt);
    for (std::size_t k = 0; k < nb; k++) spl[k] = KB::out(lo[k] + 1); // lo < max key: count(<= v)
    count_below(le);
    for (std::size_t k = 0; k < nb; k++) {
      std::uint64_t need = g[k];
      for (std::size_t s = 0; s < P; s++) need -= lt[s][k];
      for (std::size_t s = 0; s < P; s++) {
        const std::uint64_t eq = (lo[k] == ~U(0) ? parts[s].size() : le[s][k]) - lt[s][k];
        const std::uint64_t take = std::min<std::uint64_t>(eq, need);
        split[s][k] = lt[s][k] + take;
        need -= take;
      }
    }
    for (std::size_t s = 0; s < P; s++) split[s][nb] = parts[s].size();
  }
  // 3. move pieces: source s range [split[s][k-1], split[s][k]) -> dest k
  std::vector<void *> buf(P, nullptr);
  for (std::size_t k = 0; k < P; k++)
    detail::check(drhip_malloc(static_cast<int>(parts[k].rank()), parts[k].size() * sizeof(T), &buf[k]), "drhip_malloc");
  for (std::size_t k = 0; k < P; k++) {
    std::size_t off = 0;
    for (std::size_t s = 0; s < P; s++) {
      const std::size_t a = k == 0 ? 0 : split[s][k - 1], b = split[s][k];
      if (b > a)
        detail::check(drhip_memcpy_d2d(static_cast<int>(parts[k].rank()), static_cast<T *>(buf[k]) + off,
                                       parts[s].data() + a, (b - a) * sizeof(T)),
                      "sort piece copy");
      off += b - a;
    }
    if (off != parts[k].size()) throw std::runtime_error("shp::sort: splitting did not balance");
  }
  sync_all();
  // 4. destination merge of the P sorted runs (drhip_merge_runs: ceil(log2 P)
  //    merge-path passes instead of a second radix sort) + copy back
  std::vector<void *> mws(P, nullptr);
  for (std::size_t k = 0; k < P; k++) {
    const int rk = static_cast<int>(parts[k].rank());
    std::vector<std::size_t> offs(P + 1, 0);
    for (std::size_t s = 0; s < P; s++)
      offs[s + 1] = offs[s] + (split[s][k] - (k == 0 ? 0 : split[s][k - 1]));
    std::size_t wsb = 0;
    detail::check(drhip_merge_workspace(rk, detail::dtype_code<T>(), parts[k].size(), static_cast<int>(P), &wsb),
                  "drhip_merge_workspace");
    detail::check(drhip_malloc(rk, wsb, &mws[k]), "drhip_malloc");
    detail::check(drhip_merge_runs(rk, detail::dtype_code<T>(), buf[k], parts[k].size(), offs.data(),
                                   static_cast<int>(P), mws[k], wsb),
                  "drhip_merge_runs");
    detail::check(drhip_memcpy_d2d(static_cast<int>(parts[k].rank()), parts[k].data(), buf[k],
                                   parts[k].size() * sizeof(T)),
                  "sort copy back");
  }
  sync_all();
  for (std::size_t k = 0; k < P; k++) {
    detail::check(drhip_free(static_cast<int>(parts[k].rank()), buf[k]), "drhip_free");
    detail::check(drhip_free(static_cast<int>(parts[k].rank()), mws[k]), "drhip_free");
  }
}

template <typename ExecutionPolicy, typename R, typename Compare>
  requires lib::distributed_contiguous_range<R>
void sort(ExecutionPolicy &&policy, R &&r, Compare) {
  static_assert(std::is_same_v<std::remove_cvref_t<Compare>, std::less<>> ||
                    std::is_same_v<std::remove_cvref_t<Compare>, std::less<std::ranges::range_value_t<R>>>,
                "shp::sort: only std::less is supported");
  shp::sort(std::forward<ExecutionPolicy>(policy), std::forward<R>(r));
}

template <typename ExecutionPolicy, lib::distributed_iterator Iter>
void sort(ExecutionPolicy &&policy, Iter first, Iter last) {
  shp::sort(std::forward<ExecutionPolicy>(policy), std::ranges::subrange(first, last));
}

} // namespace shp
