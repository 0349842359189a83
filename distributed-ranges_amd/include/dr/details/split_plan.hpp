// split_plan.hpp -- host-only exact splitting of the distributed sort
// (the arithmetic behind drhip_split_windows / drhip_split_exact,
// csrc/split.hip).  No HIP dependency, so the CPU sanitizer build
// (tests/cpp/Makefile `sanitize`, tests/test_sanitize.py) runs it directly.
//
// shp::sort (absent from the reference) keeps the range's
// segmentation, so after the local radix sorts every destination segment k
// must receive EXACTLY the keys of global sorted ranks [g_{k-1}, g_k).  The
// splitting below needs two small exchanges of data that every rank already
// holds (SURVEY.md 8e "sort": samples allgather, then counts):
//
//   1. every rank publishes n_i, a stride t_i and its regular samples
//      s_i[j] = keys_i[j * t_i] (sorted keys, radix-order bits);
//   2. drhip_split_windows (identical on every rank): for each boundary g_k
//      a value bracket [lo_k, hi_k] that provably contains the key of global
//      rank g_k, and for each rank the slice [a, b) of its sorted keys that
//      holds every key of the bracket.  With c_i(u) = #samples < u and
//      c'_i(u) = #samples <= u, a sorted run satisfies
//          count_i(< u)  <= min(n_i, c_i(u) t_i)
//          count_i(<= u) >= (c'_i(u) - 1) t_i + 1       (c'_i(u) >= 1)
//      so lo_k = the largest sample whose upper bound is <= g_k and hi_k = the
//      smallest sample whose lower bound is > g_k bracket rank g_k, and each
//      rank's slice is at most (#its samples in the bracket + 1) t_i keys;
//   3. every rank publishes its slices (sizes known to all from step 2);
//   4. drhip_split_exact (identical on every rank): the key v_k of global
//      rank g_k by bisection over the bracket on the merged slices, then
//      split[s][k] = count_s(< v_k) + the share of keys equal to v_k given
//      to source s in segment order, so destination k's size is exact.
//
// Two allgathers of O(P * samples) and O(P * slices) elements plus the data
// all-to-all: 3 collectives per distributed sort, no device round trip per
// bisection step.  Keys are passed as radix-order bits widened to uint64
// (order-preserving images of int32/uint32/float/int64/uint64/double keys).
#pragma once

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <vector>

namespace dr_plan {

using u64 = std::uint64_t;

// #elements of the sorted array [p, p + n) below / not above v
inline std::size_t count_lt(const u64 *p, std::size_t n, u64 v) { return (std::size_t)(std::lower_bound(p, p + n, v) - p); }
inline std::size_t count_le(const u64 *p, std::size_t n, u64 v) { return (std::size_t)(std::upper_bound(p, p + n, v) - p); }

// step 2; returns nullptr, or the reason the arguments were refused
inline const char *split_windows(int p, const u64 *n, const u64 *stride, const u64 *nsamples, const u64 *samples,
                                 int nb, const u64 *g, u64 *lo, u64 *hi, u64 *win) {
  if (p <= 0 || nb < 0 || !n || !stride || !nsamples || (nb && (!g || !lo || !hi || !win)))
    return "drhip_split_windows: bad argument";
  std::vector<const u64 *> s(p);
  std::vector<u64> all;
  {
    std::size_t off = 0;
    for (int i = 0; i < p; i++) {
      if (nsamples[i] && !stride[i]) return "drhip_split_windows: zero stride";
      off += nsamples[i];
    }
    if (off && !samples) return "drhip_split_windows: bad argument";
    off = 0;
    for (int i = 0; i < p; i++) {
      s[i] = samples ? samples + off : nullptr;
      off += nsamples[i];
    }
    if (off) all.assign(samples, samples + off);
    std::sort(all.begin(), all.end());
    all.erase(std::unique(all.begin(), all.end()), all.end());
  }
  // upper bound of count(< u) and lower bound of count(<= u), summed over ranks
  auto ub_lt = [&](u64 u) {
    u64 t = 0;
    for (int i = 0; i < p; i++) t += std::min<u64>(n[i], count_lt(s[i], nsamples[i], u) * stride[i]);
    return t;
  };
  auto lb_le = [&](u64 u) {
    u64 t = 0;
    for (int i = 0; i < p; i++) {
      const u64 c = count_le(s[i], nsamples[i], u);
      if (c) t += (c - 1) * stride[i] + 1;
    }
    return t;
  };
  for (int k = 0; k < nb; k++) {
    // lo: largest sample with ub_lt <= g (ub_lt is monotone); 0 if none
    std::size_t a = 0, b = all.size(); // first index with ub_lt > g
    while (a < b) {
      const std::size_t m = (a + b) / 2;
      if (ub_lt(all[m]) <= g[k]) a = m + 1;
      else b = m;
    }
    lo[k] = a ? all[a - 1] : 0;
    // hi: smallest sample with lb_le > g; ~0 if none
    a = 0, b = all.size();
    while (a < b) {
      const std::size_t m = (a + b) / 2;
      if (lb_le(all[m]) > g[k]) b = m;
      else a = m + 1;
    }
    hi[k] = a < all.size() ? all[a] : ~u64(0);
    if (hi[k] < lo[k]) hi[k] = lo[k];
    for (int i = 0; i < p; i++) {
      const u64 c = count_lt(s[i], nsamples[i], lo[k]);
      const u64 c2 = count_le(s[i], nsamples[i], hi[k]);
      // keys at index <= (c-1) t are < lo; keys at index >= c2 t are > hi
      const u64 wa = c ? std::min<u64>(n[i], (c - 1) * stride[i] + 1) : 0;
      const u64 wb = std::min<u64>(n[i], c2 * stride[i]);
      win[2 * ((std::size_t)i * nb + k)] = wa;
      win[2 * ((std::size_t)i * nb + k) + 1] = std::max(wa, wb);
    }
  }
  return nullptr;
}

// step 4; returns nullptr, or the reason the arguments were refused
inline const char *split_exact(int p, const u64 *n, int nb, const u64 *g, const u64 *lo, const u64 *hi,
                               const u64 *win, const u64 *wkeys, u64 *split) {
  if (p <= 0 || nb < 0 || !n || (nb && (!g || !lo || !hi || !win || !split)))
    return "drhip_split_exact: bad argument";
  // slice (i, k) starts at offset sum of the lengths of slices before it in
  // (rank, boundary) order
  std::vector<const u64 *> w((std::size_t)p * nb);
  {
    std::size_t off = 0;
    for (int i = 0; i < p; i++)
      for (int k = 0; k < nb; k++) {
        w[(std::size_t)i * nb + k] = wkeys + off;
        off += win[2 * ((std::size_t)i * nb + k) + 1] - win[2 * ((std::size_t)i * nb + k)];
      }
  }
  auto cnt = [&](int i, int k, u64 v, bool le) -> u64 {
    const u64 a = win[2 * ((std::size_t)i * nb + k)], b = win[2 * ((std::size_t)i * nb + k) + 1];
    const u64 *q = w[(std::size_t)i * nb + k];
    return a + (le ? count_le(q, b - a, v) : count_lt(q, b - a, v));
  };
  u64 ntot = 0;
  for (int i = 0; i < p; i++) ntot += n[i];
  for (int k = 0; k < nb; k++) {
    if (g[k] >= ntot) { // boundary at or past the end: every key goes below it
      for (int i = 0; i < p; i++) split[(std::size_t)i * (nb + 1) + k] = n[i];
      continue;
    }
    auto total = [&](u64 v, bool le) {
      u64 t = 0;
      for (int i = 0; i < p; i++) t += cnt(i, k, v, le);
      return t;
    };
    if (total(lo[k], false) > g[k] || (hi[k] != ~u64(0) && total(hi[k], true) <= g[k]))
      return "drhip_split_exact: bracket does not hold the boundary rank";
    // v = smallest value in [lo, hi] with count(<= v) > g
    u64 a = lo[k], b = hi[k];
    while (a < b) {
      const u64 m = a + (b - a) / 2;
      if (total(m, true) > g[k]) b = m;
      else a = m + 1;
    }
    u64 need = g[k];
    std::vector<u64> lt(p), le(p);
    for (int i = 0; i < p; i++) {
      lt[i] = cnt(i, k, a, false);
      le[i] = cnt(i, k, a, true);
      need -= lt[i];
    }
    for (int i = 0; i < p; i++) {
      const u64 take = std::min(le[i] - lt[i], need);
      split[(std::size_t)i * (nb + 1) + k] = lt[i] + take;
      need -= take;
    }
  }
  for (int i = 0; i < p; i++) split[(std::size_t)i * (nb + 1) + nb] = n[i];
  return nullptr;
}

// ---- the same two steps under a comparator (shp::sort's general tier,
// dr/shp/merge_sort.hpp): keys are the elements themselves, ordered by
// `comp` (a strict weak ordering, callable on the host).  Equivalent keys are
// ranked in segment order, so with stable local sorts and a stable run merge
// the distributed result is std::stable_sort's.  The value bisection of
// split_exact becomes a bisection over the window elements, which hold the
// key of every boundary rank.
struct cmp_bracket {
  bool has_lo = false, has_hi = false;
  std::size_t lo = 0, hi = 0; // indices into the sorted sample list
};

template <typename T, typename Comp>
inline std::size_t count_lt_c(const T *p, std::size_t n, const T &v, Comp &comp) {
  return (std::size_t)(std::lower_bound(p, p + n, v, comp) - p);
}
template <typename T, typename Comp>
inline std::size_t count_le_c(const T *p, std::size_t n, const T &v, Comp &comp) {
  return (std::size_t)(std::upper_bound(p, p + n, v, comp) - p);
}

// step 2 under comp; samples of rank i at samples + sum(nsamples[< i]);
// win[2 (i nb + k) + {0, 1}] as split_windows
template <typename T, typename Comp>
inline const char *split_windows_cmp(int p, const u64 *n, const u64 *stride, const u64 *nsamples, const T *samples,
                                     int nb, const u64 *g, Comp comp, u64 *win) {
  if (p <= 0 || nb < 0 || !n || !stride || !nsamples || (nb && (!g || !win))) return "split_windows_cmp: bad argument";
  std::vector<const T *> s(p);
  std::vector<T> all;
  {
    std::size_t off = 0;
    for (int i = 0; i < p; i++) {
      if (nsamples[i] && !stride[i]) return "split_windows_cmp: zero stride";
      s[i] = samples ? samples + off : nullptr;
      off += nsamples[i];
    }
    if (off && !samples) return "split_windows_cmp: bad argument";
    if (off) all.assign(samples, samples + off);
    std::stable_sort(all.begin(), all.end(), comp);
  }
  auto ub_lt = [&](const T &u) {
    u64 t = 0;
    for (int i = 0; i < p; i++) t += std::min<u64>(n[i], count_lt_c(s[i], nsamples[i], u, comp) * stride[i]);
    return t;
  };
  auto lb_le = [&](const T &u) {
    u64 t = 0;
    for (int i = 0; i < p; i++) {
      const u64 c = count_le_c(s[i], nsamples[i], u, comp);
      if (c) t += (c - 1) * stride[i] + 1;
    }
    return t;
  };
  for (int k = 0; k < nb; k++) {
    std::size_t a = 0, b = all.size();
    while (a < b) {
      const std::size_t m = (a + b) / 2;
      if (ub_lt(all[m]) <= g[k]) a = m + 1;
      else b = m;
    }
    const bool has_lo = a > 0;
    const std::size_t lo = has_lo ? a - 1 : 0;
    a = 0, b = all.size();
    while (a < b) {
      const std::size_t m = (a + b) / 2;
      if (lb_le(all[m]) > g[k]) b = m;
      else a = m + 1;
    }
    const bool has_hi = a < all.size();
    std::size_t hi = has_hi ? a : 0;
    if (has_hi && has_lo && hi < lo) hi = lo;
    for (int i = 0; i < p; i++) {
      const u64 c = has_lo ? count_lt_c(s[i], nsamples[i], all[lo], comp) : 0;
      const u64 c2 = has_hi ? count_le_c(s[i], nsamples[i], all[hi], comp) : nsamples[i];
      const u64 wa = c ? std::min<u64>(n[i], (c - 1) * stride[i] + 1) : 0;
      const u64 wb = has_hi ? std::min<u64>(n[i], c2 * stride[i]) : n[i];
      win[2 * ((std::size_t)i * nb + k)] = wa;
      win[2 * ((std::size_t)i * nb + k) + 1] = std::max(wa, wb);
    }
  }
  return nullptr;
}

// step 4 under comp: wkeys holds the slices in (rank, boundary) order;
// split[i (nb + 1) + k] as split_exact
template <typename T, typename Comp>
inline const char *split_exact_cmp(int p, const u64 *n, int nb, const u64 *g, const u64 *win, const T *wkeys, Comp comp,
                                   u64 *split) {
  if (p <= 0 || nb < 0 || !n || (nb && (!g || !win || !split))) return "split_exact_cmp: bad argument";
  std::vector<const T *> w((std::size_t)p * nb);
  {
    std::size_t off = 0;
    for (int i = 0; i < p; i++)
      for (int k = 0; k < nb; k++) {
        w[(std::size_t)i * nb + k] = wkeys + off;
        off += win[2 * ((std::size_t)i * nb + k) + 1] - win[2 * ((std::size_t)i * nb + k)];
      }
  }
  auto cnt = [&](int i, int k, const T &v, bool le) -> u64 {
    const u64 a = win[2 * ((std::size_t)i * nb + k)], b = win[2 * ((std::size_t)i * nb + k) + 1];
    const T *q = w[(std::size_t)i * nb + k];
    return a + (le ? count_le_c(q, b - a, v, comp) : count_lt_c(q, b - a, v, comp));
  };
  u64 ntot = 0;
  for (int i = 0; i < p; i++) ntot += n[i];
  std::vector<T> cand;
  for (int k = 0; k < nb; k++) {
    if (g[k] >= ntot) {
      for (int i = 0; i < p; i++) split[(std::size_t)i * (nb + 1) + k] = n[i];
      continue;
    }
    auto total_le = [&](const T &v) {
      u64 t = 0;
      for (int i = 0; i < p; i++) t += cnt(i, k, v, true);
      return t;
    };
    cand.clear();
    for (int i = 0; i < p; i++) {
      const u64 a = win[2 * ((std::size_t)i * nb + k)], b = win[2 * ((std::size_t)i * nb + k) + 1];
      cand.insert(cand.end(), w[(std::size_t)i * nb + k], w[(std::size_t)i * nb + k] + (b - a));
    }
    std::stable_sort(cand.begin(), cand.end(), comp);
    // the key of rank g: the first candidate with count(<= c) > g
    std::size_t a = 0, b = cand.size();
    while (a < b) {
      const std::size_t m = (a + b) / 2;
      if (total_le(cand[m]) > g[k]) b = m;
      else a = m + 1;
    }
    if (a == cand.size()) return "split_exact_cmp: the windows do not hold the boundary rank";
    const T v = cand[a];
    u64 need = g[k];
    std::vector<u64> lt(p), le(p);
    for (int i = 0; i < p; i++) {
      lt[i] = cnt(i, k, v, false);
      le[i] = cnt(i, k, v, true);
      if (lt[i] > need) return "split_exact_cmp: the windows do not hold the boundary rank";
      need -= lt[i];
    }
    for (int i = 0; i < p; i++) {
      const u64 take = std::min(le[i] - lt[i], need);
      split[(std::size_t)i * (nb + 1) + k] = lt[i] + take;
      need -= take;
    }
  }
  for (int i = 0; i < p; i++) split[(std::size_t)i * (nb + 1) + nb] = n[i];
  return nullptr;
}

} // namespace dr_plan
