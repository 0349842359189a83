// split_plan_test.cpp -- CPU test of the distributed sort's exact splitting
// (distributed-ranges_amd/include/dr/details/split_plan.hpp, the arithmetic
// behind drhip_split_windows / drhip_split_exact).  Built plain and under
// AddressSanitizer + UndefinedBehaviorSanitizer (tests/cpp/Makefile
// `sanitize`, tests/test_sanitize.py).
//
// Random sorted runs on P = 1..9 ranks (empty runs, heavy duplicates, the
// full 64-bit key range, strides 1..n), the sort's destination boundaries
// g_k = k * ceil(N / P) plus boundaries past the end.  Checks, per boundary:
//   * the bracket [lo_k, hi_k] holds the key of global rank g_k;
//   * every rank's window [a, b) holds every key of the bracket;
//   * split sizes sum to min(g_k, N) and grow with k on every rank;
//   * exact partition: every key below a split <= every key above it.
#include <dr/details/split_plan.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

using u64 = std::uint64_t;

static int g_fail = 0;
#define CHECK(c)                                                                 \
  do {                                                                           \
    if (!(c)) {                                                                  \
      if (g_fail++ < 20) std::printf("FAILED %s:%d: %s (case %d)\n", __FILE__, __LINE__, #c, g_case); \
    }                                                                            \
  } while (0)
static int g_case = 0;

static void one_case(std::mt19937_64 &rng) {
  const int p = 1 + (int)(rng() % 9);
  const int kind = (int)(rng() % 3); // 0: few distinct keys, 1: medium, 2: full range
  std::vector<std::vector<u64>> keys(p);
  for (auto &r : keys) {
    const std::size_t n = (rng() % 5 == 0) ? 0 : rng() % 3000;
    r.resize(n);
    for (auto &v : r) v = kind == 0 ? rng() % 5 : kind == 1 ? rng() % 1000 : rng();
    std::sort(r.begin(), r.end());
  }
  std::vector<u64> n(p), stride(p), ns(p), samples;
  u64 ntot = 0;
  for (int i = 0; i < p; i++) {
    n[i] = keys[i].size();
    ntot += n[i];
    stride[i] = n[i] ? 1 + rng() % (n[i] + 1) : 1 + rng() % 4;
    for (u64 j = 0; j * stride[i] < n[i]; j++) samples.push_back(keys[i][j * stride[i]]);
    ns[i] = n[i] ? (n[i] + stride[i] - 1) / stride[i] : 0;
  }
  const u64 seg = (ntot + p - 1) / p;
  std::vector<u64> g;
  for (int k = 1; k < p; k++) g.push_back(k * seg);
  g.push_back(ntot + (rng() % 3)); // at or past the end
  const int nb = (int)g.size();
  std::vector<u64> lo(nb), hi(nb), win(2 * (std::size_t)p * nb);
  CHECK(dr_plan::split_windows(p, n.data(), stride.data(), ns.data(), samples.empty() ? nullptr : samples.data(), nb,
                               g.data(), lo.data(), hi.data(), win.data()) == nullptr);
  std::vector<u64> all;
  for (auto &r : keys) all.insert(all.end(), r.begin(), r.end());
  std::sort(all.begin(), all.end());
  std::vector<u64> wkeys;
  for (int i = 0; i < p; i++)
    for (int k = 0; k < nb; k++) {
      const u64 a = win[2 * ((std::size_t)i * nb + k)], b = win[2 * ((std::size_t)i * nb + k) + 1];
      CHECK(a <= b && b <= n[i]);
      if (!(a <= b && b <= n[i])) return;
      // every key of the bracket lies inside the window
      for (u64 j = 0; j < n[i]; j++)
        if (keys[i][j] >= lo[k] && keys[i][j] <= hi[k] && g[k] < ntot) CHECK(j >= a && j < b);
      wkeys.insert(wkeys.end(), keys[i].begin() + a, keys[i].begin() + b);
    }
  for (int k = 0; k < nb; k++)
    if (g[k] < ntot) CHECK(lo[k] <= all[g[k]] && all[g[k]] <= hi[k]);
  std::vector<u64> split((std::size_t)p * (nb + 1));
  CHECK(dr_plan::split_exact(p, n.data(), nb, g.data(), lo.data(), hi.data(), win.data(),
                             wkeys.empty() ? nullptr : wkeys.data(), split.data()) == nullptr);
  for (int k = 0; k < nb; k++) {
    u64 s = 0, below_max = 0, above_min = ~u64(0);
    bool any_below = false;
    for (int i = 0; i < p; i++) {
      const u64 c = split[(std::size_t)i * (nb + 1) + k];
      CHECK(c <= n[i]);
      if (k) CHECK(c >= split[(std::size_t)i * (nb + 1) + k - 1]);
      s += c;
      if (c) {
        below_max = std::max(below_max, keys[i][c - 1]);
        any_below = true;
      }
      if (c < n[i]) above_min = std::min(above_min, keys[i][c]);
    }
    CHECK(s == std::min(g[k], ntot));
    if (any_below && above_min != ~u64(0)) CHECK(below_max <= above_min);
  }
  for (int i = 0; i < p; i++) CHECK(split[(std::size_t)i * (nb + 1) + nb] == n[i]);
}

// The comparator form (split_windows_cmp / split_exact_cmp, shp::sort's
// general tier): records ordered by one field, the whole distributed stable
// sort simulated on the host -- local stable sorts, the splits, pieces in
// source order, a stable merge per destination -- must equal std::stable_sort
// of the ranks' data in rank order, record for record.
struct rec {
  u64 key;
  int src;
  std::size_t idx;
};
static void one_cmp_case(std::mt19937_64 &rng) {
  const int p = 1 + (int)(rng() % 9);
  const u64 mod = rng() % 3 == 0 ? 3 : rng() % 2 ? 1000 : ~u64(0);
  auto comp = [](const rec &a, const rec &b) { return a.key < b.key; };
  std::vector<std::vector<rec>> keys(p);
  std::vector<rec> orig;
  for (int i = 0; i < p; i++) {
    const std::size_t n = (rng() % 5 == 0) ? 0 : rng() % 3000;
    for (std::size_t j = 0; j < n; j++) keys[i].push_back({mod == ~u64(0) ? rng() : rng() % mod, i, j});
    orig.insert(orig.end(), keys[i].begin(), keys[i].end());
    std::stable_sort(keys[i].begin(), keys[i].end(), comp);
  }
  std::vector<u64> n(p), stride(p), ns(p);
  std::vector<rec> samples;
  u64 ntot = 0;
  for (int i = 0; i < p; i++) {
    n[i] = keys[i].size();
    ntot += n[i];
    stride[i] = n[i] ? 1 + rng() % (n[i] + 1) : 1 + rng() % 4;
    for (u64 j = 0; j * stride[i] < n[i]; j++) samples.push_back(keys[i][j * stride[i]]);
    ns[i] = n[i] ? (n[i] + stride[i] - 1) / stride[i] : 0;
  }
  const u64 seg = (ntot + p - 1) / p;
  std::vector<u64> g;
  for (int k = 1; k < p; k++) g.push_back(std::min<u64>(k * seg, ntot));
  const int nb = (int)g.size();
  std::vector<u64> win(2 * (std::size_t)p * nb + 2);
  CHECK(dr_plan::split_windows_cmp(p, n.data(), stride.data(), ns.data(), samples.empty() ? nullptr : samples.data(), nb,
                                   g.data(), comp, win.data()) == nullptr);
  std::vector<rec> wkeys;
  for (int i = 0; i < p; i++)
    for (int k = 0; k < nb; k++) {
      const u64 a = win[2 * ((std::size_t)i * nb + k)], b = win[2 * ((std::size_t)i * nb + k) + 1];
      CHECK(a <= b && b <= n[i]);
      if (!(a <= b && b <= n[i])) return;
      wkeys.insert(wkeys.end(), keys[i].begin() + a, keys[i].begin() + b);
    }
  std::vector<u64> split((std::size_t)p * (nb + 1));
  const char *why = dr_plan::split_exact_cmp(p, n.data(), nb, g.data(), win.data(), wkeys.empty() ? nullptr : wkeys.data(),
                                             comp, split.data());
  CHECK(why == nullptr);
  if (why) return;
  std::vector<rec> out;
  for (int k = 0; k < p; k++) {
    std::vector<rec> d;
    for (int i = 0; i < p; i++) {
      const u64 a = k ? split[(std::size_t)i * (nb + 1) + k - 1] : 0, b = split[(std::size_t)i * (nb + 1) + k];
      CHECK(a <= b);
      if (a > b) return;
      d.insert(d.end(), keys[i].begin() + a, keys[i].begin() + b);
    }
    if (k + 1 < p) CHECK(d.size() == (k ? g[k] - g[k - 1] : g[0]));
    std::stable_sort(d.begin(), d.end(), comp); // = the pairwise stable run merge
    out.insert(out.end(), d.begin(), d.end());
  }
  std::stable_sort(orig.begin(), orig.end(), comp);
  CHECK(out.size() == orig.size());
  bool same = out.size() == orig.size();
  for (std::size_t i = 0; same && i < out.size(); i++)
    same = out[i].key == orig[i].key && out[i].src == orig[i].src && out[i].idx == orig[i].idx;
  CHECK(same);
}

int main(int argc, char **argv) {
  const int cases = argc > 1 ? std::atoi(argv[1]) : 400;
  std::mt19937_64 rng(0x5eed);
  for (g_case = 0; g_case < cases; g_case++) one_case(rng);
  for (g_case = 0; g_case < cases; g_case++) one_cmp_case(rng);
  // refused arguments
  u64 one = 1;
  CHECK(dr_plan::split_windows(0, &one, &one, &one, &one, 0, nullptr, nullptr, nullptr, nullptr) != nullptr);
  u64 zero = 0;
  CHECK(dr_plan::split_windows(1, &one, &zero, &one, &one, 0, nullptr, nullptr, nullptr, nullptr) != nullptr);
  CHECK(dr_plan::split_windows(1, &one, &one, &one, nullptr, 0, nullptr, nullptr, nullptr, nullptr) != nullptr);
  std::printf("%s: %d cases, %d failures\n", g_fail ? "FAILED" : "PASSED", cases, g_fail);
  return g_fail ? 1 : 0;
}
