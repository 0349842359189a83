// dr/details/halo_plan.hpp -- the span_halo message sequence and the mhp
// block layout as plain host data, shared by every transport.
//
// Host code only (no HIP, no MPI): the RCCL C-ABI (csrc/comm.hip
// drhip_halo_exchange), the MPI transport of dr/mhp_mpi.hpp and the CPU
// message test (tests/cpp/halo_plan_mpi.cpp, 1-4 MPICH ranks on host
// buffers) all issue exactly the messages listed here, so the sequence is
// checked on the CPU at every rank count the reference's mhp suite uses.
//
// Reference:
//   span_halo owned groups   details/halo.hpp:358-372 -- first `prev` owned
//                            cells to rank-1 (halo_reverse), last `next`
//                            owned cells to rank+1 (halo_forward)
//   span_halo halo groups    details/halo.hpp:374-386 -- prev halo from
//                            rank-1 (halo_forward), next halo from rank+1
//                            (halo_reverse); non-periodic ends skipped
//   exchange()               details/halo.hpp:55-70 (receives posted, then
//                            sends; received cells REPLACE the halo: `second`)
//   block layout             mhp/containers/distributed_vector.hpp:190-207
//                            (segment = max(ceil(n/P), prev, next), buffer
//                            [prev | segment | next])
#pragma once

#include <algorithm>
#include <cstddef>
#include <vector>

namespace dr_plan {

// communicator::tag values the reference uses for halo messages
enum halo_tag : int { tag_halo_forward = 1, tag_halo_reverse = 2 };

struct halo_msg {
  bool send;             // send or receive
  int peer;              // the other rank
  std::size_t cell_off;  // first cell, counted from the start of [prev | owned | next]
  std::size_t cells;     // number of cells
  int tag;               // halo_forward / halo_reverse (the reference's tags)
};

// The messages of one rank's exchange(), in issue order: sends [reverse to
// rank-1, forward to rank+1], then receives [from rank+1 into the next halo,
// from rank-1 into the prev halo].  A transport that matches a peer's sends
// to our receives IN ORDER without tags (RCCL) gets the right pairing from
// this order even when one peer is both neighbours (2 periodic ranks, or a
// periodic rank alone); a tagged transport (MPI) pairs by tag.
// Requires prev == next when both ends exchange (the reference's receive of
// `next` cells is matched by the neighbour's send of its `prev` cells).
inline std::vector<halo_msg> halo_messages(int rank, int nranks, std::size_t n_owned, std::size_t prev,
                                           std::size_t next, bool periodic) {
  std::vector<halo_msg> m;
  if (nranks < 1 || rank < 0 || rank >= nranks) return m;
  const bool first = rank == 0, last = rank == nranks - 1;
  const int rprev = first ? nranks - 1 : rank - 1, rnext = last ? 0 : rank + 1;
  const bool do_prev = prev > 0 && (periodic || !first), do_next = next > 0 && (periodic || !last);
  if (do_prev) m.push_back({true, rprev, prev, prev, tag_halo_reverse});               // first prev owned cells
  if (do_next) m.push_back({true, rnext, prev + n_owned - next, next, tag_halo_forward}); // last next owned cells
  if (do_next) m.push_back({false, rnext, prev + n_owned, next, tag_halo_reverse});    // next halo
  if (do_prev) m.push_back({false, rprev, 0, prev, tag_halo_forward});                 // prev halo
  return m;
}

// mhp::distributed_vector's block of rank r (distributed_vector.hpp:190-207)
struct block {
  std::size_t segment; // cells per rank (every rank's buffer holds prev + segment + next)
  std::size_t first;   // global index of this rank's first owned cell
  std::size_t local;   // owned cells that lie inside [0, n)
};
inline block block_of(std::size_t n, std::size_t nranks, std::size_t rank, std::size_t prev, std::size_t next) {
  const std::size_t p = std::max<std::size_t>(nranks, 1);
  const std::size_t seg = std::max({(n + p - 1) / p, prev, next});
  const std::size_t g0 = std::min(rank * seg, n);
  return {seg, g0, std::min(seg, n - g0)};
}

// Segments of a global range [a, b) of a block-distributed vector (n
// elements, `seg` per rank): rank r holds [max(a, r*seg), min(b, (r+1)*seg, n)).
// The reference's segments of a subrange (details/segments_tools.hpp:37-94
// take/drop of the container's segments); empty pieces are left out.
struct piece {
  std::size_t rank, begin, end; // global [begin, end) on `rank`
};
inline std::vector<piece> range_pieces(std::size_t n, std::size_t seg, std::size_t nranks, std::size_t a,
                                       std::size_t b) {
  std::vector<piece> v;
  b = std::min(b, n);
  for (std::size_t r = 0; r < nranks && seg; r++) {
    const std::size_t lo = std::max(a, r * seg), hi = std::min(b, std::min((r + 1) * seg, n));
    if (lo < hi) v.push_back({r, lo, hi});
  }
  return v;
}

// mhp/alignment.hpp:8-27 `aligned`: two ranges are aligned when their
// segments pair up rank by rank with equal sizes (so a copy / transform /
// zip between them is local to every rank).
inline bool pieces_aligned(const std::vector<piece> &x, const std::vector<piece> &y) {
  if (x.size() != y.size() || x.empty()) return false;
  for (std::size_t i = 0; i < x.size(); i++)
    if (x[i].rank != y[i].rank || x[i].end - x[i].begin != y[i].end - y[i].begin) return false;
  return true;
}

// The collective exchange that replaces the reference's serial fallback of
// mhp::copy / mhp::transform between MISALIGNED ranges
// (mhp/algorithms/cpu_algorithms.hpp:36-50, :147-161: rng::copy through
// per-element MPI_Put/Rget, then fence): element a + k of the input goes to
// output position o + k, k < b - a.  Every rank sends the input elements it
// owns to the ranks owning their output positions and receives its own
// output elements -- one alltoallv, no per-element traffic.  Counts and
// offsets are in ELEMENTS: send offsets from this rank's first owned input
// element (rank * seg_in), receive offsets from its first owned output
// element (rank * seg_out).  Pieces are in rank order on both sides, and
// both sides are monotone in k, so sends are consecutive slices of the
// owned input and receives consecutive slices of the owned output.
struct exchange {
  std::vector<std::size_t> send_cnt, send_off, recv_cnt, recv_off;
  std::size_t recv_total = 0;
};
inline exchange exchange_plan(std::size_t n_in, std::size_t seg_in, std::size_t a, std::size_t b, std::size_t n_out,
                              std::size_t seg_out, std::size_t o, std::size_t nranks, std::size_t rank) {
  exchange e;
  e.send_cnt.assign(nranks, 0);
  e.send_off.assign(nranks, 0);
  e.recv_cnt.assign(nranks, 0);
  e.recv_off.assign(nranks, 0);
  if (b <= a) return e;
  // output pieces of [o, o + len), and the input interval each maps from
  const auto outs = range_pieces(n_out, seg_out, nranks, o, o + (b - a));
  const auto ins = range_pieces(n_in, seg_in, nranks, a, b);
  for (const auto &pi : ins)
    for (const auto &po : outs) {
      // input [pi.begin, pi.end) -> output [pi.begin - a + o, ...) intersect po
      const std::size_t lo = std::max(pi.begin - a + o, po.begin), hi = std::min(pi.end - a + o, po.end);
      if (lo >= hi) continue;
      if (pi.rank == rank) {
        e.send_cnt[po.rank] = hi - lo;
        e.send_off[po.rank] = lo + a - o - rank * seg_in;
      }
      if (po.rank == rank) {
        e.recv_cnt[pi.rank] = hi - lo;
        e.recv_off[pi.rank] = lo - rank * seg_out;
        e.recv_total += hi - lo;
      }
    }
  return e;
}

// mhp::reduce's root fold (cpu_algorithms.hpp:124-138): init, then every
// rank's local result in rank order
template <typename T, typename It, typename Op> T fold_locals(T init, It first, It last, Op op) {
  for (; first != last; ++first) init = op(init, *first);
  return init;
}

} // namespace dr_plan
