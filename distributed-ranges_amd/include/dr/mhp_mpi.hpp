// dr/mhp_mpi.hpp -- MPI bootstrap and MPI transport for dr/mhp.hpp.
//
// The reference's mhp backend is MPI end to end (details/communicator.hpp:
// isend/irecv with the halo tags, MPI_Gather for mhp::reduce).  This header
// gives dr/mhp.hpp the same two options an MPI program has:
//   init_mpi(device, /*rccl=*/true)   one rank per GPU, RCCL communicator
//                                     bootstrapped by MPI_Bcast of the id
//                                     (the production path over xGMI);
//   init_mpi(device, /*rccl=*/false)  MPI messages for the cross-rank steps
//                                     (device buffers staged through host
//                                     memory; MPICH here is not GPU-aware) --
//                                     what runs 2..4 ranks on ONE GPU, which
//                                     RCCL refuses.
// Include it only in programs linked against MPI; dr/mhp.hpp itself has no
// MPI dependency.
#pragma once

#include <mpi.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "mhp.hpp"

namespace mhp {

struct mpi_transport final : transport {
  explicit mpi_transport(MPI_Comm c = MPI_COMM_WORLD) : comm_(c) {}
  const char *name() const override { return "mpi"; }

  // halo.hpp:55-70 exchange(): receives posted first, then the sends, wait
  // for all, received cells replace the halo (`second`)
  void halo(void *buf, std::size_t n_owned, std::size_t cell_bytes, std::size_t prev, std::size_t next,
            bool periodic) override {
    int rank = 0, nranks = 1;
    MPI_Comm_rank(comm_, &rank);
    MPI_Comm_size(comm_, &nranks);
    const auto msgs = dr_plan::halo_messages(rank, nranks, n_owned, prev, next, periodic);
    std::vector<std::vector<char>> host(msgs.size());
    std::vector<MPI_Request> req(msgs.size(), MPI_REQUEST_NULL);
    char *b = static_cast<char *>(buf);
    for (std::size_t i = 0; i < msgs.size(); i++) {
      const auto &m = msgs[i];
      host[i].resize(m.cells * cell_bytes);
      if (!m.send) {
        MPI_Irecv(host[i].data(), (int)host[i].size(), MPI_BYTE, m.peer, m.tag, comm_, &req[i]);
      }
    }
    for (std::size_t i = 0; i < msgs.size(); i++) {
      const auto &m = msgs[i];
      if (m.send) {
        detail::check(drhip_memcpy_d2h(0, host[i].data(), b + m.cell_off * cell_bytes, host[i].size()),
                      "drhip_memcpy_d2h");
        MPI_Isend(host[i].data(), (int)host[i].size(), MPI_BYTE, m.peer, m.tag, comm_, &req[i]);
      }
    }
    MPI_Waitall((int)req.size(), req.data(), MPI_STATUSES_IGNORE);
    for (std::size_t i = 0; i < msgs.size(); i++) {
      const auto &m = msgs[i];
      if (!m.send)
        detail::check(drhip_memcpy_h2d(0, b + m.cell_off * cell_bytes, host[i].data(), host[i].size()),
                      "drhip_memcpy_h2d");
    }
    detail::sync();
  }

  // communicator.hpp:51-56 gather (MPI_Gather of `bytes` per rank to root)
  void gather(const void *send, void *recv, std::size_t bytes, int root) override {
    int rank = 0, nranks = 1;
    MPI_Comm_rank(comm_, &rank);
    MPI_Comm_size(comm_, &nranks);
    std::vector<char> s(bytes), r(rank == root ? bytes * nranks : 0);
    if (bytes) detail::check(drhip_memcpy_d2h(0, s.data(), send, bytes), "drhip_memcpy_d2h");
    MPI_Gather(s.data(), (int)bytes, MPI_BYTE, r.data(), (int)bytes, MPI_BYTE, root, comm_);
    if (rank == root && bytes)
      detail::check(drhip_memcpy_h2d(0, recv, r.data(), r.size()), "drhip_memcpy_h2d");
    detail::sync();
  }

  void barrier() override { MPI_Barrier(comm_); }

  // the misaligned copy's exchange: owned pieces staged through the host,
  // MPI_Alltoallv of bytes, each received piece copied to its slot
  void alltoallv(const void *send, const std::size_t *send_bytes, const std::size_t *send_off, void *recv,
                 const std::size_t *recv_bytes, const std::size_t *recv_off) override {
    int nranks = 1;
    MPI_Comm_size(comm_, &nranks);
    std::size_t send_end = 0, recv_tot = 0;
    std::vector<int> sc(nranks), sd(nranks), rc(nranks), rd(nranks);
    for (int r = 0; r < nranks; r++) {
      if (send_bytes[r]) send_end = std::max(send_end, send_off[r] + send_bytes[r]);
      if (send_off[r] + send_bytes[r] > (std::size_t)INT32_MAX || recv_tot + recv_bytes[r] > (std::size_t)INT32_MAX)
        throw std::runtime_error("mhp mpi_transport: alltoallv piece above 2 GiB");
      sc[r] = (int)send_bytes[r];
      sd[r] = (int)send_off[r];
      rc[r] = (int)recv_bytes[r];
      rd[r] = (int)recv_tot;
      recv_tot += recv_bytes[r];
    }
    std::vector<char> s(send_end), rbuf(recv_tot);
    if (send_end) detail::check(drhip_memcpy_d2h(0, s.data(), send, send_end), "drhip_memcpy_d2h");
    MPI_Alltoallv(s.data(), sc.data(), sd.data(), MPI_BYTE, rbuf.data(), rc.data(), rd.data(), MPI_BYTE, comm_);
    for (int r = 0; r < nranks; r++)
      if (recv_bytes[r])
        detail::check(drhip_memcpy_h2d(0, static_cast<char *>(recv) + recv_off[r], rbuf.data() + rd[r], recv_bytes[r]),
                      "drhip_memcpy_h2d");
    detail::sync();
  }

private:
  MPI_Comm comm_;
};

// mhp::init for an MPI program (MPI_Init already called): rank and size
// from MPI_COMM_WORLD; device < 0 picks rank % visible devices.
inline void init_mpi(int device = -1, bool rccl = true) {
  int rank = 0, nranks = 1;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &nranks);
  if (device < 0) {
    int ndev = 0;
    detail::check(drhip_device_count(&ndev), "drhip_device_count");
    device = ndev > 0 ? rank % ndev : 0;
  }
  if (!rccl) {
    init(rank, nranks, device, std::make_unique<mpi_transport>());
    return;
  }
  comm_id id{};
  if (rank == 0) id = make_comm_id();
  MPI_Bcast(id.data(), (int)id.size(), MPI_BYTE, 0, MPI_COMM_WORLD);
  init(rank, nranks, device, id);
}

} // namespace mhp
