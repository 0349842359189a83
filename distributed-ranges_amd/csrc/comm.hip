// comm.hip -- RCCL collectives over xGMI behind the C-ABI (include/drhip.h
// "RCCL over xGMI").
//
// Replaces the reference's MPI communicator for the cross-segment steps
// (include/dr/details/communicator.hpp:51-56 gather, :97-149 isend/irecv,
// details/halo.hpp:55-137 halo exchange) and, for multi-process use, the
// peer USM copies of shp (gemv.hpp:30-42 x replication).  Host code only:
// every call enqueues RCCL work on the segment's stream.
#include "common.hpp"

#include <rccl/rccl.h>

#include "../include/dr/details/halo_plan.hpp"

#include <string>
#include <vector>

namespace drhip {

namespace {
int set_nccl_error(ncclResult_t r, const char *what) {
  return set_error(DRHIP_ERR_COMM, (std::string(what) + ": " + ncclGetErrorString(r)).c_str());
}
#define DRHIP_CHECK_NCCL(expr)                                       \
  do {                                                               \
    ncclResult_t _r = (expr);                                        \
    if (_r != ncclSuccess) return set_nccl_error(_r, #expr);         \
  } while (0)

bool nccl_dtype(int dtype, ncclDataType_t *t) {
  switch (dtype) {
  case DRHIP_I32: *t = ncclInt32; return true;
  case DRHIP_U32: *t = ncclUint32; return true;
  case DRHIP_I64: *t = ncclInt64; return true;
  case DRHIP_U64: *t = ncclUint64; return true;
  case DRHIP_F32: *t = ncclFloat32; return true;
  case DRHIP_F64: *t = ncclFloat64; return true;
  default: return false;
  }
}
bool nccl_op(int op, ncclRedOp_t *o) {
  switch (op) {
  case DRHIP_PLUS: *o = ncclSum; return true;
  case DRHIP_MUL: *o = ncclProd; return true;
  case DRHIP_MIN: *o = ncclMin; return true;
  case DRHIP_MAX: *o = ncclMax; return true;
  default: return false;
  }
}
} // namespace

void comm_release(Segment &s) {
  if (s.comm) {
    (void)ncclCommDestroy((ncclComm_t)s.comm);
    s.comm = nullptr;
  }
}

} // namespace drhip

using namespace drhip;

#define DRHIP_GET_COMM(s, seg, c)                                                        \
  DRHIP_GET_SEG(s, seg);                                                                 \
  if (!s->comm) return set_error(DRHIP_ERR_NOT_INIT, "segment has no communicator"); \
  ncclComm_t c = (ncclComm_t)s->comm

extern "C" {

int drhip_comm_unique_id(void *id) {
  if (!id) return set_error(DRHIP_ERR_BAD_ARG, "drhip_comm_unique_id: null");
  ncclUniqueId u;
  DRHIP_CHECK_NCCL(ncclGetUniqueId(&u));
  memcpy(id, &u, sizeof(u));
  return DRHIP_OK;
}

int drhip_comm_init_rank(int seg, int nranks, int rank, const void *id) {
  DRHIP_GET_SEG(s, seg);
  if (!id || nranks < 1 || rank < 0 || rank >= nranks)
    return set_error(DRHIP_ERR_BAD_ARG, "drhip_comm_init_rank: bad rank/nranks/id");
  comm_release(*s);
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  ncclComm_t c;
  DRHIP_CHECK_NCCL(ncclCommInitRank(&c, nranks, u, rank));
  s->comm = c;
  return DRHIP_OK;
}

int drhip_comm_init_all(void) {
  const int p = num_segments();
  if (!p) return set_error(DRHIP_ERR_NOT_INIT, "drhip_init not called");
  std::vector<int> devs(p);
  for (int i = 0; i < p; i++) {
    devs[i] = segment(i)->device;
    for (int j = 0; j < i; j++)
      if (devs[j] == devs[i])
        return set_error(DRHIP_ERR_UNSUPPORTED, "drhip_comm_init_all: segments share a device (RCCL needs one rank per GPU)");
  }
  for (int i = 0; i < p; i++) comm_release(*segment(i));
  std::vector<ncclComm_t> c(p);
  DRHIP_CHECK_NCCL(ncclCommInitAll(c.data(), p, devs.data()));
  for (int i = 0; i < p; i++) segment(i)->comm = c[i];
  return DRHIP_OK;
}

int drhip_comm_destroy(int seg) {
  DRHIP_GET_SEG(s, seg);
  comm_release(*s);
  return DRHIP_OK;
}

int drhip_comm_rank(int seg, int *rank, int *nranks) {
  DRHIP_GET_COMM(s, seg, c);
  if (!rank || !nranks) return set_error(DRHIP_ERR_BAD_ARG, "drhip_comm_rank: null");
  DRHIP_CHECK_NCCL(ncclCommUserRank(c, rank));
  DRHIP_CHECK_NCCL(ncclCommCount(c, nranks));
  return DRHIP_OK;
}

int drhip_comm_group_start(void) {
  DRHIP_CHECK_NCCL(ncclGroupStart());
  return DRHIP_OK;
}

int drhip_comm_group_end(void) {
  DRHIP_CHECK_NCCL(ncclGroupEnd());
  return DRHIP_OK;
}

int drhip_allreduce(int seg, int dtype, int op, const void *send, void *recv, size_t n) {
  DRHIP_GET_COMM(s, seg, c);
  ncclDataType_t t;
  ncclRedOp_t o;
  if (!nccl_dtype(dtype, &t) || !nccl_op(op, &o)) return set_error(DRHIP_ERR_BAD_ARG, "drhip_allreduce: dtype/op");
  if (n && (!send || !recv)) return set_error(DRHIP_ERR_BAD_ARG, "drhip_allreduce: null");
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  DRHIP_CHECK_NCCL(ncclAllReduce(send, recv, n, t, o, c, s->stream));
  return DRHIP_OK;
}

int drhip_allgather(int seg, const void *send, void *recv, size_t bytes) {
  DRHIP_GET_COMM(s, seg, c);
  if (bytes && (!send || !recv)) return set_error(DRHIP_ERR_BAD_ARG, "drhip_allgather: null");
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  DRHIP_CHECK_NCCL(ncclAllGather(send, recv, bytes, ncclInt8, c, s->stream));
  return DRHIP_OK;
}

int drhip_gather(int seg, const void *send, void *recv, size_t bytes, int root) {
  DRHIP_GET_COMM(s, seg, c);
  int rank = 0, nranks = 0;
  DRHIP_CHECK_NCCL(ncclCommUserRank(c, &rank));
  DRHIP_CHECK_NCCL(ncclCommCount(c, &nranks));
  if (root < 0 || root >= nranks) return set_error(DRHIP_ERR_BAD_ARG, "drhip_gather: root");
  if (bytes && (!send || (rank == root && !recv))) return set_error(DRHIP_ERR_BAD_ARG, "drhip_gather: null");
  if (!bytes) return DRHIP_OK;
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  DRHIP_CHECK_NCCL(ncclGroupStart());
  if (rank == root)
    for (int r = 0; r < nranks; r++)
      DRHIP_CHECK_NCCL(ncclRecv((char *)recv + (size_t)r * bytes, bytes, ncclInt8, r, c, s->stream));
  DRHIP_CHECK_NCCL(ncclSend(send, bytes, ncclInt8, root, c, s->stream));
  DRHIP_CHECK_NCCL(ncclGroupEnd());
  return DRHIP_OK;
}

int drhip_alltoallv(int seg, const void *send, const size_t *send_bytes, const size_t *send_off, void *recv,
                    const size_t *recv_bytes, const size_t *recv_off) {
  DRHIP_GET_COMM(s, seg, c);
  if (!send_bytes || !send_off || !recv_bytes || !recv_off)
    return set_error(DRHIP_ERR_BAD_ARG, "drhip_alltoallv: null counts/offsets");
  int nranks = 0;
  DRHIP_CHECK_NCCL(ncclCommCount(c, &nranks));
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  DRHIP_CHECK_NCCL(ncclGroupStart());
  for (int r = 0; r < nranks; r++) {
    if (send_bytes[r])
      DRHIP_CHECK_NCCL(ncclSend((const char *)send + send_off[r], send_bytes[r], ncclInt8, r, c, s->stream));
    if (recv_bytes[r])
      DRHIP_CHECK_NCCL(ncclRecv((char *)recv + recv_off[r], recv_bytes[r], ncclInt8, r, c, s->stream));
  }
  DRHIP_CHECK_NCCL(ncclGroupEnd());
  return DRHIP_OK;
}

int drhip_halo_exchange(int seg, void *buf, size_t n_owned, size_t cell_bytes, size_t prev, size_t next,
                        int periodic) {
  DRHIP_GET_COMM(s, seg, c);
  if (prev != next) return set_error(DRHIP_ERR_UNSUPPORTED, "drhip_halo_exchange: prev != next (see drhip.h)");
  if (!prev || !cell_bytes) return DRHIP_OK;
  if (!buf) return set_error(DRHIP_ERR_BAD_ARG, "drhip_halo_exchange: null");
  // span_halo's check (halo.hpp:355): size >= prev + next + max(prev, next)
  if (n_owned < prev) return set_error(DRHIP_ERR_BAD_ARG, "drhip_halo_exchange: owned part shorter than the halo");
  int rank = 0, nranks = 0;
  DRHIP_CHECK_NCCL(ncclCommUserRank(c, &rank));
  DRHIP_CHECK_NCCL(ncclCommCount(c, &nranks));
  // the span_halo message list (dr/details/halo_plan.hpp): sends [reverse
  // to rank-1, forward to rank+1], then receives [from rank+1 into the next
  // halo, from rank-1 into the prev halo] -- RCCL matches a peer's sends to
  // our receives in order, so a peer that is both neighbours (2 ranks
  // periodic, or itself) pairs its reverse message with our next halo and
  // its forward message with our prev halo
  char *b = (char *)buf;
  DRHIP_CHECK_HIP(hipSetDevice(s->device));
  DRHIP_CHECK_NCCL(ncclGroupStart());
  for (const auto &m : dr_plan::halo_messages(rank, nranks, n_owned, prev, next, periodic != 0)) {
    char *p = b + m.cell_off * cell_bytes;
    if (m.send) DRHIP_CHECK_NCCL(ncclSend(p, m.cells * cell_bytes, ncclInt8, m.peer, c, s->stream));
    else DRHIP_CHECK_NCCL(ncclRecv(p, m.cells * cell_bytes, ncclInt8, m.peer, c, s->stream));
  }
  DRHIP_CHECK_NCCL(ncclGroupEnd());
  return DRHIP_OK;
}

} // extern "C"
