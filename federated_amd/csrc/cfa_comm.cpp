// cfa_comm.cpp — RCCL (over xGMI) transport for sharded CFA populations, one process per GPU.
//
// The reference moves neighbour models between simulated devices as files on a shared
// directory (TF1/consensus/cfa.py:119-130 polls datamat{j}_{e-1}.mat; TF2 consensus_v3.py:82-141
// polls results/dump_train_model{j}.npy). When the population is sharded over the GPUs of one
// node, the only cross-shard traffic of a consensus round is the set of boundary buckets a
// rank's devices need from the neighbouring ranks: a grouped point-to-point halo exchange.
// FedAvg / parameter-split sums map to all-reduce / reduce of pre-scaled buckets.
//
// Communicators are explicit objects created and destroyed by the caller; the library keeps
// no global state. Collectives are enqueued on the caller's stream.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>

#include "cfa_engine.h"

// Defined in cfa_mix.hip: records the thread-local message cfa_last_error() returns.
extern "C" void cfa_internal_set_error(const char* msg);

static int comm_fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
static int comm_fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  cfa_internal_set_error(buf);
  return code;
}

// RCCL's own text for the last failure (ncclGetLastError: the warning it logged, e.g. which
// transport or IPC call refused), so a failure on a node this build never ran on says why.
static const char* rccl_detail() {
  const char* d = ncclGetLastError(nullptr);
  return d ? d : "";
}

#define CFA_NCCL_CHECK(expr)                                                               \
  do {                                                                                     \
    ncclResult_t r_ = (expr);                                                              \
    if (r_ != ncclSuccess)                                                                 \
      return comm_fail(CFA_E_RCCL, "%s failed: %s [rccl: %s]", #expr, ncclGetErrorString(r_), \
                       rccl_detail());                                                      \
  } while (0)

static_assert(sizeof(ncclUniqueId) == CFA_UNIQUE_ID_BYTES, "unique id size");

extern "C" int cfa_rccl_version(int* version) {
  if (!version) return comm_fail(CFA_E_INVALID, "null version");
  CFA_NCCL_CHECK(ncclGetVersion(version));
  return CFA_OK;
}

extern "C" int cfa_comm_unique_id(void* id) {
  if (!id) return comm_fail(CFA_E_INVALID, "null unique-id buffer");
  ncclUniqueId uid;
  CFA_NCCL_CHECK(ncclGetUniqueId(&uid));
  memcpy(id, &uid, sizeof(uid));
  return CFA_OK;
}

extern "C" int cfa_comm_init(void** comm, int rank, int nranks, const void* id, int device) {
  if (!comm || !id) return comm_fail(CFA_E_INVALID, "null comm/id");
  if (nranks < 1 || rank < 0 || rank >= nranks)
    return comm_fail(CFA_E_INVALID, "bad rank %d of %d", rank, nranks);
  hipError_t he = hipSetDevice(device);
  if (he != hipSuccess)
    return comm_fail(CFA_E_HIP, "hipSetDevice(%d): %s", device, hipGetErrorString(he));
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  ncclComm_t c = nullptr;
  CFA_NCCL_CHECK(ncclCommInitRank(&c, nranks, uid, rank));
  *comm = c;
  return CFA_OK;
}

extern "C" int cfa_comm_destroy(void* comm) {
  if (!comm) return CFA_OK;
  CFA_NCCL_CHECK(ncclCommDestroy(static_cast<ncclComm_t>(comm)));
  return CFA_OK;
}

extern "C" int cfa_halo_exchange_f32(void* comm, const float* const* send_bufs,
                                     const int* send_peers, int nsend, float* const* recv_bufs,
                                     const int* recv_peers, int nrecv, size_t P, void* stream) {
  if (!comm) return comm_fail(CFA_E_INVALID, "null communicator");
  if (nsend < 0 || nrecv < 0) return comm_fail(CFA_E_INVALID, "negative transfer count");
  if ((nsend && (!send_bufs || !send_peers)) || (nrecv && (!recv_bufs || !recv_peers)))
    return comm_fail(CFA_E_INVALID, "null transfer table");
  if (P == 0 || (nsend == 0 && nrecv == 0)) return CFA_OK;
  ncclComm_t c = static_cast<ncclComm_t>(comm);
  hipStream_t st = static_cast<hipStream_t>(stream);
  CFA_NCCL_CHECK(ncclGroupStart());
  for (int i = 0; i < nsend; ++i) {
    ncclResult_t r = ncclSend(send_bufs[i], P, ncclFloat32, send_peers[i], c, st);
    if (r != ncclSuccess) {
      ncclGroupEnd();
      return comm_fail(CFA_E_RCCL, "ncclSend to %d: %s [rccl: %s]", send_peers[i], ncclGetErrorString(r),
                       rccl_detail());
    }
  }
  for (int i = 0; i < nrecv; ++i) {
    ncclResult_t r = ncclRecv(recv_bufs[i], P, ncclFloat32, recv_peers[i], c, st);
    if (r != ncclSuccess) {
      ncclGroupEnd();
      return comm_fail(CFA_E_RCCL, "ncclRecv from %d: %s [rccl: %s]", recv_peers[i], ncclGetErrorString(r),
                       rccl_detail());
    }
  }
  CFA_NCCL_CHECK(ncclGroupEnd());
  return CFA_OK;
}

extern "C" int cfa_p2p_group_f32(void* comm, const float* const* send_bufs, const size_t* send_counts,
                                 const int* send_peers, int nsend, float* const* recv_bufs,
                                 const size_t* recv_counts, const int* recv_peers, int nrecv,
                                 void* stream) {
  if (!comm) return comm_fail(CFA_E_INVALID, "null communicator");
  if (nsend < 0 || nrecv < 0) return comm_fail(CFA_E_INVALID, "negative transfer count");
  if ((nsend && (!send_bufs || !send_counts || !send_peers)) ||
      (nrecv && (!recv_bufs || !recv_counts || !recv_peers)))
    return comm_fail(CFA_E_INVALID, "null transfer table");
  if (nsend == 0 && nrecv == 0) return CFA_OK;
  ncclComm_t c = static_cast<ncclComm_t>(comm);
  int nranks = 0;
  CFA_NCCL_CHECK(ncclCommCount(c, &nranks));
  for (int i = 0; i < nsend; ++i)
    if (send_peers[i] < 0 || send_peers[i] >= nranks || (send_counts[i] && !send_bufs[i]))
      return comm_fail(CFA_E_INVALID, "send %d: bad peer %d or null buffer", i, send_peers[i]);
  for (int i = 0; i < nrecv; ++i)
    if (recv_peers[i] < 0 || recv_peers[i] >= nranks || (recv_counts[i] && !recv_bufs[i]))
      return comm_fail(CFA_E_INVALID, "recv %d: bad peer %d or null buffer", i, recv_peers[i]);
  hipStream_t st = static_cast<hipStream_t>(stream);
  CFA_NCCL_CHECK(ncclGroupStart());
  for (int i = 0; i < nsend; ++i) {
    if (!send_counts[i]) continue;
    ncclResult_t r = ncclSend(send_bufs[i], send_counts[i], ncclFloat32, send_peers[i], c, st);
    if (r != ncclSuccess) {
      ncclGroupEnd();
      return comm_fail(CFA_E_RCCL, "ncclSend to %d: %s [rccl: %s]", send_peers[i], ncclGetErrorString(r),
                       rccl_detail());
    }
  }
  for (int i = 0; i < nrecv; ++i) {
    if (!recv_counts[i]) continue;
    ncclResult_t r = ncclRecv(recv_bufs[i], recv_counts[i], ncclFloat32, recv_peers[i], c, st);
    if (r != ncclSuccess) {
      ncclGroupEnd();
      return comm_fail(CFA_E_RCCL, "ncclRecv from %d: %s [rccl: %s]", recv_peers[i], ncclGetErrorString(r),
                       rccl_detail());
    }
  }
  CFA_NCCL_CHECK(ncclGroupEnd());
  return CFA_OK;
}

extern "C" int cfa_allreduce_sum_f32(void* comm, const float* send, float* recv, size_t count,
                                     void* stream) {
  if (!comm) return comm_fail(CFA_E_INVALID, "null communicator");
  if (count == 0) return CFA_OK;
  if (!send || !recv) return comm_fail(CFA_E_INVALID, "null buffer");
  CFA_NCCL_CHECK(ncclAllReduce(send, recv, count, ncclFloat32, ncclSum,
                               static_cast<ncclComm_t>(comm), static_cast<hipStream_t>(stream)));
  return CFA_OK;
}

extern "C" int cfa_reduce_sum_f32(void* comm, const float* send, float* recv, size_t count,
                                  int root, void* stream) {
  if (!comm) return comm_fail(CFA_E_INVALID, "null communicator");
  if (count == 0) return CFA_OK;
  if (!send) return comm_fail(CFA_E_INVALID, "null buffer");
  CFA_NCCL_CHECK(ncclReduce(send, recv, count, ncclFloat32, ncclSum, root,
                            static_cast<ncclComm_t>(comm), static_cast<hipStream_t>(stream)));
  return CFA_OK;
}
