// Recording implementation of the RCCL / HIP test doubles (see rccl/rccl.h). Each communicator
// keeps a text log, one line per call:
//   start | send <peer> <count> <ptr> <stream> | recv <peer> <count> <ptr> <stream> | end
//   allreduce <count> <send> <recv> | reduce <root> <count> <send> <recv>
// A group call outside ncclGroupStart/End is refused (ncclInvalidArgument), like a misuse RCCL
// would not pair.
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>

#include "rccl/rccl.h"

struct ncclStubComm {
  int rank, nranks;
  std::string log;
};

namespace {
thread_local int group_depth = 0;
thread_local ncclStubComm* group_comm = nullptr;
std::mutex mu;
thread_local std::string last_error;

void append(ncclStubComm* c, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
void append(ncclStubComm* c, const char* fmt, ...) {
  char buf[256];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  std::lock_guard<std::mutex> g(mu);
  c->log += buf;
  c->log += '\n';
}
}  // namespace

extern "C" {
hipError_t hipSetDevice(int device) { return device >= 0 ? hipSuccess : hipErrorInvalidDevice; }
const char* hipGetErrorString(hipError_t e) { return e == hipSuccess ? "hipSuccess" : "hipErrorInvalidDevice"; }

ncclResult_t ncclGetVersion(int* v) {
  *v = 99999;
  return ncclSuccess;
}
ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  for (int i = 0; i < 128; ++i) id->internal[i] = char(i);
  return ncclSuccess;
}
ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId, int rank) {
  if (rank < 0 || rank >= nranks) return ncclInvalidArgument;
  *comm = new ncclStubComm{rank, nranks, std::string()};
  return ncclSuccess;
}
ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  delete comm;
  return ncclSuccess;
}
ncclResult_t ncclCommCount(ncclComm_t comm, int* count) {
  *count = comm->nranks;
  return ncclSuccess;
}
ncclResult_t ncclGroupStart() {
  if (group_depth++ == 0) group_comm = nullptr;
  return ncclSuccess;
}
ncclResult_t ncclGroupEnd() {
  if (group_depth <= 0) return ncclInvalidArgument;
  if (--group_depth == 0 && group_comm) append(group_comm, "end");
  return ncclSuccess;
}
static ncclResult_t p2p(const char* op, const void* buf, size_t count, ncclDataType_t type, int peer,
                        ncclComm_t comm, hipStream_t stream) {
  if (group_depth <= 0 || type != ncclFloat32 || peer < 0 || peer >= comm->nranks || count == 0)
    return ncclInvalidArgument;
  if (!group_comm) {
    group_comm = comm;
    append(comm, "start");
  } else if (group_comm != comm) {
    return ncclInvalidArgument;  // one communicator per group in libcfa
  }
  append(comm, "%s %d %zu %llu %llu", op, peer, count, (unsigned long long)(uintptr_t)buf,
         (unsigned long long)(uintptr_t)stream);
  return ncclSuccess;
}
ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm,
                      hipStream_t stream) {
  return p2p("send", buf, count, type, peer, comm, stream);
}
ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm,
                      hipStream_t stream) {
  return p2p("recv", buf, count, type, peer, comm, stream);
}
ncclResult_t ncclAllReduce(const void* send, void* recv, size_t count, ncclDataType_t, ncclRedOp_t,
                           ncclComm_t comm, hipStream_t) {
  append(comm, "allreduce %zu %llu %llu", count, (unsigned long long)(uintptr_t)send,
         (unsigned long long)(uintptr_t)recv);
  return ncclSuccess;
}
ncclResult_t ncclReduce(const void* send, void* recv, size_t count, ncclDataType_t, ncclRedOp_t, int root,
                        ncclComm_t comm, hipStream_t) {
  append(comm, "reduce %d %zu %llu %llu", root, count, (unsigned long long)(uintptr_t)send,
         (unsigned long long)(uintptr_t)recv);
  return ncclSuccess;
}
const char* ncclGetErrorString(ncclResult_t r) { return r == ncclSuccess ? "ncclSuccess" : "ncclInvalidArgument"; }
const char* ncclGetLastError(ncclComm_t) { return "stub: peer refused"; }

// libcfa's error hook (cfa_mix.hip in the real library)
void cfa_internal_set_error(const char* msg) { last_error = msg ? msg : ""; }
const char* stub_last_error() { return last_error.c_str(); }

// The call log of one communicator, and clearing it.
size_t stub_log(void* comm, char* dst, size_t cap) {
  std::lock_guard<std::mutex> g(mu);
  const std::string& s = static_cast<ncclStubComm*>(comm)->log;
  if (dst && cap) {
    const size_t n = s.size() < cap - 1 ? s.size() : cap - 1;
    memcpy(dst, s.data(), n);
    dst[n] = 0;
  }
  return s.size();
}
void stub_clear(void* comm) {
  std::lock_guard<std::mutex> g(mu);
  static_cast<ncclStubComm*>(comm)->log.clear();
}
}
