// Test double of the RCCL API subset libcfa's cfa_comm.cpp uses (CPU build, test only).
// tests/native/rccl_stub/rccl_stub.cpp records every call per communicator so that
// tests/test_comm_stub.py can check the exact ncclGroupStart / ncclSend / ncclRecv / ncclGroupEnd
// sequence libcfa issues for a routed halo plan, without a GPU or RCCL.
#pragma once
#include <stddef.h>

#include "hip/hip_runtime.h"

typedef struct ncclStubComm* ncclComm_t;
typedef enum { ncclSuccess = 0, ncclInvalidArgument = 4 } ncclResult_t;
typedef enum { ncclFloat32 = 7 } ncclDataType_t;
typedef enum { ncclSum = 0 } ncclRedOp_t;
typedef struct {
  char internal[128];
} ncclUniqueId;

extern "C" {
ncclResult_t ncclGetVersion(int* version);
ncclResult_t ncclGetUniqueId(ncclUniqueId* id);
ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank);
ncclResult_t ncclCommDestroy(ncclComm_t comm);
ncclResult_t ncclCommCount(ncclComm_t comm, int* count);
ncclResult_t ncclGroupStart();
ncclResult_t ncclGroupEnd();
ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm,
                      hipStream_t stream);
ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm,
                      hipStream_t stream);
ncclResult_t ncclAllReduce(const void* send, void* recv, size_t count, ncclDataType_t type, ncclRedOp_t op,
                           ncclComm_t comm, hipStream_t stream);
ncclResult_t ncclReduce(const void* send, void* recv, size_t count, ncclDataType_t type, ncclRedOp_t op,
                        int root, ncclComm_t comm, hipStream_t stream);
const char* ncclGetErrorString(ncclResult_t r);
const char* ncclGetLastError(ncclComm_t comm);
}
