// Test double of the HIP runtime subset cfa_comm.cpp uses (CPU build, test only).
#pragma once
typedef struct ihipStream_t* hipStream_t;
typedef enum { hipSuccess = 0, hipErrorInvalidDevice = 101 } hipError_t;
extern "C" {
hipError_t hipSetDevice(int device);
const char* hipGetErrorString(hipError_t e);
}
