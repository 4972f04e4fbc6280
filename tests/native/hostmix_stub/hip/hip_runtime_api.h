// Test double of the HIP runtime subset csrc/cfa_hostmix.cpp uses (CPU build, test only): streams
// are host worker threads that run enqueued work in order, events are tickets on a stream, so the
// chunk pipeline's ordering (pack -> kernel -> event -> unpack) runs asynchronously under
// ThreadSanitizer. See tests/native/hostmix_stub/hostmix_stub.cpp.
#pragma once
typedef struct StubStream* hipStream_t;
typedef struct StubEvent* hipEvent_t;
typedef enum { hipSuccess = 0, hipErrorNotReady = 600, hipErrorInvalidValue = 1 } hipError_t;
#define hipEventDisableTiming 0x2
extern "C" {
hipError_t hipEventCreateWithFlags(hipEvent_t* ev, unsigned flags);
hipError_t hipEventRecord(hipEvent_t ev, hipStream_t st);
hipError_t hipEventQuery(hipEvent_t ev);
hipError_t hipEventSynchronize(hipEvent_t ev);
hipError_t hipEventDestroy(hipEvent_t ev);
hipError_t hipStreamSynchronize(hipStream_t st);
}
