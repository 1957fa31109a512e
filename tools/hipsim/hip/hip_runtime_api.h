// Host-only simulation of the few HIP runtime calls csrc/ingest_pipe.cpp makes,
// for tools/ingest_pipe_stress.cpp: the pipe's threading (copy workers, issuer,
// slot states, backpressure) runs under ThreadSanitizer / AddressSanitizer on a
// machine without a GPU.  Streams execute every operation synchronously on the
// calling thread, in call order, so "device" memory is plain host memory and an
// event is complete once recorded.  Test tooling only: never part of a build of
// libfedavg_hip.so.
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef int hipError_t;
typedef struct ihipStream_t* hipStream_t;
typedef struct ihipEvent_t* hipEvent_t;
enum { hipSuccess = 0, hipErrorOutOfMemory = 2 };
enum hipMemcpyKind { hipMemcpyHostToDevice = 1 };
#define hipStreamNonBlocking 1
#define hipHostMallocDefault 0
#define hipEventDisableTiming 2

inline const char* hipGetErrorString(hipError_t e) { return e ? "simulated error" : "no error"; }
inline hipError_t hipGetLastError() { return hipSuccess; }
inline hipError_t hipGetDevice(int* d) { *d = 0; return hipSuccess; }
inline hipError_t hipSetDevice(int) { return hipSuccess; }
inline hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned) {
    *s = reinterpret_cast<hipStream_t>(malloc(1));
    return hipSuccess;
}
inline hipError_t hipStreamDestroy(hipStream_t s) { free(s); return hipSuccess; }
inline hipError_t hipHostMalloc(void** p, size_t n, unsigned) { *p = malloc(n); return *p ? hipSuccess : hipErrorOutOfMemory; }
inline hipError_t hipHostFree(void* p) { free(p); return hipSuccess; }
inline hipError_t hipMalloc(void** p, size_t n) { *p = malloc(n); return *p ? hipSuccess : hipErrorOutOfMemory; }
inline hipError_t hipFree(void* p) { free(p); return hipSuccess; }
inline hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind, hipStream_t) {
    memcpy(d, s, n);
    return hipSuccess;
}
inline hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) {
    *e = reinterpret_cast<hipEvent_t>(malloc(1));
    return hipSuccess;
}
inline hipError_t hipEventDestroy(hipEvent_t e) { free(e); return hipSuccess; }
inline hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipSuccess; }
inline hipError_t hipStreamWaitEvent(hipStream_t, hipEvent_t, unsigned) { return hipSuccess; }
inline hipError_t hipEventSynchronize(hipEvent_t) { return hipSuccess; }
