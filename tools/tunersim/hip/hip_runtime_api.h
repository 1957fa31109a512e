// A simulated HIP runtime for the host stress test of csrc/tuner.hpp
// (tools/tuner_stress.cpp): streams carry a virtual clock that the test's
// "launches" advance, events take the clock of their stream when recorded,
// and an event reports hipErrorNotReady for its first few queries (work still
// in flight).  Only what tuner.hpp calls.
#pragma once
#include <atomic>
#include <cstdlib>

typedef enum hipError_t {
    hipSuccess = 0,
    hipErrorOutOfMemory = 2,
    hipErrorInvalidValue = 1,
    hipErrorNotReady = 600,
} hipError_t;
typedef enum hipStreamCaptureStatus {
    hipStreamCaptureStatusNone = 0,
    hipStreamCaptureStatusActive = 1,
} hipStreamCaptureStatus;

struct SimStream {
    double clock = 0.0;  // ms
    bool capturing = false;
    int device = 0;
};
struct SimEvent {
    double t = 0.0;
    bool recorded = false;
    int queries_left = 0;
};
typedef SimStream* hipStream_t;
typedef SimEvent* hipEvent_t;

namespace tunersim {
inline std::atomic<int>& not_ready_queries() {
    static std::atomic<int> n{2};
    return n;
}
inline std::atomic<long>& live_events() {
    static std::atomic<long> n{0};
    return n;
}
inline int& current_device() {
    static thread_local int d = 0;
    return d;
}
}  // namespace tunersim

inline hipError_t hipGetLastError() { return hipSuccess; }
inline hipError_t hipGetDevice(int* d) {
    *d = tunersim::current_device();
    return hipSuccess;
}
inline hipError_t hipEventCreate(hipEvent_t* e) {
    *e = new SimEvent();
    tunersim::live_events()++;
    return hipSuccess;
}
inline hipError_t hipEventDestroy(hipEvent_t e) {
    delete e;
    tunersim::live_events()--;
    return hipSuccess;
}
inline hipError_t hipEventRecord(hipEvent_t e, hipStream_t s) {
    e->t = s->clock;
    e->recorded = true;
    e->queries_left = tunersim::not_ready_queries().load();
    return hipSuccess;
}
inline hipError_t hipEventQuery(hipEvent_t e) {
    if (!e->recorded) return hipSuccess;
    if (e->queries_left > 0) {
        --e->queries_left;
        return hipErrorNotReady;
    }
    return hipSuccess;
}
inline hipError_t hipEventElapsedTime(float* ms, hipEvent_t a, hipEvent_t b) {
    if (!a->recorded || !b->recorded) return hipErrorInvalidValue;
    *ms = (float)(b->t - a->t);
    return hipSuccess;
}
inline hipError_t hipStreamIsCapturing(hipStream_t s, hipStreamCaptureStatus* st) {
    *st = s->capturing ? hipStreamCaptureStatusActive : hipStreamCaptureStatusNone;
    return hipSuccess;
}
