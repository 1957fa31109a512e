// libfedavg_hip.so — MI355X (gfx950, CDNA4) FedAvg / FedLesScan aggregation:
// the product C-ABI (include/fedavg_hip.h).  Kernels: fold_kernels.hpp.
//
// Reference interface replaced (all numpy on one CPU core):
//   fedless/aggregator/fed_avg_aggregator.py:24-42        FedAvgAggregator._aggregate
//   fedless/aggregator/stall_aware_aggregation.py:42-67   StallAwareAggregator._aggregate
// Kernel variants, the synthetic input generator and the read-sweep
// calibration kernel live in libfedavg_hip_bench.so (fedavg_bench.hip), which
// bench.py and the variant tests load; nothing here depends on them.
#include "fold_kernels.hpp"
#include "peer_exchange.hpp"

#include <mutex>

namespace {

// ---- per-client factors handed over in HOST memory (the *_hostf entries) ----
// The reference's weights are Python numbers; its caller has them on the host.
// A ring of slots per device, each a page-locked buffer, a device buffer and
// two events: the factors are copied into the slot's pinned buffer and travel
// in one async H2D on the ring's own staging stream, so the copy (a small
// blit kernel) runs beside whatever the caller's stream is still doing, and
// the caller's stream waits for it (an event: no dispatch of its own in front
// of the fold -- on the fold's stream it cost a kernel and ~15 us of dispatch
// gaps per step, profiles/r06_peer/); the fold reads the device copy, and an
// event recorded after the fold guards the slot, which is reused only after
// that fold has completed.  One C call instead of an allocation, a copy and an
// event from the host language per fold.
constexpr int kFactorSlots = 8;
struct FactorSlot {
    float* host = nullptr;
    float* dev = nullptr;
    size_t cap = 0;  // floats
    hipEvent_t ready = nullptr;  // the slot's H2D has completed (staging stream)
    hipEvent_t done = nullptr;   // the fold that read the slot has completed (caller's stream)
    bool pending = false;
};
struct FactorRing {
    std::mutex mu;
    FactorSlot slot[kFactorSlots];
    int next = 0;
    hipStream_t stage = nullptr;  // the H2D copies' stream (created on first use, per device)
};
FactorRing g_factor_rings[16];

// Under a HIP graph capture the ring cannot be used (waiting for a slot's
// event is not allowed while a stream captures, and a captured copy would read
// the slot again at every replay, after later calls rewrote it), and the
// library owns no memory that lives as long as a graph: the *_hostf entries
// refuse capture, and a capturing caller stages the factors with
// fa_factors_fill -- fill kernels whose arguments carry the values, captured by
// value -- into memory the graph owns, then calls the device-factor entry.
// (Round 6 staged them here in a stream-ordered allocation of the graph; a
// replay inside the full GPU suite read part of it as zeros.)
constexpr int kFillFloats = 256;
struct FillArgs {
    float v[kFillFloats];
};
__global__ __launch_bounds__(64) void k_fill_factors(float* dst, FillArgs f, int n) {
    for (int i = threadIdx.x; i < n; i += 64) dst[i] = f.v[i];
}

// Stage a[0..N) (and s[0..N) when s != NULL) and run launch(a_dev, s_dev) on
// `stream` with the ring slot held; the slot's event is recorded after it.
template <class Launch>
int with_host_factors(const float* a, const float* s, int64_t N, void* stream, Launch launch) {
    if (N <= 0) return launch((const float*)nullptr, (const float*)nullptr);  // the entry's own checks report
    if (!a) return fail(FA_ERR_ARG, "null host factor pointer");
    {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing((hipStream_t)stream, &cs) != hipSuccess) (void)hipGetLastError();
        else if (cs != hipStreamCaptureStatusNone)
            return fail(FA_ERR_ARG, "host factors under graph capture: stage them with fa_factors_fill into memory "
                                    "the graph owns and call the device-factor entry");
    }
    // the slot (and its device buffer) of the GPU that owns the stream, not of
    // the calling thread's current device
    StreamDevice on_stream_device(stream);
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return fail(FA_ERR_HIP, "hipGetDevice");
    FactorRing& R = g_factor_rings[dev];
    std::lock_guard<std::mutex> lk(R.mu);
    FactorSlot& S = R.slot[R.next];
    R.next = (R.next + 1) % kFactorSlots;
    hipStream_t st = (hipStream_t)stream;
    const size_t need = (size_t)N * (s ? 2 : 1);
    if (S.pending) {
        hipError_t e = hipEventSynchronize(S.done);
        if (e != hipSuccess) return fail(FA_ERR_HIP, "factor slot wait: %s", hipGetErrorString(e));
        S.pending = false;
    }
    if (need > S.cap) {
        if (S.host) (void)hipHostFree(S.host);
        if (S.dev) (void)hipFree(S.dev);
        S.host = nullptr;
        S.dev = nullptr;
        S.cap = 0;
        const size_t cap = need < 16384 ? 16384 : need;
        hipError_t e = hipHostMalloc((void**)&S.host, cap * sizeof(float), hipHostMallocDefault);
        if (e == hipSuccess) e = hipMalloc((void**)&S.dev, cap * sizeof(float));
        if (e != hipSuccess) return fail(FA_ERR_HIP, "factor slot allocation: %s", hipGetErrorString(e));
        S.cap = cap;
    }
    if (!S.done) {
        hipError_t e = hipEventCreateWithFlags(&S.done, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&S.ready, hipEventDisableTiming);
        if (e != hipSuccess) return fail(FA_ERR_HIP, "hipEventCreate: %s", hipGetErrorString(e));
    }
    if (!R.stage) {
        hipError_t e = hipStreamCreateWithFlags(&R.stage, hipStreamNonBlocking);
        if (e != hipSuccess) return fail(FA_ERR_HIP, "factor staging stream: %s", hipGetErrorString(e));
    }
    memcpy(S.host, a, (size_t)N * sizeof(float));
    if (s) memcpy(S.host + N, s, (size_t)N * sizeof(float));
    // the device buffer is free: the fold that last read it has completed (S.done, above)
    hipError_t e = hipMemcpyAsync(S.dev, S.host, need * sizeof(float), hipMemcpyHostToDevice, R.stage);
    if (e == hipSuccess) e = hipEventRecord(S.ready, R.stage);
    if (e == hipSuccess) e = hipStreamWaitEvent(st, S.ready, 0);
    if (e != hipSuccess) return fail(FA_ERR_HIP, "factor H2D: %s", hipGetErrorString(e));
    const int rc = launch((const float*)S.dev, s ? (const float*)(S.dev + N) : (const float*)nullptr);
    e = hipEventRecord(S.done, st);
    if (e != hipSuccess) return fail(FA_ERR_HIP, "hipEventRecord: %s", hipGetErrorString(e));
    S.pending = true;
    return rc;
}

// One client row into a running fold with scalar factors (fa_accumulate_f32):
// acc = (first ? t : acc + t), t = fl(fl(x*a)*s).  s == 1 multiplies exactly.
__global__ __launch_bounds__(kBlock) void k_accumulate_f32(float* acc, const float* __restrict__ x, float a,
                                                            float s, int first, int64_t P) {
    const int64_t c0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * 4;
    if (c0 >= P) return;
    if (c0 + 4 <= P && aligned16(acc + c0) && aligned16(x + c0)) {
        f32x4 t = term4<true>(__builtin_nontemporal_load(reinterpret_cast<const f32x4*>(x + c0)), a, s);
        f32x4* p = reinterpret_cast<f32x4*>(acc + c0);
        *p = first ? t : add4(*p, t);
    } else {
        for (int64_t c = c0; c < P && c < c0 + 4; ++c) {
            const float t = term1<true>(x[c], a, s);
            acc[c] = first ? t : acc[c] + t;
        }
    }
}

}  // namespace

// error text for the host entries of ingest_host.cpp (another TU)
__attribute__((visibility("hidden"))) int fa_internal_fail(int code, const char* msg) { return fail(code, "%s", msg); }

// ===========================================================================
// C-ABI
// ===========================================================================
extern "C" {

int fa_abi_version(void) { return FA_ABI_VERSION; }
const char* fa_last_error(void) { return g_err; }

int fa_fedavg_f32(const float* X, int64_t N, int64_t P, int64_t ldx, const float* a, const float* s,
                  float divisor, float* out, void* stream) {
    return fold_f32_auto(X, N, P, ldx, a, s, nullptr, divisor, 1, out, stream);
}

int fa_fold_f32(const float* X, int64_t N, int64_t P, int64_t ldx, const float* a, const float* s,
                const float* acc_in, float divisor, int finalize, float* out, void* stream) {
    return fold_f32_auto(X, N, P, ldx, a, s, acc_in, divisor, finalize, out, stream);
}

int fa_accumulate_f32(float* acc, const float* x, float a, float s, int first, int64_t P, void* stream) {
    StreamDevice on_stream_device(stream);
    if (P < 0 || (P > 0 && (!acc || !x))) return fail(FA_ERR_ARG, "null acc/x or negative P");
    if (P == 0) { g_err[0] = 0; return FA_OK; }
    hipLaunchKernelGGL(k_accumulate_f32, grid_for((P + 3) / 4), dim3(kBlock), 0, (hipStream_t)stream, acc, x, a, s,
                       first, P);
    return check_launch("k_accumulate_f32");
}

int fa_finalize_f32(const float* acc, float divisor, float* out, int64_t P, void* stream) {
    return fold_f32_auto(nullptr, 0, P, P, nullptr, nullptr, acc, divisor, 1, out, stream);
}

int fa_fedavg_f32_splitn(const float* X, int64_t N, int64_t P, int64_t ldx, const float* a, const float* s,
                         float divisor, float* out, void* stream) {
    int rc = check_common(N, P, ldx, X, a, out);
    if (rc) return rc;
    if (P == 0) { g_err[0] = 0; return FA_OK; }
    if (!aligned16(X) || (ldx % 4) || !aligned16(out))
        return fail(FA_ERR_ARG, "fa_fedavg_f32_splitn needs 16-B aligned X and out and ldx %% 4 == 0");
    constexpr int NW = 8;
    const int64_t blocks = (((P + 3) >> 2) + 15) / 16;
    if (blocks > 0x7FFFFFFF / (NW * 64)) return fail(FA_ERR_ARG, "P too large for fa_fedavg_f32_splitn");
    hipStream_t st = (hipStream_t)stream;
    StreamDevice on_stream_device(stream);
    if (s)
        hipLaunchKernelGGL((k_fold_f32_splitn<NW, true>), dim3((unsigned)blocks), dim3(NW * 64), 0, st, X, N, P,
                           ldx, a, s, divisor, out);
    else
        hipLaunchKernelGGL((k_fold_f32_splitn<NW, false>), dim3((unsigned)blocks), dim3(NW * 64), 0, st, X, N, P,
                           ldx, a, s, divisor, out);
    return check_launch("k_fold_f32_splitn");
}

int fa_fedavg_f32_ptrs_aligned(const float* const* xi, int64_t N, int64_t P, const float* a, const float* s,
                               float divisor, float* out, void* stream) {
    int rc = check_common(N, P, P, xi, a, out);
    if (rc) return rc;
    if (P == 0) { g_err[0] = 0; return FA_OK; }
    if (!aligned16(out)) return fail(FA_ERR_ARG, "fa_fedavg_f32_ptrs_aligned needs a 16-B aligned out");
    hipStream_t st = (hipStream_t)stream;
    StreamDevice on_stream_device(stream);
    const PtrsForm policy = pick_ptrs(N, P);
    const bool sc = s != nullptr;
    rc = g_tuner.run(kTunePtrs, N, P, P, sc, (int)policy, (double)N * (double)P * 4.0, st,
                     [&](std::vector<int>& c) { ptrs_candidates(N, P, (int)policy, c); },
                     [&](int form) { return launch_ptrs_form((PtrsForm)form, st, xi, N, P, a, s, divisor, out); });
    if (rc) return rc;
    return check_launch("fa_fedavg_f32_ptrs_aligned");
}

int fa_fedavg_f32_ptrs(const float* const* xi, int64_t N, int64_t P, const float* a, const float* s,
                       float divisor, float* out, void* stream) {
    int rc = check_common(N, P, P, xi, a, out);
    if (rc) return rc;
    if (P == 0) { g_err[0] = 0; return FA_OK; }
    hipStream_t st = (hipStream_t)stream;
    StreamDevice on_stream_device(stream);
    // rows at any 4-B offset.  Narrow models: the LDS-staged fold with 4-byte
    // loads and row bases from the table; otherwise one lane per column, row
    // bases wave-uniform.  (The round-2 kernel, a lane per 4 columns with a
    // per-row alignment test, ran 7-10x slower on unaligned rows:
    // profiles/r02_lds/dw_ptrs.log.)
    const int64_t nq = P >> 2;
    const float* X = (const float*)xi;
    const bool sc = s != nullptr;
    if (nq > 0 && nq < (1 << 13))
        rc = launch_lds_flags<2, 32, 16, 4, false, true, true, 4, true>(st, sc, false, true, X, N, P, P, a, s, nullptr,
                                                                        divisor, out);
    else if (nq > 0 && N >= 256 && nq < (1 << 16))
        rc = launch_lds_flags<4, 32, 24, 2, false, true, true, 0, true>(st, sc, false, true, X, N, P, P, a, s, nullptr,
                                                                        divisor, out);
    else if (sc)
        hipLaunchKernelGGL(k_fold_f32_rows_scalar<true>, grid_for(P), dim3(kBlock), 0, st, xi, N, P, a, s, divisor,
                           out);
    else
        hipLaunchKernelGGL(k_fold_f32_rows_scalar<false>, grid_for(P), dim3(kBlock), 0, st, xi, N, P, a, s, divisor,
                           out);
    if (rc) return rc;
    return check_launch("fa_fedavg_f32_ptrs");
}

int fa_fedavg_bf16(const uint16_t* X, int64_t N, int64_t P, int64_t ldx, const float* a, const float* s,
                   float divisor, float* out_f32, uint16_t* out_bf16, void* stream) {
    return bf16_auto(X, N, P, ldx, a, s, divisor, out_f32, out_bf16, stream);
}

// ---- one launch per exchange step (struct fa_rounds: peer_exchange.hpp) ------

int fa_rounds_create(fa_rounds** r, int device) {
    if (!r) return fail(FA_ERR_ARG, "fa_rounds_create: null handle");
    *r = nullptr;
    fa_rounds* o = new fa_rounds();
    const int rc = rounds_state_init(*o, device);
    if (rc) {
        delete o;
        return rc;
    }
    *r = o;
    g_err[0] = 0;
    return FA_OK;
}

int fa_rounds_destroy(fa_rounds* r) {
    if (!r) return FA_OK;
    rounds_state_free(*r);
    delete r;
    return FA_OK;
}

int fa_fedavg_bf16_rounds(fa_rounds* r, const uint16_t* X, int64_t N, int64_t ldx, const float* a, const float* s,
                          float divisor, float* out_f32, uint16_t* out_bf16, int rounds, const int64_t* offsets,
                          const int64_t* out_offsets, void* stream) {
    if (!r) return fail(FA_ERR_ARG, "null fa_rounds");
    StreamDevice on_stream_device(stream);
    return launch_step(*r, pick_step(true), (hipStream_t)stream, X, N, ldx, a, s, divisor, out_f32, out_bf16,
                       rounds, offsets, out_offsets);
}

int fa_fedavg_f32_rounds(fa_rounds* r, const float* X, int64_t N, int64_t ldx, const float* a, const float* s,
                         float divisor, float* out, int rounds, const int64_t* offsets, const int64_t* out_offsets,
                         void* stream) {
    if (!r) return fail(FA_ERR_ARG, "null fa_rounds");
    StreamDevice on_stream_device(stream);
    return launch_step(*r, pick_step(false), (hipStream_t)stream, X, N, ldx, a, s, divisor, out, nullptr, rounds,
                       offsets, out_offsets);
}

const char* fa_rounds_form(int bf16) { return step_form_name(pick_step(bf16 != 0)); }

int fa_rounds_wait(fa_rounds* r, int round, void* stream) {
    if (!r) return fail(FA_ERR_ARG, "null fa_rounds");
    StreamDevice on_stream_device(stream);
    return rounds_wait(*r, round, (hipStream_t)stream);
}

int fa_rounds_check(fa_rounds* r) {
    if (!r) return -fail(FA_ERR_ARG, "null fa_rounds");
    return rounds_check(*r);
}

int fa_rounds_timeouts(fa_rounds* r) {
    if (!r) return -fail(FA_ERR_ARG, "null fa_rounds");
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(r->device);
    unsigned int v = 0;
    const hipError_t e = hipMemcpy(&v, r->sig + kSigTimeout, sizeof(v), hipMemcpyDeviceToHost);
    (void)hipSetDevice(prev);
    if (e != hipSuccess) return -fail(FA_ERR_HIP, "fa_rounds_timeouts: %s", hipGetErrorString(e));
    return (int)v;
}

// ---- kernel-free peer exchange ----------------------------------------------
int fa_peers_create(fa_peers** x, int device, int world, int rank, int64_t send_bytes) {
    if (!x) return fail(FA_ERR_ARG, "fa_peers_create: null handle");
    *x = nullptr;
    if (world < 1 || world > kMaxPeers || rank < 0 || rank >= world || send_bytes < 16 || send_bytes % 16)
        return fail(FA_ERR_ARG, "fa_peers_create: world %d (1..%d), rank %d, send_bytes %lld (16-B multiple)", world,
                    kMaxPeers, rank, (long long)send_bytes);
    fa_peers* o = new fa_peers();
    const int rc = peers_init(*o, device, world, rank, send_bytes);
    if (rc) {
        peers_free(*o);
        delete o;
        return rc;
    }
    *x = o;
    g_err[0] = 0;
    return FA_OK;
}

int fa_peers_destroy(fa_peers* x) {
    if (!x) return FA_OK;
    peers_free(*x);
    delete x;
    return FA_OK;
}

int fa_peers_handle_bytes(void) { return kPeerHandleBytes; }

int fa_peers_handle(fa_peers* x, void* out) {
    if (!x || !out) return fail(FA_ERR_ARG, "fa_peers_handle: null argument");
    StreamDevice on_device(nullptr);
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(x->device);
    const int rc = peers_handle(*x, out);
    (void)hipSetDevice(prev);
    if (!rc) g_err[0] = 0;
    return rc;
}

int fa_peers_open(fa_peers* x, const void* all_handles) {
    if (!x || !all_handles) return fail(FA_ERR_ARG, "fa_peers_open: null argument");
    const int rc = peers_open(*x, static_cast<const uint8_t*>(all_handles));
    if (!rc) g_err[0] = 0;
    return rc;
}

void* fa_peers_send(fa_peers* x) { return x ? peers_next_send(*x) : nullptr; }

fa_rounds* fa_peers_rounds(fa_peers* x) { return x ? &x->R : nullptr; }

int fa_peers_exchange(fa_peers* x, int rounds, const int64_t* src_offsets, void* dst, const int64_t* dst_offsets,
                      void* stream) {
    if (!x) return fail(FA_ERR_ARG, "null fa_peers");
    StreamDevice on_stream_device(stream);
    return peers_exchange(*x, rounds, src_offsets, dst, dst_offsets, (hipStream_t)stream);
}

int fa_step_lookup(const char* key) {
    if (!key) return -2;
    return g_tuner.step_lookup(std::string(key));
}

int fa_step_record(const char* key, int one_launch) {
    if (!key || !g_tuner.step_record(std::string(key), one_launch != 0))
        return fail(FA_ERR_ARG, "fa_step_record: malformed key '%s'", key ? key : "(null)");
    g_err[0] = 0;
    return FA_OK;
}

int fa_set_autotune(int mode) { return g_tuner.set_mode(mode); }
int fa_autotune_pending(void) { return g_tuner.pending(); }

const char* fa_fold_form(int kind, int64_t N, int64_t P, int64_t ldx, int scored, void* stream) {
    if ((kind != FA_FOLD_F32 && kind != FA_FOLD_BF16 && kind != FA_FOLD_F32_ROWS) || N < 1 || P < 1) return "";
    StreamDevice on_stream_device(stream);
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) {
        (void)hipGetLastError();
        return "";
    }
    const int policy = kind == FA_FOLD_F32 ? (int)pick_f32(N, P)
                       : kind == FA_FOLD_F32_ROWS ? (int)pick_ptrs(N, P) : (int)pick_bf16(N, P);
    const int tuned = g_tuner.set_mode(-1) ? g_tuner.chosen(dev, kind, N, policy, P, ldx, scored != 0) : -2;
    if (tuned == -1) return "";
    return tune_form_name(kind, tuned >= 0 ? tuned : policy);
}

int fa_tune_cache_path(const char* path) {
    g_tuner.set_cache_path(path ? std::string(path) : std::string());
    g_err[0] = 0;
    return FA_OK;
}

int64_t fa_tune_export(char* buf, int64_t cap) {
    const std::string t = g_tuner.export_text();
    if (buf && cap > 0) {
        const size_t n = t.size() < (size_t)(cap - 1) ? t.size() : (size_t)(cap - 1);
        memcpy(buf, t.data(), n);
        buf[n] = 0;
    }
    return (int64_t)t.size();
}

int fa_tune_import(const char* text) {
    if (!text) return fail(FA_ERR_ARG, "fa_tune_import: null text");
    g_err[0] = 0;
    return g_tuner.import_text(std::string(text));
}

int fa_fedavg_f64(const double* X, int64_t N, int64_t P, int64_t ldx, const double* a, const double* s,
                  double divisor, double* out, void* stream) {
    int rc = check_common(N, P, ldx, X, a, out);
    if (rc) return rc;
    if (P == 0) { g_err[0] = 0; return FA_OK; }
    hipStream_t st = (hipStream_t)stream;
    StreamDevice on_stream_device(stream);
    if (aligned16(X) && aligned16(out) && (ldx % 2 == 0)) {
        if (s)
            hipLaunchKernelGGL((k_fedavg_f64_v2<8, true>), grid_for((P >> 1) + 1), dim3(kBlock), 0, st, X, N, P,
                               ldx, a, s, divisor, out);
        else
            hipLaunchKernelGGL((k_fedavg_f64_v2<8, false>), grid_for((P >> 1) + 1), dim3(kBlock), 0, st, X, N, P,
                               ldx, a, s, divisor, out);
        return check_launch("k_fedavg_f64_v2");
    }
    if (s)
        hipLaunchKernelGGL(k_fedavg_f64<true>, grid_for(P), dim3(kBlock), 0, st, X, N, P, ldx, a, s, divisor,
                           out);
    else
        hipLaunchKernelGGL(k_fedavg_f64<false>, grid_for(P), dim3(kBlock), 0, st, X, N, P, ldx, a, s, divisor,
                           out);
    return check_launch("k_fedavg_f64");
}

int fa_fedavg_i32(const int32_t* X, int64_t N, int64_t P, int64_t ldx, const int64_t* a, double divisor,
                  double* out, void* stream) {
    int rc = check_common(N, P, ldx, X, a, out);
    if (rc) return rc;
    if (P == 0) { g_err[0] = 0; return FA_OK; }
    StreamDevice on_stream_device(stream);
    hipLaunchKernelGGL((k_fedavg_int<int32_t, uint32_t>), grid_for(P), dim3(kBlock), 0, (hipStream_t)stream,
                       X, N, P, ldx, a, divisor, out);
    return check_launch("k_fedavg_int<int32>");
}

int fa_fedavg_i64(const int64_t* X, int64_t N, int64_t P, int64_t ldx, const int64_t* a, double divisor,
                  double* out, void* stream) {
    int rc = check_common(N, P, ldx, X, a, out);
    if (rc) return rc;
    if (P == 0) { g_err[0] = 0; return FA_OK; }
    StreamDevice on_stream_device(stream);
    hipLaunchKernelGGL((k_fedavg_int<int64_t, uint64_t>), grid_for(P), dim3(kBlock), 0, (hipStream_t)stream,
                       X, N, P, ldx, a, divisor, out);
    return check_launch("k_fedavg_int<int64>");
}

// ---- the same folds with the per-client factors in host memory ---------------
int fa_factors_fill(float* dst, const float* a, const float* s, int64_t N, void* stream) {
    if (N < 0 || (N > 0 && (!dst || !a))) return fail(FA_ERR_ARG, "fa_factors_fill: N %lld, null pointer", (long long)N);
    StreamDevice on_stream_device(stream);
    const int64_t need = N * (s ? 2 : 1);
    for (int64_t off = 0; off < need; off += kFillFloats) {
        FillArgs f;
        const int n = (int)(need - off < kFillFloats ? need - off : kFillFloats);
        for (int i = 0; i < n; ++i) {
            const int64_t j = off + i;
            f.v[i] = j < N ? a[j] : s[j - N];
        }
        hipLaunchKernelGGL(k_fill_factors, dim3(1), dim3(64), 0, (hipStream_t)stream, dst + off, f, n);
        const int rc = check_launch("fa_factors_fill");
        if (rc) return rc;
    }
    return FA_OK;
}

int fa_fedavg_f32_hostf(const float* X, int64_t N, int64_t P, int64_t ldx, const float* a, const float* s,
                        float divisor, float* out, void* stream) {
    return with_host_factors(a, s, N, stream, [&](const float* ad, const float* sd) {
        return fold_f32_auto(X, N, P, ldx, ad, sd, nullptr, divisor, 1, out, stream);
    });
}

int fa_fedavg_f32_ptrs_hostf(const float* const* xi, int64_t N, int64_t P, const float* a, const float* s,
                             float divisor, int rows_aligned, float* out, void* stream) {
    return with_host_factors(a, s, N, stream, [&](const float* ad, const float* sd) {
        return rows_aligned ? fa_fedavg_f32_ptrs_aligned(xi, N, P, ad, sd, divisor, out, stream)
                            : fa_fedavg_f32_ptrs(xi, N, P, ad, sd, divisor, out, stream);
    });
}

int fa_fedavg_bf16_hostf(const uint16_t* X, int64_t N, int64_t P, int64_t ldx, const float* a, const float* s,
                         float divisor, float* out_f32, uint16_t* out_bf16, void* stream) {
    return with_host_factors(a, s, N, stream, [&](const float* ad, const float* sd) {
        return bf16_auto(X, N, P, ldx, ad, sd, divisor, out_f32, out_bf16, stream);
    });
}

int fa_fedavg_f32_rounds_hostf(fa_rounds* r, const float* X, int64_t N, int64_t ldx, const float* a, const float* s,
                               float divisor, float* out, int rounds, const int64_t* offsets,
                               const int64_t* out_offsets, void* stream) {
    if (!r) return fail(FA_ERR_ARG, "null fa_rounds");
    return with_host_factors(a, s, N, stream, [&](const float* ad, const float* sd) {
        return fa_fedavg_f32_rounds(r, X, N, ldx, ad, sd, divisor, out, rounds, offsets, out_offsets, stream);
    });
}

int fa_fedavg_bf16_rounds_hostf(fa_rounds* r, const uint16_t* X, int64_t N, int64_t ldx, const float* a,
                                const float* s, float divisor, float* out_f32, uint16_t* out_bf16, int rounds,
                                const int64_t* offsets, const int64_t* out_offsets, void* stream) {
    if (!r) return fail(FA_ERR_ARG, "null fa_rounds");
    return with_host_factors(a, s, N, stream, [&](const float* ad, const float* sd) {
        return fa_fedavg_bf16_rounds(r, X, N, ldx, ad, sd, divisor, out_f32, out_bf16, rounds, offsets, out_offsets,
                                     stream);
    });
}

// ---- host staging: page-locked documents and direct DMA ---------------------
int fa_host_is_pinned(const void* p, int64_t n) {
    if (!p || n <= 0) return 0;
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();  // unregistered pageable memory: not an error for the caller
        return 0;
    }
    if (at.type != hipMemoryTypeHost) return 0;
    // the whole range must lie inside that one allocation
    hipDeviceptr_t start = nullptr;
    size_t size = 0;
    if (hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, (hipDeviceptr_t)p) != hipSuccess ||
        hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, (hipDeviceptr_t)p) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    const uintptr_t lo = reinterpret_cast<uintptr_t>(start), q = reinterpret_cast<uintptr_t>(p);
    return q >= lo && q + (uint64_t)n <= lo + size ? 1 : 0;
}

int fa_host_alloc(void** p, int64_t n) {
    if (!p || n <= 0) return fail(FA_ERR_ARG, "fa_host_alloc: bad size %lld", (long long)n);
    *p = nullptr;
    hipError_t e = hipHostMalloc(p, (size_t)n, hipHostMallocDefault);
    if (e != hipSuccess) return fail(FA_ERR_HIP, "hipHostMalloc(%lld): %s", (long long)n, hipGetErrorString(e));
    g_err[0] = 0;
    return FA_OK;
}

int fa_host_free(void* p) {
    if (!p) return FA_OK;
    hipError_t e = hipHostFree(p);
    if (e != hipSuccess) return fail(FA_ERR_HIP, "hipHostFree: %s", hipGetErrorString(e));
    return FA_OK;
}

int fa_copy_h2d(void* dst, const void* src, int64_t n, void* stream) {
    if (n < 0 || (n && (!dst || !src))) return fail(FA_ERR_ARG, "fa_copy_h2d: bad arguments");
    if (n == 0) return FA_OK;
    hipError_t e = hipMemcpyAsync(dst, src, (size_t)n, hipMemcpyHostToDevice, (hipStream_t)stream);
    if (e != hipSuccess) return fail(FA_ERR_HIP, "hipMemcpyAsync H2D: %s", hipGetErrorString(e));
    return FA_OK;
}

// ---- single-process multi-GPU: reassembling the model over xGMI -------------
int fa_copy_peer(void* dst, int dst_device, const void* src, int src_device, int64_t n, void* stream) {
    if (n < 0 || (n && (!dst || !src)) || dst_device < 0 || src_device < 0 || dst_device >= 16 ||
        src_device >= 16)
        return fail(FA_ERR_ARG, "fa_copy_peer: bad arguments");
    if (n == 0) { g_err[0] = 0; return FA_OK; }
    StreamDevice on_stream_device(stream);
    if (dst_device != src_device) {
        // peer access both ways, once per pair (without it the runtime stages
        // the copy through host memory)
        static std::mutex mu;
        static bool tried[16][16] = {};
        std::lock_guard<std::mutex> lk(mu);
        if (!tried[src_device][dst_device]) {
            tried[src_device][dst_device] = tried[dst_device][src_device] = true;
            int prev = 0;
            (void)hipGetDevice(&prev);
            const int pair[2][2] = {{src_device, dst_device}, {dst_device, src_device}};
            for (const auto& pr : pair) {
                int can = 0;
                if (hipDeviceCanAccessPeer(&can, pr[0], pr[1]) == hipSuccess && can && hipSetDevice(pr[0]) == hipSuccess) {
                    const hipError_t pe = hipDeviceEnablePeerAccess(pr[1], 0);
                    if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled)
                        (void)hipGetLastError();  // the copy below still works, staged
                }
            }
            (void)hipGetLastError();  // clear any failed enable: the copy reports its own status
            (void)hipSetDevice(prev);
        }
    }
    hipError_t e = hipMemcpyPeerAsync(dst, dst_device, src, src_device, (size_t)n, (hipStream_t)stream);
    if (e != hipSuccess) return fail(FA_ERR_HIP, "hipMemcpyPeerAsync: %s", hipGetErrorString(e));
    g_err[0] = 0;
    return FA_OK;
}

}  // extern "C"
