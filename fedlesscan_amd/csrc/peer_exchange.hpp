// peer_exchange.hpp -- the kernel-free exchange of a multi-GPU step (fa_peers,
// include/fedavg_hip.h), included by fedavg.hip after fold_kernels.hpp.
//
// Reference reassembly point: aggregation.py:125-138 -> ParameterDao.save
// (client_daos.py:351-378) stores ONE global model; at N > 1 every rank folds
// its column slots and the slots of all ranks are gathered into that model.
// The RCCL all-gather (sharding.py) runs copy kernels on a few CUs of every
// GPU while the next round's fold runs; on one GPU the fold lost 16-21 % beside
// a copy kernel on 16-64 blocks, and 1-5 % beside copy-engine (SDMA) copies of
// the same bytes (profiles/r05_exchange/).  Here each rank PULLS
// its peers' finished slots with hipMemcpyAsync on copy streams (the copy
// engines, no CU) from their send buffers, opened once through IPC handles:
//
//   fold stream:  fence (every peer has finished reading this rank's send
//                 buffer from the last step) -> the one-launch fold (the rank's
//                 own fa_rounds state, rounds published at system scope)
//   caller stream, per round k: one wave polls every rank's round-k flag
//                 (peer memory over xGMI, system-scope loads) -> each copy
//                 stream q pulls rank q's round-k slot into the global model
//   then:         the streams join; one wave writes this step's epoch into
//                 every peer's ack word for this rank (system-scope stores)
//
// Every rank runs the same steps, so the epochs of their fold launches agree.
// A wait that gives up (30 s, FEDAVG_ROUND_WAIT_US) records its epoch in the
// state's mapped status words like fa_rounds_wait's, and fa_rounds_check
// reports it: the caller raises instead of using the model.
#pragma once

namespace {
constexpr int kMaxPeers = 16;
struct PeerPtrs {
    unsigned int* p[kMaxPeers];
};
}  // namespace

// the C-ABI's opaque handles (include/fedavg_hip.h)
struct fa_rounds : RoundsState {};

struct fa_peers {
    int device = 0, world = 0, rank = 0;
    fa_rounds R;                               // the rank's fold launches (rounds published at system scope)
    void* send = nullptr;                      // the rank's own slots, side by side (the fold's output)
    int64_t send_bytes = 0;
    unsigned int* ack = nullptr;               // [world]: ack[q] = the last epoch rank q finished pulling
    void* peer_send[kMaxPeers] = {};           // opened IPC pointers (own rank: send)
    unsigned int* peer_sig[kMaxPeers] = {};    // peers' signal words (own: R.sig)
    unsigned int* peer_ack[kMaxPeers] = {};    // peers' ack words (own: ack)
    bool opened = false;
    hipStream_t copy[kMaxPeers] = {};          // one copy stream per source rank
    hipEvent_t round_ready[kMaxRounds] = {};   // every rank's round k is complete (caller stream)
    hipEvent_t copied[kMaxPeers] = {};         // a copy stream's last copy of the step
};

namespace {

// Lane i polls word p[i] (i < n) until it reaches epoch (wrapping compare), or
// gives up after max_ticks and stores `record` (the epoch of the launch the
// wait guards) into `status` (mapped host memory).  System-scope loads: the words live in other GPUs' memory (or are
// written by them) and must be read from memory, not a stale cache line.
__global__ __launch_bounds__(64) void k_wait_words(PeerPtrs w, int n, unsigned int epoch, unsigned int record,
                                                   unsigned int* status, long long max_ticks) {
    const int i = threadIdx.x;
    if (i >= n) return;
    const long long t0 = wall_clock64();
    while ((int)(__hip_atomic_load(w.p[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
        if (wall_clock64() - t0 > max_ticks) {
            if (status) __hip_atomic_store(status, record, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        __builtin_amdgcn_s_sleep(4);
    }
}

// Lane i stores v into word p[i] (i < n): system-scope vector stores.
__global__ __launch_bounds__(64) void k_store_words(PeerPtrs w, int n, unsigned int v) {
    const int i = threadIdx.x;
    if (i < n) __hip_atomic_store(w.p[i], v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// IPC handles of one rank: its send buffer, signal words, ack words
constexpr int kPeerHandleBytes = 3 * (int)sizeof(hipIpcMemHandle_t);

inline void peers_free(fa_peers& x) {
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(x.device);
    (void)hipDeviceSynchronize();
    for (int q = 0; q < x.world && q < kMaxPeers; ++q) {
        if (q == x.rank || !x.opened) continue;
        if (x.peer_send[q]) (void)hipIpcCloseMemHandle(x.peer_send[q]);
        if (x.peer_sig[q]) (void)hipIpcCloseMemHandle(x.peer_sig[q]);
        if (x.peer_ack[q]) (void)hipIpcCloseMemHandle(x.peer_ack[q]);
    }
    for (int q = 0; q < kMaxPeers; ++q) {
        if (x.copy[q]) (void)hipStreamDestroy(x.copy[q]);
        if (x.copied[q]) (void)hipEventDestroy(x.copied[q]);
    }
    for (int k = 0; k < kMaxRounds; ++k)
        if (x.round_ready[k]) (void)hipEventDestroy(x.round_ready[k]);
    if (x.send) (void)hipFree(x.send);
    if (x.ack) (void)hipFree(x.ack);
    (void)hipGetLastError();
    (void)hipSetDevice(prev);
    rounds_state_free(x.R);
}

inline int peers_init(fa_peers& x, int device, int world, int rank, int64_t send_bytes) {
    if (world < 1 || world > kMaxPeers || rank < 0 || rank >= world || send_bytes < 16 || send_bytes % 16)
        return fail(FA_ERR_ARG, "fa_peers_create: world %d (1..%d), rank %d, send_bytes %lld (16-B multiple)", world,
                    kMaxPeers, rank, (long long)send_bytes);
    int rc = rounds_state_init(x.R, device);
    if (rc) return rc;
    x.R.sys = true;
    x.device = device;
    x.world = world;
    x.rank = rank;
    x.send_bytes = send_bytes;
    int prev = 0;
    (void)hipGetDevice(&prev);
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipMalloc(&x.send, (size_t)send_bytes);
    if (e == hipSuccess) e = hipMalloc((void**)&x.ack, kMaxPeers * sizeof(unsigned int));
    if (e == hipSuccess) e = hipMemset(x.ack, 0, kMaxPeers * sizeof(unsigned int));
    for (int q = 0; q < world && e == hipSuccess; ++q) {
        e = hipStreamCreateWithFlags(&x.copy[q], hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&x.copied[q], hipEventDisableTiming);
    }
    for (int k = 0; k < kMaxRounds && e == hipSuccess; ++k)
        e = hipEventCreateWithFlags(&x.round_ready[k], hipEventDisableTiming);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    (void)hipSetDevice(prev);
    if (e != hipSuccess) return fail(FA_ERR_HIP, "fa_peers_create: %s", hipGetErrorString(e));
    x.peer_send[rank] = x.send;
    x.peer_sig[rank] = x.R.sig;
    x.peer_ack[rank] = x.ack;
    return FA_OK;
}

inline int peers_handle(fa_peers& x, void* out) {
    hipIpcMemHandle_t h[3];
    hipError_t e = hipIpcGetMemHandle(&h[0], x.send);
    if (e == hipSuccess) e = hipIpcGetMemHandle(&h[1], x.R.sig);
    if (e == hipSuccess) e = hipIpcGetMemHandle(&h[2], x.ack);
    if (e != hipSuccess) return fail(FA_ERR_HIP, "fa_peers_handle: hipIpcGetMemHandle: %s", hipGetErrorString(e));
    memcpy(out, h, sizeof(h));
    return FA_OK;
}

inline int peers_open(fa_peers& x, const uint8_t* all) {
    if (x.opened) return fail(FA_ERR_ARG, "fa_peers_open: already open");
    int prev = 0;
    (void)hipGetDevice(&prev);
    hipError_t e = hipSetDevice(x.device);
    for (int q = 0; q < x.world && e == hipSuccess; ++q) {
        if (q == x.rank) continue;
        hipIpcMemHandle_t h[3];
        memcpy(h, all + (size_t)q * kPeerHandleBytes, sizeof(h));
        e = hipIpcOpenMemHandle(&x.peer_send[q], h[0], hipIpcMemLazyEnablePeerAccess);
        if (e == hipSuccess) e = hipIpcOpenMemHandle((void**)&x.peer_sig[q], h[1], hipIpcMemLazyEnablePeerAccess);
        if (e == hipSuccess) e = hipIpcOpenMemHandle((void**)&x.peer_ack[q], h[2], hipIpcMemLazyEnablePeerAccess);
    }
    (void)hipSetDevice(prev);
    x.opened = true;  // what was opened is closed by peers_free, also after a failure
    if (e != hipSuccess) return fail(FA_ERR_HIP, "fa_peers_open: hipIpcOpenMemHandle: %s", hipGetErrorString(e));
    return FA_OK;
}

// Before this rank's next fold launch overwrites its send buffer: every peer
// has finished pulling the last step from it (their acks reached its epoch).
inline int peers_fence(fa_peers& x, hipStream_t st) {
    if (!x.opened) return fail(FA_ERR_ARG, "fa_peers_fence: handles not opened (fa_peers_open)");
    if (x.R.epoch == 0) return FA_OK;  // no step yet
    PeerPtrs w{};
    for (int q = 0; q < x.world; ++q) w.p[q] = x.ack + q;
    // a fence that gives up records the epoch of the launch it guards
    const unsigned int guarded = x.R.epoch + 1 == 0 ? 1 : x.R.epoch + 1;
    hipLaunchKernelGGL(k_wait_words, dim3(1), dim3(64), 0, st, w, x.world, x.R.epoch, guarded,
                       x.R.status_dev ? x.R.status_dev + kMaxRounds : nullptr, x.R.max_ticks);
    return check_launch("fa_peers_fence");
}

// Pull every rank's round-k slot into dst as soon as that rank has completed
// round k: src_off [rounds + 1] byte offsets into every rank's send buffer,
// dst_off [rounds][world] byte offsets into dst.
inline int peers_exchange(fa_peers& x, int rounds, const int64_t* src_off, void* dst, const int64_t* dst_off,
                          hipStream_t st) {
    if (!x.opened) return fail(FA_ERR_ARG, "fa_peers_exchange: handles not opened (fa_peers_open)");
    if (!x.R.launched) return fail(FA_ERR_ARG, "fa_peers_exchange: no fold launched on the exchange's rounds state");
    if (rounds != x.R.rounds || !src_off || !dst_off || !dst)
        return fail(FA_ERR_ARG, "fa_peers_exchange: %d rounds (the launch had %d) or null offsets", rounds,
                    x.R.rounds);
    for (int k = 0; k < rounds; ++k)
        if (src_off[k] < 0 || src_off[k + 1] < src_off[k] || src_off[k + 1] > x.send_bytes)
            return fail(FA_ERR_ARG, "fa_peers_exchange: round %d source bytes [%lld, %lld) outside the send buffer", k,
                        (long long)src_off[k], (long long)src_off[k + 1]);
    const unsigned int epoch = x.R.epoch;
    // the polls start with this rank's own fold (their give-up clock with it)
    if (x.R.start && hipStreamWaitEvent(st, x.R.start, 0) != hipSuccess) return check_launch("fa_peers_exchange");
    for (int k = 0; k < rounds; ++k) {
        PeerPtrs w{};
        for (int q = 0; q < x.world; ++q) w.p[q] = x.peer_sig[q] + kSigFlag + k;
        hipLaunchKernelGGL(k_wait_words, dim3(1), dim3(64), 0, st, w, x.world, epoch, epoch,
                           x.R.status_dev ? x.R.status_dev + k : nullptr, x.R.max_ticks);
        int rc = check_launch("fa_peers_exchange: wait");
        if (rc) return rc;
        if (hipEventRecord(x.round_ready[k], st) != hipSuccess) return check_launch("fa_peers_exchange: event");
        const int64_t n = src_off[k + 1] - src_off[k];
        for (int q = 0; q < x.world && n > 0; ++q) {
            hipError_t e = hipStreamWaitEvent(x.copy[q], x.round_ready[k], 0);
            if (e == hipSuccess)
                e = hipMemcpyAsync(static_cast<uint8_t*>(dst) + dst_off[(size_t)k * x.world + q],
                                   static_cast<const uint8_t*>(x.peer_send[q]) + src_off[k], (size_t)n,
                                   hipMemcpyDeviceToDevice, x.copy[q]);
            if (e != hipSuccess) return fail(FA_ERR_HIP, "fa_peers_exchange: copy: %s", hipGetErrorString(e));
        }
    }
    for (int q = 0; q < x.world; ++q) {
        hipError_t e = hipEventRecord(x.copied[q], x.copy[q]);
        if (e == hipSuccess) e = hipStreamWaitEvent(st, x.copied[q], 0);
        if (e != hipSuccess) return fail(FA_ERR_HIP, "fa_peers_exchange: join: %s", hipGetErrorString(e));
    }
    // done reading every peer's send buffer for this step: tell them
    PeerPtrs w{};
    for (int q = 0; q < x.world; ++q) w.p[q] = x.peer_ack[q] + x.rank;
    hipLaunchKernelGGL(k_store_words, dim3(1), dim3(64), 0, st, w, x.world, epoch);
    return check_launch("fa_peers_exchange: ack");
}

}  // namespace
