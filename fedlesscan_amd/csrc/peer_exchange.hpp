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
// its peers' finished slots with hipMemcpyAsync on copy streams from their
// send buffers, opened once through IPC handles:
//
//   fold stream:  the one-launch fold into this step's send buffer (two, used
//                 alternately), its rounds published at system scope (the
//                 rank's own fa_rounds state: sc0 sc1 tile stores, a
//                 system-scope flag store per round)
//   exchange stream, per round k: one wave polls every rank's round-k flag
//                 (peer memory over xGMI, system-scope loads) -> the peers'
//                 round-k slots are pulled into the global model, alternately
//                 on this stream and on one side stream, then this rank's own
//                 slot (a local copy; the last round's on the fold stream, in
//                 order behind the launch); then the side stream joins
//
// No fence and no acknowledgement (round 5 had both: a wave on the fold
// stream before every fold, one writing every peer's ack word after every
// exchange): the next fold with this state waits for this exchange (the
// state's gate event, launch_step), so a rank folds step e+1 only after it
// has pulled step e; a peer that folds step e+2 -- overwriting the buffer of
// step e -- has waited in its step-e+1 exchange for this rank's step-e+1
// flags, which this rank raised after its step-e pulls.  Step e's buffer is
// therefore free before anyone writes it again.
//
// Every rank runs the same steps, so the epochs of their fold launches agree.
// A wait that gives up (30 s, FEDAVG_ROUND_WAIT_US) counts the timeout and
// records its epoch in the state's mapped status words like fa_rounds_wait's,
// and fa_rounds_check reports it: the caller raises instead of using the model.
#pragma once

namespace {
constexpr int kMaxPeers = 16;
// Copy streams per rank, whatever the world size: HIP maps a process's
// streams onto GPU_MAX_HW_QUEUES (4) hardware queues, which the fold, gather,
// default and RCCL streams already share; one stream per peer (8 at world 8)
// would put copies on the fold's queue.  The exchange stream itself and ONE
// side stream keep two copies in flight; the peers' copies of a round
// alternate between them.
constexpr int kCopyStreams = 1;  // side streams besides the exchange stream
struct PeerPtrs {
    unsigned int* p[kMaxPeers];
};
}  // namespace

// the C-ABI's opaque handles (include/fedavg_hip.h)
struct fa_rounds : RoundsState {};

struct fa_peers {
    int device = 0, world = 0, rank = 0;
    fa_rounds R;                               // the rank's fold launches (rounds published at system scope)
    void* send = nullptr;                      // two send buffers of send_bytes, side by side: step e's fold
    int64_t send_bytes = 0;                    // writes buffer e % 2 (the rank's slots, side by side)
    void* peer_send[kMaxPeers] = {};           // opened IPC pointers to every rank's pair (own rank: send)
    unsigned int* peer_sig[kMaxPeers] = {};    // peers' signal words (own: R.sig)
    bool opened = false;
    hipStream_t copy[kCopyStreams] = {};       // the side copy stream: every other peer's slot goes there
    hipEvent_t round_ready[kMaxRounds] = {};   // every rank's round k is complete (exchange stream)
    hipEvent_t copied[kCopyStreams] = {};      // the side stream's last copy of the step
};

namespace {

// Lane i polls word p[i] (i < n) until it reaches epoch (wrapping compare), or
// gives up after max_ticks, counts the timeout in `timeouts` (device memory)
// and stores `record` (the epoch of the launch the wait guards) into `status`
// (mapped host memory).  System-scope loads: the words live in other GPUs' memory (or are
// written by them) and must be read from memory, not a stale cache line.
__global__ __launch_bounds__(64) void k_wait_words(PeerPtrs w, int n, unsigned int epoch, unsigned int record,
                                                   unsigned int* timeouts, unsigned int* status, long long max_ticks) {
    const int i = threadIdx.x;
    if (i >= n) return;
    const long long t0 = wall_clock64();
    while ((int)(__hip_atomic_load(w.p[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
        if (wall_clock64() - t0 > max_ticks) {
            // counted like k_wait_round's (fa_rounds_timeouts), recorded for fa_rounds_check
            atomicAdd(timeouts, 1u);
            if (status) __hip_atomic_store(status, record, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        __builtin_amdgcn_s_sleep(4);
    }
}

// IPC handles of one rank: its send buffers, its signal words
constexpr int kPeerHandleBytes = 2 * (int)sizeof(hipIpcMemHandle_t);

inline void peers_free(fa_peers& x) {
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(x.device);
    (void)hipDeviceSynchronize();
    for (int q = 0; q < x.world && q < kMaxPeers; ++q) {
        if (q == x.rank || !x.opened) continue;
        if (x.peer_send[q]) (void)hipIpcCloseMemHandle(x.peer_send[q]);
        if (x.peer_sig[q]) (void)hipIpcCloseMemHandle(x.peer_sig[q]);
    }
    for (int c = 0; c < kCopyStreams; ++c) {
        if (x.copy[c]) (void)hipStreamDestroy(x.copy[c]);
        if (x.copied[c]) (void)hipEventDestroy(x.copied[c]);
    }
    for (int k = 0; k < kMaxRounds; ++k)
        if (x.round_ready[k]) (void)hipEventDestroy(x.round_ready[k]);
    if (x.send) (void)hipFree(x.send);
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
    x.R.sys = 1;  // system-coherent tile stores, rounds published at system scope
    x.device = device;
    x.world = world;
    x.rank = rank;
    x.send_bytes = send_bytes;
    int prev = 0;
    (void)hipGetDevice(&prev);
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipMalloc(&x.send, 2 * (size_t)send_bytes);
    // the exchange's end, which the state's next fold launch waits for (launch_step)
    if (e == hipSuccess) e = hipEventCreateWithFlags(&x.R.gate, hipEventDisableTiming);
    for (int c = 0; c < kCopyStreams && e == hipSuccess; ++c) {
        e = hipStreamCreateWithFlags(&x.copy[c], hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&x.copied[c], hipEventDisableTiming);
    }
    for (int k = 0; k < kMaxRounds && e == hipSuccess; ++k)
        e = hipEventCreateWithFlags(&x.round_ready[k], hipEventDisableTiming);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    (void)hipSetDevice(prev);
    if (e != hipSuccess) return fail(FA_ERR_HIP, "fa_peers_create: %s", hipGetErrorString(e));
    x.peer_send[rank] = x.send;
    x.peer_sig[rank] = x.R.sig;
    return FA_OK;
}

inline int peers_handle(fa_peers& x, void* out) {
    hipIpcMemHandle_t h[2];
    hipError_t e = hipIpcGetMemHandle(&h[0], x.send);
    if (e == hipSuccess) e = hipIpcGetMemHandle(&h[1], x.R.sig);
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
        hipIpcMemHandle_t h[2];
        memcpy(h, all + (size_t)q * kPeerHandleBytes, sizeof(h));
        e = hipIpcOpenMemHandle(&x.peer_send[q], h[0], hipIpcMemLazyEnablePeerAccess);
        if (e == hipSuccess) e = hipIpcOpenMemHandle((void**)&x.peer_sig[q], h[1], hipIpcMemLazyEnablePeerAccess);
    }
    (void)hipSetDevice(prev);
    x.opened = true;  // what was opened is closed by peers_free, also after a failure
    if (e != hipSuccess) return fail(FA_ERR_HIP, "fa_peers_open: hipIpcOpenMemHandle: %s", hipGetErrorString(e));
    return FA_OK;
}

// The send buffer of the state's NEXT fold launch (epoch parity).
inline void* peers_next_send(const fa_peers& x) {
    const unsigned int e = x.R.epoch + 1 == 0 ? 1 : x.R.epoch + 1;
    return static_cast<uint8_t*>(x.send) + (size_t)(e & 1u) * (size_t)x.send_bytes;
}

// Pull every rank's round-k slot into dst as soon as that rank has completed
// round k: src_off [rounds + 1] byte offsets into every rank's send buffer of
// this step, dst_off [rounds][world] byte offsets into dst.
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
    const size_t half = (size_t)(epoch & 1u) * (size_t)x.send_bytes;  // the buffer this step's folds wrote
    // the polls start with this rank's own fold (their give-up clock with it)
    if (x.R.start && hipStreamWaitEvent(st, x.R.start, 0) != hipSuccess) return check_launch("fa_peers_exchange");
    auto copy_slot = [&](int k, int q, hipStream_t cs) {
        const int64_t n = src_off[k + 1] - src_off[k];
        if (n <= 0) return hipSuccess;
        return hipMemcpyAsync(static_cast<uint8_t*>(dst) + dst_off[(size_t)k * x.world + q],
                              static_cast<const uint8_t*>(x.peer_send[q]) + half + src_off[k], (size_t)n,
                              hipMemcpyDeviceToDevice, cs);
    };
    bool side_used = false;
    for (int k = 0; k < rounds; ++k) {
        const bool last = k == rounds - 1;
        if (!(last && x.world == 1)) {  // the last round of a lone rank needs no wait: see below
            PeerPtrs w{};
            for (int q = 0; q < x.world; ++q) w.p[q] = x.peer_sig[q] + kSigFlag + k;
            hipLaunchKernelGGL(k_wait_words, dim3(1), dim3(64), 0, st, w, x.world, epoch, epoch,
                               x.R.sig + kSigTimeout, x.R.status_dev ? x.R.status_dev + k : nullptr, x.R.max_ticks);
            const int rc = check_launch("fa_peers_exchange: wait");
            if (rc) return rc;
        }
        // the peers' slots, starting after this rank (each rank pulls in a
        // different order, so the ranks' first pulls land on different peers),
        // alternating between the exchange stream itself (in order behind the
        // wait) and the side copy stream (behind an event)
        if (x.world > 2) {
            if (hipEventRecord(x.round_ready[k], st) != hipSuccess || hipStreamWaitEvent(x.copy[0], x.round_ready[k], 0))
                return fail(FA_ERR_HIP, "fa_peers_exchange: round %d event", k);
            side_used = true;
        }
        for (int j = 1; j < x.world; ++j) {
            const hipError_t e = copy_slot(k, (x.rank + j) % x.world, (j % 2 == 1 || x.world == 2) ? st : x.copy[0]);
            if (e != hipSuccess) return fail(FA_ERR_HIP, "fa_peers_exchange: copy: %s", hipGetErrorString(e));
        }
        // this rank's own slot: a local copy, behind the round's wait -- the last
        // round's on the fold's own stream, in order behind the launch (no wait,
        // no hop: the tail of the step)
        const hipError_t e = copy_slot(k, x.rank, last && x.R.last_stream ? x.R.last_stream : st);
        if (e != hipSuccess) return fail(FA_ERR_HIP, "fa_peers_exchange: own copy: %s", hipGetErrorString(e));
    }
    if (side_used) {
        hipError_t e = hipEventRecord(x.copied[0], x.copy[0]);
        if (e == hipSuccess) e = hipStreamWaitEvent(st, x.copied[0], 0);
        if (e != hipSuccess) return fail(FA_ERR_HIP, "fa_peers_exchange: join: %s", hipGetErrorString(e));
    }
    // the state's next fold waits for this exchange (launch_step): the buffer
    // of step e is rewritten at step e + 2 only after every rank pulled it
    if (hipEventRecord(x.R.gate, st) != hipSuccess) return check_launch("fa_peers_exchange: gate");
    x.R.gated = true;
    return FA_OK;
}

}  // namespace
