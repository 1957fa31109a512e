// ingest_pipe.cpp — native streaming ingest for libfedavg_hip.so:
// client rows in host memory -> packed into page-locked slots by a persistent
// worker pool -> one DMA per slot on a copy stream -> the in-order chunked fold
// (fa_fold_f32) on the caller's compute stream.
//
// Reference path replaced: the strategies' aggregate() materialises every
// decoded client (fed_avg_aggregator.py:64-92, stall_aware_aggregation.py:
// 82-117) and then folds on one core.  Here the caller hands over each
// decoded row as soon as it has it (fa_ingest_add returns once the row's copy
// tasks are queued): decoding row i+1 (caller), packing rows i, i-1, ...
// (workers), the DMA of the previous slot (copy engine) and the fold of the
// one before (GPU) all overlap.  Slots are filled and folded strictly in row
// order with the accumulator carried across them, so the result is
// bit-identical to one fa_fedavg_f32 over all rows (the property fa_fold_f32
// documents).
//
// Threads: the caller's thread (add / finish, which block only for
// backpressure: a slot is refilled after its fold has completed), one issuer
// thread per pipe (waits for a full slot's packs, then enqueues its DMA and
// fold: the HIP calls stay in slot order) and a process-wide pool of copy
// workers shared by every pipe (one pipe per GPU for the multi-GPU drop-in).
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "fedavg_hip.h"
#include "host_copy.hpp"

__attribute__((visibility("hidden"))) int fa_internal_fail(int code, const char* msg);

namespace {

// ---- process-wide copy workers ------------------------------------------------
class CopyPool {
  public:
    static CopyPool& get() {
        static CopyPool pool;
        return pool;
    }
    void submit(std::function<void()> f) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (workers_.empty()) start(per_device());
            q_.push_back(std::move(f));
        }
        cv_.notify_one();
    }
    // A pipe on a new device: the pool grows by one device's share of workers
    // (each GPU of a node comes with its own share of host cores, and each
    // GPU's pipe packs its own column bucket: multigpu.py), up to the host's
    // hardware threads.  FEDAVG_COPY_THREADS fixes the size instead.
    void add_device(int device) {
        std::lock_guard<std::mutex> lk(mu_);
        for (int d : devices_)
            if (d == device) return;
        devices_.push_back(device);
        if (!workers_.empty() && !getenv("FEDAVG_COPY_THREADS")) start(per_device());
    }
    int threads() {
        std::lock_guard<std::mutex> lk(mu_);
        return (int)workers_.size();
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }

  private:
    static int per_device() { return 16; }  // the GPU box's CPU share of one GPU
    // Grow the pool by `add` workers (under mu_); the total follows the
    // devices with pipes, FEDAVG_COPY_THREADS overrides it, the host's
    // hardware threads cap it.
    void start(int add) {
        int target = (int)workers_.size() + add;
        if (workers_.empty()) target = per_device() * std::max<int>(1, (int)devices_.size());
        if (const char* e = getenv("FEDAVG_COPY_THREADS")) target = std::max(1, atoi(e));
        target = std::min<int>(target, std::max(1u, std::thread::hardware_concurrency()));
        while ((int)workers_.size() < target) workers_.emplace_back([this] { loop(); });
    }
    void loop() {
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
            if (q_.empty()) return;  // stop_
            std::function<void()> f = std::move(q_.front());
            q_.pop_front();
            lk.unlock();
            f();
            lk.lock();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::function<void()>> q_;
    std::vector<std::thread> workers_;
    std::vector<int> devices_;  // devices that have had a pipe
    bool stop_ = false;
};

constexpr int64_t kTaskBytes = 1 << 20;  // one copy task: >= 1 MiB keeps the pool's overhead small

enum class SlotState { kFree, kFilling, kQueued, kIssued };

struct Slot {
    float* host = nullptr;      // [R][ldx] page-locked
    float* dev = nullptr;       // [R][ldx]
    float* fac_host = nullptr;  // [2][R] page-locked: a, then s (the head of the slot's one allocation)
    float* fac_dev = nullptr;   // [2][R]
    hipEvent_t h2d_done = nullptr, fold_done = nullptr;
    SlotState state = SlotState::kFree;
    int64_t rows = 0;
    int64_t cap = 0;  // rows this use of the slot takes before it is sent (<= R: the ramps)
    bool has_s = false;
    std::atomic<int64_t> outstanding{0};  // copy tasks not yet finished
};

struct QueueItem {
    int slot;  // -1: finalize only (every row already folded)
    bool final_chunk;
};

}  // namespace

struct fa_ingest {
    int64_t P = 0, ldx = 0, R = 0;
    int64_t fac_pad = 0;  // floats of factors (2R) rounded up to 64: the rows stay 256-B aligned
    int K = 0, device = 0;
    std::vector<Slot> slots;
    hipStream_t copy[2] = {nullptr, nullptr};  // chunks alternate between two copy streams
    int64_t issued = 0;                         // chunks issued (issuer thread)
    // per round
    float* acc = nullptr;
    hipStream_t compute = nullptr;
    int cur = 0;
    int64_t rows = 0;
    int64_t expected = 0;  // rows the caller announced for the round (0: unknown)
    int64_t chunks = 0;    // slots started this round
    bool started = false;  // acc holds a partial fold (issuer side)
    int scored = -1;       // -1 unknown, 0 FedAvg, 1 stall-aware
    float divisor = 0.f;
    // issuer
    std::thread issuer;
    std::mutex mu;
    std::condition_variable cv;       // issuer wake-up, slot state changes, pack completion
    std::deque<QueueItem> queue;
    int in_flight = 0;                // queue items not yet issued
    bool stop = false;
    int err = FA_OK;
    std::string errmsg;
};

namespace {

int set_err(fa_ingest* p, int code, const std::string& msg) {
    std::lock_guard<std::mutex> lk(p->mu);
    if (p->err == FA_OK) {
        p->err = code;
        p->errmsg = msg;
    }
    p->cv.notify_all();
    return code;
}

int hip_err(fa_ingest* p, const char* what, hipError_t e) {
    return set_err(p, FA_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

// Issue one full slot (or the finalize-only step) on the streams.  Runs on the
// issuer thread, in queue (= row) order.
int issue(fa_ingest* p, const QueueItem& it) {
    if (it.slot < 0) {  // every row was in earlier slots: divide only
        return fa_fold_f32(nullptr, 0, p->P, p->ldx, nullptr, nullptr, p->acc, p->divisor, 1, p->acc, p->compute);
    }
    Slot& S = p->slots[it.slot];
    {
        std::unique_lock<std::mutex> lk(p->mu);
        p->cv.wait(lk, [&] { return S.outstanding.load() == 0 || p->err != FA_OK; });
        if (p->err != FA_OK) return p->err;
    }
    // one DMA per chunk: the factors sit right before the rows in the slot's
    // allocation (a separate small copy ran as a blit kernel between two SDMA
    // transfers and left ~25 us of idle DMA engine per chunk).  Consecutive
    // chunks alternate between two copy streams: on one stream each transfer
    // started ~17 us after the previous one ended (profiles/r03_e2e_trace/);
    // the fold of each chunk still waits for exactly its own transfer.
    hipStream_t cs = p->copy[p->issued++ & 1];
    hipError_t e = hipMemcpyAsync(S.fac_dev, S.fac_host, (size_t)(p->fac_pad + S.rows * p->ldx) * sizeof(float),
                                  hipMemcpyHostToDevice, cs);
    if (e == hipSuccess) e = hipEventRecord(S.h2d_done, cs);
    if (e == hipSuccess) e = hipStreamWaitEvent(p->compute, S.h2d_done, 0);
    if (e != hipSuccess) return hip_err(p, "ingest H2D", e);
    const int rc = fa_fold_f32(S.dev, S.rows, p->P, p->ldx, S.fac_dev, S.has_s ? S.fac_dev + p->R : nullptr,
                               p->started ? p->acc : nullptr, it.final_chunk ? p->divisor : 0.f,
                               it.final_chunk ? 1 : 0, p->acc, p->compute);
    if (rc != FA_OK) return set_err(p, rc, std::string("ingest fold: ") + fa_last_error());
    p->started = true;
    e = hipEventRecord(S.fold_done, p->compute);
    if (e != hipSuccess) return hip_err(p, "ingest event", e);
    return FA_OK;
}

void issuer_loop(fa_ingest* p) {
    (void)hipSetDevice(p->device);
    std::unique_lock<std::mutex> lk(p->mu);
    for (;;) {
        p->cv.wait(lk, [&] { return p->stop || !p->queue.empty(); });
        if (p->queue.empty()) return;  // stop
        const QueueItem it = p->queue.front();
        p->queue.pop_front();
        const bool ok = p->err == FA_OK;  // after a failure the rest of the round is drained, not issued
        lk.unlock();
        const int rc = ok ? issue(p, it) : FA_OK;
        lk.lock();
        if (it.slot >= 0) p->slots[it.slot].state = SlotState::kIssued;
        if (rc != FA_OK && p->err == FA_OK) {
            p->err = rc;
            p->errmsg = fa_last_error();
        }
        --p->in_flight;
        p->cv.notify_all();
    }
}

void enqueue(fa_ingest* p, int slot, bool final_chunk) {
    std::lock_guard<std::mutex> lk(p->mu);
    if (slot >= 0) p->slots[slot].state = SlotState::kQueued;
    p->queue.push_back({slot, final_chunk});
    ++p->in_flight;
    p->cv.notify_all();
}

// Wait until slot k may be refilled: its previous contents were issued and
// their fold has completed.
int claim(fa_ingest* p, int k) {
    Slot& S = p->slots[k];
    {
        std::unique_lock<std::mutex> lk(p->mu);
        p->cv.wait(lk, [&] { return S.state != SlotState::kQueued || p->err != FA_OK; });
        if (p->err != FA_OK) return p->err;
    }
    if (S.state == SlotState::kIssued) {
        hipError_t e = hipEventSynchronize(S.fold_done);
        if (e != hipSuccess) return hip_err(p, "ingest slot wait", e);
    }
    S.state = SlotState::kFilling;
    S.rows = 0;
    return FA_OK;
}

void free_slots(fa_ingest* p) {
    for (Slot& S : p->slots) {
        if (S.fold_done) (void)hipEventSynchronize(S.fold_done);
        if (S.h2d_done) (void)hipEventDestroy(S.h2d_done);
        if (S.fold_done) (void)hipEventDestroy(S.fold_done);
        if (S.fac_host) (void)hipHostFree(S.fac_host);  // the slot's one allocation (factors, then rows)
        if (S.fac_dev) (void)hipFree(S.fac_dev);
    }
    for (hipStream_t cs : p->copy)
        if (cs) (void)hipStreamDestroy(cs);
}

// Wait until no copy task of any slot is running (they read the caller's rows
// and write the slots).  Under p->mu.
void wait_packs(fa_ingest* p, std::unique_lock<std::mutex>& lk) {
    p->cv.wait(lk, [&] {
        for (const Slot& S : p->slots)
            if (S.outstanding.load() != 0) return false;
        return true;
    });
}

int report(fa_ingest* p) {
    std::lock_guard<std::mutex> lk(p->mu);
    if (p->err == FA_OK) return FA_OK;
    return fa_internal_fail(p->err, p->errmsg.c_str());
}

}  // namespace

extern "C" {

int fa_ingest_create(fa_ingest** out, int64_t P, int64_t chunk_bytes, int slots, int device) {
    if (!out || P <= 0 || chunk_bytes <= 0 || slots < 2 || slots > 64 || device < 0)
        return fa_internal_fail(FA_ERR_ARG, "fa_ingest_create: bad arguments");
    *out = nullptr;
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess) {
        (void)hipGetLastError();
        return fa_internal_fail(FA_ERR_HIP, "fa_ingest_create: cannot select the device");
    }
    fa_ingest* p = new fa_ingest();
    p->P = P;
    p->ldx = (P + 63) / 64 * 64;  // 256-B row pitch: the vector folds
    p->R = std::max<int64_t>(1, chunk_bytes / (p->ldx * (int64_t)sizeof(float)));
    p->K = slots;
    p->fac_pad = (2 * p->R + 63) / 64 * 64;
    p->device = device;
    p->slots = std::vector<Slot>(slots);
    hipError_t e = hipStreamCreateWithFlags(&p->copy[0], hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&p->copy[1], hipStreamNonBlocking);
    for (Slot& S : p->slots) {
        const size_t rowbytes = (size_t)(p->R * p->ldx) * sizeof(float), facbytes = (size_t)p->fac_pad * sizeof(float);
        if (e == hipSuccess) e = hipHostMalloc((void**)&S.fac_host, facbytes + rowbytes, hipHostMallocDefault);
        if (e == hipSuccess) e = hipMalloc((void**)&S.fac_dev, facbytes + rowbytes);
        if (e == hipSuccess) {
            S.host = S.fac_host + p->fac_pad;  // rows start 256-B aligned after the factors
            S.dev = S.fac_dev + p->fac_pad;
        }
        if (e == hipSuccess) e = hipEventCreateWithFlags(&S.h2d_done, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&S.fold_done, hipEventDisableTiming);
        if (e == hipSuccess) memset(S.fac_host, 0, facbytes);
    }
    if (e != hipSuccess) {
        const std::string msg = std::string("fa_ingest_create: ") + hipGetErrorString(e);
        free_slots(p);
        delete p;
        (void)hipSetDevice(prev);
        return fa_internal_fail(FA_ERR_HIP, msg.c_str());
    }
    p->issuer = std::thread(issuer_loop, p);
    (void)hipSetDevice(prev);
    CopyPool::get().add_device(device);
    *out = p;
    return FA_OK;
}

int fa_ingest_rows_per_chunk(const fa_ingest* p) { return p ? (int)p->R : 0; }

int fa_ingest_begin(fa_ingest* p, float* acc, void* stream, int64_t expected_rows) {
    if (!p || !acc || expected_rows < 0) return fa_internal_fail(FA_ERR_ARG, "fa_ingest_begin: bad arguments");
    {  // a round abandoned half-way (an error in add, or no finish) may still
       // have chunks queued and copies running, and a slot half filled: they
       // drain first (the issuer stops issuing once the round has failed), and
       // the half-filled slot's rows do not join this round
        std::unique_lock<std::mutex> lk(p->mu);
        if (p->in_flight && p->err == FA_OK) {
            p->err = FA_ERR_ARG;  // the queued chunks of the abandoned round are drained, not issued
            p->errmsg = "round abandoned";
            p->cv.notify_all();
        }
        p->cv.wait(lk, [&] { return p->in_flight == 0; });
        wait_packs(p, lk);
        for (Slot& S : p->slots)
            if (S.state == SlotState::kFilling) {
                S.state = SlotState::kFree;
                S.rows = 0;
            }
        p->err = FA_OK;
        p->errmsg.clear();
    }
    p->acc = acc;
    p->compute = (hipStream_t)stream;
    p->cur = 0;
    p->rows = 0;
    p->expected = expected_rows;
    p->chunks = 0;
    p->started = false;
    p->scored = -1;
    return FA_OK;
}

int fa_ingest_add(fa_ingest* p, const void* const* srcs, const int64_t* sizes, int64_t n, float a, float s,
                  int has_s) {
    if (!p || n < 0 || (n > 0 && (!srcs || !sizes))) return fa_internal_fail(FA_ERR_ARG, "fa_ingest_add: bad arguments");
    if (p->scored >= 0 && p->scored != (has_s ? 1 : 0))
        return fa_internal_fail(FA_ERR_SHAPE, "either every row has a score or none does");
    int64_t total = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (sizes[i] < 0 || (sizes[i] && !srcs[i])) return fa_internal_fail(FA_ERR_ARG, "fa_ingest_add: bad piece");
        total += sizes[i];
    }
    if (total != p->P * (int64_t)sizeof(float))
        return fa_internal_fail(FA_ERR_SHAPE, "fa_ingest_add: row bytes != P * 4");
    if (int rc = report(p)) return rc;
    p->scored = has_s ? 1 : 0;
    Slot& S = p->slots[p->cur];
    if (S.state != SlotState::kFilling) {
        if (claim(p, p->cur) != FA_OK) return report(p);
        // Ramps: the round's first chunks hold 1, 2, 4, ... rows, so the first
        // DMA starts after one row instead of a full chunk; with the row count
        // announced, the last ones shrink the same way (at most half of what
        // is left), so the tail the round waits for after its last row is
        // about one row's DMA and fold instead of a chunk's.
        int64_t cap = p->chunks < 62 ? std::min<int64_t>(p->R, (int64_t)1 << p->chunks) : p->R;
        if (p->expected > p->rows) cap = std::min(cap, std::max<int64_t>(1, (p->expected - p->rows + 1) / 2));
        S.cap = cap;
        ++p->chunks;
    }
    const int64_t r = S.rows++;
    S.has_s = has_s != 0;
    S.fac_host[r] = a;
    S.fac_host[p->R + r] = has_s ? s : 1.0f;
    // copy tasks of 1 MiB, split across pieces and inside large pieces; 256 KiB
    // while the round's first chunks ramp up (the first DMA waits for them)
    const int64_t task_bytes = p->chunks <= 2 ? kTaskBytes / 4 : kTaskBytes;
    uint8_t* dst = reinterpret_cast<uint8_t*>(S.host + r * p->ldx);
    int64_t off = 0;
    struct Part { const uint8_t* src; uint8_t* dst; int64_t n; };
    std::vector<Part> batch;
    int64_t batch_bytes = 0;
    auto flush = [&] {
        if (batch.empty()) return;
        S.outstanding.fetch_add(1);
        CopyPool::get().submit([p, &S, parts = std::move(batch)] {
            for (const Part& q : parts) fa_host::pack_copy(q.dst, q.src, (size_t)q.n);
            // decrement under the pipe's lock: once a waiter sees 0 this task no longer touches the pipe
            std::lock_guard<std::mutex> lk(p->mu);
            if (S.outstanding.fetch_sub(1) == 1) p->cv.notify_all();
        });
        batch = std::vector<Part>();
        batch_bytes = 0;
    };
    for (int64_t i = 0; i < n; ++i) {
        const uint8_t* src = (const uint8_t*)srcs[i];
        for (int64_t done = 0; done < sizes[i];) {
            const int64_t take = std::min(sizes[i] - done, task_bytes - batch_bytes);
            batch.push_back({src + done, dst + off, take});
            batch_bytes += take;
            done += take;
            off += take;
            if (batch_bytes >= task_bytes) flush();
        }
    }
    flush();
    ++p->rows;
    if (S.rows == S.cap) {
        enqueue(p, p->cur, false);
        p->cur = (p->cur + 1) % p->K;
    }
    return FA_OK;
}

int fa_ingest_finish(fa_ingest* p, float divisor) {
    if (!p) return fa_internal_fail(FA_ERR_ARG, "fa_ingest_finish: bad arguments");
    if (p->rows == 0) return fa_internal_fail(FA_ERR_NO_CLIENTS, "no client results to aggregate (N == 0)");
    p->divisor = divisor;  // read by the issuer for the final item, which is queued below
    Slot& S = p->slots[p->cur];
    if (S.state == SlotState::kFilling && S.rows > 0) {
        enqueue(p, p->cur, true);
        p->cur = (p->cur + 1) % p->K;
    } else {
        enqueue(p, -1, true);
    }
    {
        std::unique_lock<std::mutex> lk(p->mu);
        p->cv.wait(lk, [&] { return p->in_flight == 0; });  // every DMA and fold enqueued
        // every pack done: after an error the drained items were never issued,
        // and their copies may still be reading the caller's rows
        wait_packs(p, lk);
    }
    return report(p);
}

int fa_ingest_destroy(fa_ingest* p) {
    if (!p) return FA_OK;
    {
        std::lock_guard<std::mutex> lk(p->mu);
        p->stop = true;
    }
    p->cv.notify_all();
    if (p->issuer.joinable()) p->issuer.join();
    {  // copy tasks still running read from the caller's rows and write the slots
        std::unique_lock<std::mutex> lk(p->mu);
        wait_packs(p, lk);
    }
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(p->device);
    free_slots(p);
    (void)hipSetDevice(prev);
    delete p;
    return FA_OK;
}

}  // extern "C"
