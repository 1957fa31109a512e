// tuner.hpp -- measured kernel-form choice for the fold entries of
// libfedavg_hip.so (host code only: the HIP runtime API, no kernels, so the
// state machine also builds against tools/tunersim for a host stress test,
// tools/tuner_stress.cpp).  Used by fold_kernels.hpp.
#pragma once

#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

// internal linkage (the libraries export exactly their headers' symbols)
namespace {
namespace fa_tune {

constexpr int kTuneOk = 0;  // FA_OK: launch() returns an FA status

// ---------------------------------------------------------------------------
// Measured form choice (the tuner).  The shape policy's picks
// (fold_kernels.hpp pick_f32 / pick_bf16) are fitted to sweeps over measured
// shapes; between those shapes every form swings with how the tiles fall on
// the CUs (1024 x 909K params: the policy's form 0.70 ms, the even split
// 0.53 ms; 256 x 3.57M bf16: 0.337 against 0.295 ms; profiles/r03_slot_sweep/).
// Every form computes the same bits, and a plain one-shot fold overwrites its
// whole output, so the FIRST call of a new (device, dtype, N, P, pitch,
// scored) shape runs every candidate form on the caller's own data, on the
// caller's stream: one untimed launch of each (code-object load, cold TLBs,
// clocks up from idle), then two timed passes in opposite orders, `batch`
// back-to-back launches of a form between two events (batch sized to ~0.3 ms,
// so launch gaps do not decide between forms of a 20 us kernel: timing single
// launches between events misranked them,
// profiles/r03_tuner/probe_single_launch.log); a form's time is its faster
// pass.  Whichever form ran last, the output is the fold.  Nothing
// synchronises: later calls read the events with hipEventQuery and run the
// policy's pick until they are complete; from then on the shape runs the
// fastest form -- the policy's own pick unless another beats it by more than
// 3 % (box-to-box spread is ~2-5 %).
// FEDAVG_AUTOTUNE=0 (or fa_set_autotune(0)) keeps the policy pick;
// FEDAVG_AUTOTUNE_LOG=1 prints every decision with each candidate's time.
// ---------------------------------------------------------------------------
constexpr float kTuneMargin = 0.97f;
constexpr double kTuneBatchMs = 0.3;  // timed span per candidate
constexpr int kTuneMaxBatch = 32;

class Tuner {
  public:
    // names a (kind, form) pair for the decision log
    typedef const char* (*FormName)(int kind, int form);
    explicit Tuner(FormName name = nullptr) : name_(name) {}
    static int env_mode() {
        const char* e = getenv("FEDAVG_AUTOTUNE");
        return (e && e[0] == '0') ? 0 : 1;
    }
    int set_mode(int m) {
        const int prev = mode_.load();
        if (m >= 0) mode_.store(m ? 1 : 0);
        return prev;
    }
    // Run this call's fold: launch(form) enqueues one fold of that form and
    // returns an FA status.  `cands(v)` fills the candidate forms (v[0] = the
    // policy pick) the first time the shape is seen; `bytes` sizes the batch.
    // Runs on the stream's device (the callers hold a StreamDevice).
    template <class Cands, class Launch>
    int run(int kind, int64_t N, int64_t P, int64_t ldx, bool scored, int policy, double bytes, hipStream_t st,
            Cands cands, Launch launch) {
        if (!mode_.load()) return launch(policy);
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) {
            (void)hipGetLastError();
            return launch(policy);
        }
        const Key key{dev, kind, N, P, ldx, scored ? 1 : 0};
        // no event calls inside a graph capture: neither the measurement nor
        // the queries of an earlier one (hipEventQuery is not capture-safe)
        auto capturing = [&] {
            hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
            if (hipStreamIsCapturing(st, &cs) != hipSuccess) {
                (void)hipGetLastError();
                return true;  // unknown: treat as capturing
            }
            return cs != hipStreamCaptureStatusNone;
        };
        Entry* e = nullptr;
        bool explore = false;
        {
            std::lock_guard<std::mutex> lk(mu_);
            auto it = map_.find(key);
            if (it == map_.end()) {
                if (capturing()) return launch(policy);
                Entry fresh;
                cands(fresh.cand);
                fresh.kind = kind;
                fresh.N = N;
                fresh.P = P;
                fresh.ldx = ldx;
                fresh.scored = scored;
                if (fresh.cand.size() <= 1) fresh.chosen = policy;
                it = map_.emplace(key, std::move(fresh)).first;
                explore = it->second.chosen < 0;
            }
            e = &it->second;  // std::map nodes are stable
            if (!explore) {
                if (e->chosen < 0) {
                    if (capturing()) return launch(e->cand[0]);
                    harvest(*e);
                    if (e->chosen < 0) return launch(e->cand[0]);  // measurement still in flight
                }
                return launch(e->chosen);
            }
        }
        // First call of the shape: time every candidate (this thread owns the
        // entry's events until `armed` is set; other threads run the policy).
        const double est_ms = bytes / 5.0e9;  // ~5 TB/s
        int batch = (int)(kTuneBatchMs / (est_ms > 1e-6 ? est_ms : 1e-6)) + 1;
        if (batch > kTuneMaxBatch) batch = kTuneMaxBatch;
        const int n = (int)e->cand.size();
        std::vector<hipEvent_t> ev(4 * (size_t)n, nullptr);  // [pass][candidate][start, end]
        bool timed = true;
        for (auto& x : ev)
            if (hipEventCreate(&x) != hipSuccess) {
                (void)hipGetLastError();
                x = nullptr;
                timed = false;
            }
        int rc = kTuneOk;
        // untimed: one launch of every form (code-object loads, cold TLBs; the
        // clocks come up from idle), then two timed passes in opposite orders,
        // so a drift over the measurement favours no candidate
        for (int c = 0; c < n && rc == kTuneOk; ++c) rc = launch(e->cand[c]);
        for (int pass = 0; pass < 2; ++pass)
            for (int j = 0; j < n && rc == kTuneOk; ++j) {
                const int c = pass == 0 ? j : n - 1 - j;
                hipEvent_t* pe = &ev[2 * ((size_t)pass * n + c)];
                if (timed && hipEventRecord(pe[0], st) != hipSuccess) timed = false;
                for (int b = 0; b < batch && rc == kTuneOk; ++b) rc = launch(e->cand[c]);
                if (timed && hipEventRecord(pe[1], st) != hipSuccess) timed = false;
            }
        if (!timed) (void)hipGetLastError();
        std::lock_guard<std::mutex> lk(mu_);
        e->batch = batch;
        e->events = ev;
        if (rc != kTuneOk || !timed) e->chosen = e->cand[0];  // a failed or untimed measurement keeps the policy
        e->armed = true;
        if (e->chosen >= 0) release(*e);
        return rc;
    }
    int pending() {
        std::lock_guard<std::mutex> lk(mu_);
        int n = 0;
        for (auto& kv : map_) {
            if (kv.second.chosen >= 0) continue;
            harvest(kv.second);  // the shape may have all it needs without a further call
            if (kv.second.chosen < 0) ++n;
        }
        return n;
    }
    // chosen form (>= 0), -1 while the shape is being measured, -2 unknown shape
    int chosen(int dev, int kind, int64_t N, int64_t P, int64_t ldx, bool scored) {
        std::lock_guard<std::mutex> lk(mu_);
        auto it = map_.find(Key{dev, kind, N, P, ldx, scored ? 1 : 0});
        if (it == map_.end()) return -2;
        if (it->second.chosen < 0) harvest(it->second);
        return it->second.chosen;
    }

  private:
    typedef std::tuple<int, int, int64_t, int64_t, int64_t, int> Key;
    struct Entry {
        std::vector<int> cand;
        std::vector<hipEvent_t> events;  // [2(pass*n + c)] start, [... + 1] end of candidate c's batch
        int batch = 1, chosen = -1;
        bool armed = false;  // the exploring call has recorded every event
        int kind = 0;
        int64_t N = 0, P = 0, ldx = 0;
        bool scored = false;
    };
    void release(Entry& e) {
        for (hipEvent_t x : e.events)
            if (x) (void)hipEventDestroy(x);
        e.events.clear();
    }
    // Decide once the last candidate's end event has completed (the events
    // complete in stream order).  Under mu_.
    void harvest(Entry& e) {
        if (e.chosen >= 0 || !e.armed) return;
        const int n = (int)e.cand.size();
        // the second pass runs backwards: candidate 0's end event is the last one recorded
        const hipError_t q = hipEventQuery(e.events[2 * (size_t)n + 1]);
        if (q == hipErrorNotReady) return;
        std::vector<float> ms(n, 3.4e38f);  // per launch, the faster of the two passes
        bool ok = q == hipSuccess;
        for (int pass = 0; ok && pass < 2; ++pass)
            for (int c = 0; ok && c < n; ++c) {
                const size_t i = 2 * ((size_t)pass * n + c);
                float t = 0.f;
                if (hipEventElapsedTime(&t, e.events[i], e.events[i + 1]) != hipSuccess || !(t > 0.f)) ok = false;
                else if (t / (float)e.batch < ms[c]) ms[c] = t / (float)e.batch;
            }
        if (!ok) {
            (void)hipGetLastError();
            e.chosen = e.cand[0];
            release(e);
            return;
        }
        int b = 0;
        for (int c = 1; c < n; ++c)
            if (ms[c] < ms[b]) b = c;
        e.chosen = (ms[b] < kTuneMargin * ms[0]) ? e.cand[b] : e.cand[0];
        if (log_) {
            char line[1024];
            int k = snprintf(line, sizeof(line), "fedavg tuner: %s N=%lld P=%lld ldx=%lld%s batch=%d -> %s |",
                             e.kind == 1 ? "f32" : e.kind == 2 ? "bf16" : "f32 rows", (long long)e.N, (long long)e.P, (long long)e.ldx,
                             e.scored ? " scored" : "", e.batch, form_name(e.kind, e.chosen));
            for (int c = 0; c < n && k > 0 && k < (int)sizeof(line); ++c)
                k += snprintf(line + k, sizeof(line) - k, " %s %.4f", form_name(e.kind, e.cand[c]), ms[c]);
            fprintf(stderr, "%s ms\n", line);
        }
        release(e);
    }
    const char* form_name(int kind, int form) const { return name_ ? name_(kind, form) : "?"; }
    FormName name_;
    std::mutex mu_;
    std::map<Key, Entry> map_;
    std::atomic<int> mode_{env_mode()};
    const bool log_ = getenv("FEDAVG_AUTOTUNE_LOG") && getenv("FEDAVG_AUTOTUNE_LOG")[0] == '1';
};

}  // namespace fa_tune
}  // namespace
