// Host stress test of the tuner's state machine (fedlesscan_amd/csrc/tuner.hpp)
// against a simulated HIP runtime (tools/tunersim): streams with virtual
// clocks, events that stay "not ready" for a few queries.  Checks: the fastest
// candidate is chosen, the 3 % margin keeps the policy on near-ties, the
// first call runs every form (one untimed launch, then two timed batches),
// decisions wait for the events (no synchronisation), a failing launch keeps
// the policy and returns its status, graph capture and the off switch skip
// measuring, and many threads tuning many shapes at once agree (run under
// TSan and ASan + UBSan by tools/tuner_stress.sh; no events leak).
#include <cassert>
#include <cmath>
#include <cstdio>
#include <random>
#include <thread>
#include <vector>

#include "tuner.hpp"

using fa_tune::Tuner;

static int g_fail = 0;
#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) {                                                     \
            fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++g_fail;                                                   \
        }                                                               \
    } while (0)

static const char* name(int kind, int form) {
    static const char* n[] = {"f0", "f1", "f2", "f3", "f4", "f5", "f6", "f7"};
    (void)kind;
    return form >= 0 && form < 8 ? n[form] : "?";
}

// One call of shape (N, P) whose forms cost cost[form] ms per launch on stream s.
static int call(Tuner& t, SimStream* s, int64_t N, int64_t P, const std::vector<double>& cost, int* launches,
                int fail_form = -1) {
    return t.run(
        1, N, P, P, false, 0, 1.0e12, s,
        [&](std::vector<int>& v) {
            for (int f = 0; f < (int)cost.size(); ++f) v.push_back(f);
        },
        [&](int form) {
            if (launches) ++*launches;
            if (form == fail_form) return 4;  // FA_ERR_HIP
            s->clock += cost[form];
            return 0;
        });
}

int main() {
    // 1. the fastest form wins; the first call runs n untimed + 2 passes x batch launches
    {
        Tuner t(name);
        SimStream s;
        int launches = 0;
        const std::vector<double> cost = {1.0, 0.5, 0.9, 0.49};
        tunersim::not_ready_queries() = 6;  // the last event completes at its 7th query
        CHECK(call(t, &s, 10, 1000, cost, &launches) == 0);
        CHECK(launches == 4 + 2 * 4 * 1);  // bytes 1e12: batch 1
        CHECK(t.chosen(0, 1, 10, 1000, 1000, false) == -1);  // events still "in flight"
        CHECK(t.pending() == 1);
        // calls while the events are in flight run one launch each (the policy's form)
        int later = 0;
        for (int i = 0; i < 3; ++i) call(t, &s, 10, 1000, cost, &later);
        CHECK(later == 3 && t.chosen(0, 1, 10, 1000, 1000, false) == -1);
        CHECK(t.chosen(0, 1, 10, 1000, 1000, false) == 3);  // 7th query: decided
        CHECK(t.pending() == 0);
        tunersim::not_ready_queries() = 2;
    }
    // 2. near-ties keep the policy (3 % margin)
    {
        Tuner t(name);
        SimStream s;
        const std::vector<double> cost = {1.0, 0.98, 0.99};
        call(t, &s, 5, 77, cost, nullptr);
        while (t.pending()) {
        }
        CHECK(t.chosen(0, 1, 5, 77, 77, false) == 0);
    }
    // 3. small folds are timed in batches (~0.3 ms per candidate, at most 32)
    {
        Tuner t(name);
        SimStream s;
        int launches = 0;
        t.run(1, 4, 100, 100, false, 0, 1000.0, &s, [](std::vector<int>& v) { v = {0, 1}; },
              [&](int f) {
                  ++launches;
                  s.clock += f ? 0.01 : 0.02;
                  return 0;
              });
        CHECK(launches == 2 + 2 * 2 * 32);
        while (t.pending()) {
        }
        CHECK(t.chosen(0, 1, 4, 100, 100, false) == 1);
    }
    // 4. a failing launch: its status comes back, the shape keeps the policy
    {
        Tuner t(name);
        SimStream s;
        CHECK(call(t, &s, 3, 30, {1.0, 0.2, 0.3}, nullptr, /*fail_form=*/2) == 4);
        CHECK(t.chosen(0, 1, 3, 30, 30, false) == 0);
        CHECK(t.pending() == 0);
    }
    // 5. graph capture and the off switch: no measurement, the policy runs
    {
        Tuner t(name);
        SimStream s;
        s.capturing = true;
        int launches = 0;
        call(t, &s, 3, 31, {1.0, 0.2}, &launches);
        CHECK(launches == 1 && t.chosen(0, 1, 3, 31, 31, false) == -2);
        s.capturing = false;
        CHECK(t.set_mode(0) == 1);
        launches = 0;
        call(t, &s, 3, 31, {1.0, 0.2}, &launches);
        CHECK(launches == 1 && t.chosen(0, 1, 3, 31, 31, false) == -2);
        CHECK(t.set_mode(1) == 0);
    }
    // 5b. a capture that starts while a measurement is in flight: no event queries
    //     inside it (the policy runs), the decision comes after it
    {
        Tuner t(name);
        SimStream s;
        tunersim::not_ready_queries() = 1;
        call(t, &s, 4, 44, {1.0, 0.3}, nullptr);
        s.capturing = true;
        int launches = 0;
        for (int i = 0; i < 5; ++i) call(t, &s, 4, 44, {1.0, 0.3}, &launches);
        CHECK(launches == 5);
        s.capturing = false;
        call(t, &s, 4, 44, {1.0, 0.3}, nullptr);  // first query after the capture: still in flight
        CHECK(t.chosen(0, 1, 4, 44, 44, false) == 1);
        tunersim::not_ready_queries() = 2;
    }
    // 6. many threads, many shapes, each thread on its own stream and device
    {
        Tuner t(name);
        const int kThreads = 8, kShapes = 24;
        std::vector<std::vector<double>> costs(kShapes);
        std::vector<int> expect(kShapes);
        std::mt19937 rng(7);
        for (int k = 0; k < kShapes; ++k) {
            const int n = 1 + (int)(rng() % 7);
            for (int f = 0; f < n; ++f) costs[k].push_back(0.1 + (rng() % 1000) / 1000.0);
            int b = 0;
            for (int f = 1; f < n; ++f)
                if (costs[k][f] < costs[k][b]) b = f;
            expect[k] = costs[k][b] < 0.97 * costs[k][0] ? b : 0;
        }
        std::vector<std::thread> th;
        for (int i = 0; i < kThreads; ++i)
            th.emplace_back([&, i] {
                tunersim::current_device() = i % 2;
                SimStream s;
                std::mt19937 r(100 + i);
                for (int j = 0; j < 300; ++j) {
                    const int k = (int)(r() % kShapes);
                    const int rc = call(t, &s, 8 + k, 1000 + k, costs[k], nullptr);
                    if (rc != 0) ++g_fail;
                }
            });
        for (auto& x : th) x.join();
        while (t.pending()) {
        }
        for (int dev = 0; dev < 2; ++dev)
            for (int k = 0; k < kShapes; ++k) {
                const int c = t.chosen(dev, 1, 8 + k, 1000 + k, 1000 + k, false);
                CHECK(c == -2 || c == expect[k]);  // -2: this device never saw the shape
            }
    }
    CHECK(tunersim::live_events().load() == 0);  // every measurement's events are released
    if (g_fail) {
        fprintf(stderr, "%d failures\n", g_fail);
        return 1;
    }
    printf("tuner_stress: ok\n");
    return 0;
}
