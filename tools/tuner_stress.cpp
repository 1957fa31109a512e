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
#include <chrono>
#include <fcntl.h>
#include <sys/file.h>
#include <cstring>
#include <string>
#include <unistd.h>
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
static int from_name(int kind, const char* nm) {
    (void)kind;
    for (int f = 0; f < 8; ++f)
        if (strcmp(name(1, f), nm) == 0) return f;
    return -1;
}
static std::string ident(int dev) { return "sim:" + std::to_string(dev); }
static std::string slurp(const std::string& p) {
    std::string s;
    FILE* f = fopen(p.c_str(), "rb");
    if (!f) return s;
    char b[4096];
    size_t k;
    while ((k = fread(b, 1, sizeof(b), f)) > 0) s.append(b, k);
    fclose(f);
    return s;
}
static void spit(const std::string& p, const std::string& text) {
    FILE* f = fopen(p.c_str(), "wb");
    fwrite(text.data(), 1, text.size(), f);
    fclose(f);
}
static int count_lines(const std::string& s) {
    int n = 0;
    for (char c : s) n += c == '\n';
    return n;
}
// settle every measurement in flight
static void drain(Tuner& t) {
    while (t.pending()) {
    }
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
        CHECK(t.chosen(0, 1, 10, 0, 1000, 1000, false) == -1);  // events still "in flight"
        CHECK(t.pending() == 1);
        // calls while the events are in flight run one launch each (the policy's form)
        int later = 0;
        for (int i = 0; i < 3; ++i) call(t, &s, 10, 1000, cost, &later);
        CHECK(later == 3 && t.chosen(0, 1, 10, 0, 1000, 1000, false) == -1);
        CHECK(t.chosen(0, 1, 10, 0, 1000, 1000, false) == 3);  // 7th query: decided
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
        CHECK(t.chosen(0, 1, 5, 0, 77, 77, false) == 0);
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
        CHECK(t.chosen(0, 1, 4, 0, 100, 100, false) == 1);
    }
    // 4. a failing launch: its status comes back, the shape keeps the policy
    {
        Tuner t(name);
        SimStream s;
        CHECK(call(t, &s, 3, 30, {1.0, 0.2, 0.3}, nullptr, /*fail_form=*/2) == 4);
        CHECK(t.chosen(0, 1, 3, 0, 30, 30, false) == 0);
        CHECK(t.pending() == 0);
    }
    // 5. graph capture and the off switch: no measurement, the policy runs
    {
        Tuner t(name);
        SimStream s;
        s.capturing = true;
        int launches = 0;
        call(t, &s, 3, 31, {1.0, 0.2}, &launches);
        CHECK(launches == 1 && t.chosen(0, 1, 3, 0, 31, 31, false) == -2);
        s.capturing = false;
        CHECK(t.set_mode(0) == 1);
        launches = 0;
        call(t, &s, 3, 31, {1.0, 0.2}, &launches);
        CHECK(launches == 1 && t.chosen(0, 1, 3, 0, 31, 31, false) == -2);
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
        CHECK(t.chosen(0, 1, 4, 0, 44, 44, false) == 1);
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
                const int c = t.chosen(dev, 1, 8 + k, 0, 1000 + k, 1000 + k, false);
                CHECK(c == -2 || c == expect[k]);  // -2: this device never saw the shape
            }
    }
    // 7. client counts share a power-of-two bucket: a shape measured at 1000
    //    clients runs its decision at 1024 without a measurement; 1025 measures
    {
        Tuner t(name);
        SimStream s;
        const std::vector<double> cost = {1.0, 0.4};
        call(t, &s, 1000, 500, cost, nullptr);
        drain(t);
        int launches = 0;
        call(t, &s, 1024, 500, cost, &launches);
        CHECK(launches == 1 && t.chosen(0, 1, 513, 0, 500, 500, false) == 1);
        launches = 0;
        call(t, &s, 1025, 500, cost, &launches);
        CHECK(launches > 1);
        drain(t);
    }
    // 8. the cache file: a decision of one process is the first call's form in the next
    char dir[] = "/tmp/fa_tuner_stress_XXXXXX";
    CHECK(mkdtemp(dir) != nullptr);
    const std::string path = std::string(dir) + "/sub/tuner.txt";  // the directory is created
    {
        Tuner a(name, from_name, ident, 3);
        a.set_cache_path(path);
        SimStream s;
        call(a, &s, 64, 7000, {1.0, 0.9, 0.3}, nullptr);
        drain(a);
        CHECK(a.chosen(0, 1, 64, 0, 7000, 7000, false) == 2);
        CHECK(count_lines(slurp(path)) == 1);
        Tuner b(name, from_name, ident, 3);
        b.set_cache_path(path);
        int launches = 0;
        call(b, &s, 60, 7000, {1.0, 0.9, 0.3}, &launches);  // same bucket
        CHECK(launches == 1 && b.chosen(0, 1, 64, 0, 7000, 7000, false) == 2);
        // another device identity does not take it
        tunersim::current_device() = 1;
        launches = 0;
        call(b, &s, 64, 7000, {1.0, 0.9, 0.3}, &launches);
        CHECK(launches > 1);
        drain(b);
        tunersim::current_device() = 0;
        CHECK(count_lines(slurp(path)) == 2);
    }
    // 9. a stale ABI: the lines are ignored (measured again), and dropped on rewrite
    {
        Tuner c(name, from_name, ident, 4);
        c.set_cache_path(path);
        SimStream s;
        int launches = 0;
        call(c, &s, 64, 7000, {1.0, 0.2, 0.3}, &launches);
        CHECK(launches > 1);
        drain(c);
        CHECK(c.chosen(0, 1, 64, 0, 7000, 7000, false) == 1);
        const std::string after = slurp(path);
        CHECK(count_lines(after) == 1 && after.find(" 4 1 64 f0 7000 7000 0 f1") != std::string::npos);
    }
    // 10. a corrupt file: garbage, truncated and out-of-range lines are skipped,
    //     the valid line is used, and the rewrite keeps only valid lines
    {
        spit(path, std::string("garbage \x01\x02 here\n") + "fedavg-tune 1 sim:0 5 1 64 f0 9000 9000 0 f2\n" +
                       "fedavg-tune 1 sim:0 5 1 64 f0 900\n" + "fedavg-tune 1 sim:0 5 1 63 f0 100 100 0 f1\n" +
                       "fedavg-tune 1 sim:0 5 1 64 f0 100 50 0 f1\n" + "fedavg-tune 1 sim:0 5 1 64 f0 100 100 0 f9\n" +
                       std::string(5000, 'x') + "\nfedavg-tune 1 sim:0 5 1 64 f0 800 800 0 f1 extra\n");
        Tuner d(name, from_name, ident, 5);
        d.set_cache_path(path);
        SimStream s;
        int launches = 0;
        call(d, &s, 64, 9000, {1.0, 0.9, 0.95}, &launches);
        CHECK(launches == 1 && d.chosen(0, 1, 64, 0, 9000, 9000, false) == 2);
        call(d, &s, 64, 100, {1.0, 0.5}, &launches);  // the malformed lines for P = 100 did not count
        CHECK(launches > 2);
        drain(d);
        const std::string after = slurp(path);
        CHECK(count_lines(after) == 2 && after.find("garbage") == std::string::npos);
    }
    // 11. export / import: another process's decisions replace this one's
    {
        Tuner e(name, from_name, ident, 6), f(name, from_name, ident, 6);
        e.set_cache_path("");
        f.set_cache_path("");
        SimStream s;
        call(e, &s, 32, 3000, {1.0, 0.5, 0.2}, nullptr);
        call(f, &s, 32, 3000, {1.0, 0.2, 0.5}, nullptr);
        drain(e);
        drain(f);
        CHECK(e.chosen(0, 1, 32, 0, 3000, 3000, false) == 2 && f.chosen(0, 1, 32, 0, 3000, 3000, false) == 1);
        const std::string text = e.export_text();
        CHECK(count_lines(text) == 1);
        CHECK(f.import_text(text + "not a line\n") == 1);
        CHECK(f.chosen(0, 1, 32, 0, 3000, 3000, false) == 2);
        // an imported shape this process has not seen runs without measuring
        CHECK(f.import_text("fedavg-tune 1 sim:0 6 1 32 f0 4000 4000 1 f3\n") == 1);
        int launches = 0;
        f.run(1, 20, 4000, 4000, true, 0, 1e12, &s, [](std::vector<int>& v) { v = {0, 1, 2, 3}; },
              [&](int form) {
                  ++launches;
                  CHECK(form == 3);
                  return 0;
              });
        CHECK(launches == 1);
        // import while a measurement is in flight: the events are released, the import wins
        tunersim::not_ready_queries() = 50;
        call(f, &s, 8, 5000, {1.0, 0.5}, nullptr);
        CHECK(f.chosen(0, 1, 8, 0, 5000, 5000, false) == -1);
        CHECK(f.import_text("fedavg-tune 1 sim:0 6 1 8 f0 5000 5000 0 f0\n") == 1);
        CHECK(f.chosen(0, 1, 8, 0, 5000, 5000, false) == 0);
        tunersim::not_ready_queries() = 2;
    }
    // 12. several processes (tuners) deciding shapes at once: every line survives the merges
    {
        const std::string p2 = std::string(dir) + "/many.txt";
        std::vector<std::thread> th;
        for (int i = 0; i < 6; ++i)
            th.emplace_back([&, i] {
                Tuner t(name, from_name, ident, 7);
                t.set_cache_path(p2);
                SimStream s;
                for (int k = 0; k < 10; ++k) call(t, &s, 16, 20000 + 10 * i + k, {1.0, 0.3}, nullptr);
                drain(t);
            });
        for (auto& x : th) x.join();
        CHECK(count_lines(slurp(p2)) == 60);
        Tuner g(name, from_name, ident, 7);
        g.set_cache_path(p2);
        SimStream s;
        int launches = 0;
        for (int i = 0; i < 6; ++i)
            for (int k = 0; k < 10; ++k) call(g, &s, 16, 20000 + 10 * i + k, {1.0, 0.3}, &launches);
        CHECK(launches == 60);
        unlink(p2.c_str());
        unlink((p2 + ".lock").c_str());
    }
    // 13. step-form decisions: recorded by one tuner, found by the next without
    //     measuring; kept beside kernel lines through merges; malformed keys
    //     and another ABI refused; carried by export / import
    {
        const std::string p3 = std::string(dir) + "/steps.txt";
        const std::string key = "sim:0 bf16 8 256 100000000 3456,2432,1664,1152";
        {
            Tuner a(name, from_name, ident, 8);
            a.set_cache_path(p3);
            CHECK(a.step_lookup(key) == -1);
            CHECK(a.step_record(key, true));
            CHECK(a.step_lookup(key) == 1);
            CHECK(a.step_lookup("sim:0  bf16 8 256 100000000  3456,2432,1664,1152") == 1);  // canonical spacing
            CHECK(!a.step_record("sim:0 f16 8 256 100 64", true));       // dtype
            CHECK(!a.step_record("sim:0 f32 8 255 100 64", true));       // bucket not a power of two
            CHECK(!a.step_record("sim:0 f32 8 256 100 64,", true));      // trailing comma
            CHECK(!a.step_record("sim:0 f32 8 256 100 0,64", true));     // empty slot
            CHECK(!a.step_record("sim:0 f32 8 256 100 1,2,3,4,5,6,7,8,9", true));  // > 8 rounds
            CHECK(a.step_lookup("sim:0 f32 8 256 100") == -2);
            SimStream s;
            call(a, &s, 64, 7100, {1.0, 0.3}, nullptr);  // a kernel line in the same file
            drain(a);
            CHECK(a.step_record("sim:0 f32 8 1024 10000000 327680,327680,327680,40960", false));
        }
        const std::string text = slurp(p3);
        CHECK(count_lines(text) == 3 && text.find(" one\n") != std::string::npos && text.find(" per\n") != std::string::npos);
        {
            Tuner b(name, from_name, ident, 8);
            b.set_cache_path(p3);
            CHECK(b.step_lookup(key) == 1);
            CHECK(b.step_lookup("sim:0 f32 8 1024 10000000 327680,327680,327680,40960") == 0);
            CHECK(b.step_record(key, false));  // a new decision replaces the line
            const std::string ex = b.export_text();
            Tuner c(name, from_name, ident, 8);
            c.set_cache_path("");
            CHECK(c.import_text(ex) == 2 && c.step_lookup(key) == 0);
        }
        CHECK(count_lines(slurp(p3)) == 3 && slurp(p3).find(" one\n") == std::string::npos);
        {
            Tuner d(name, from_name, ident, 9);  // another ABI: the lines do not count
            d.set_cache_path(p3);
            CHECK(d.step_lookup(key) == -1);
        }
        // the file lock held elsewhere: a decision returns at once (bounded
        // retry), stays in memory, and reaches the file on a later call
        {
            const int held = open((p3 + ".lock").c_str(), O_RDWR | O_CREAT, 0644);
            CHECK(held >= 0 && flock(held, LOCK_EX) == 0);
            Tuner e(name, from_name, ident, 8);
            e.set_cache_path(p3);
            const auto t0 = std::chrono::steady_clock::now();
            CHECK(e.step_record("sim:0 f32 2 64 4096 1024,1024", true));
            const double ms =
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            CHECK(ms < 500.0);
            CHECK(e.step_lookup("sim:0 f32 2 64 4096 1024,1024") == 1);
            CHECK(slurp(p3).find("4096 1024,1024") == std::string::npos);
            flock(held, LOCK_UN);
            close(held);
            CHECK(e.step_record("sim:0 f32 2 64 8192 2048,2048", false));  // flushes both
            CHECK(slurp(p3).find("4096 1024,1024 one") != std::string::npos);
            CHECK(slurp(p3).find("8192 2048,2048 per") != std::string::npos);
        }
        unlink(p3.c_str());
        unlink((p3 + ".lock").c_str());
    }
    unlink(path.c_str());
    unlink((path + ".lock").c_str());
    rmdir((std::string(dir) + "/sub").c_str());
    rmdir(dir);
    CHECK(tunersim::live_events().load() == 0);  // every measurement's events are released
    if (g_fail) {
        fprintf(stderr, "%d failures\n", g_fail);
        return 1;
    }
    printf("tuner_stress: ok\n");
    return 0;
}
