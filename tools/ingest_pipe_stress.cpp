// Host-side stress test of the native ingest pipe (csrc/ingest_pipe.cpp) under
// ThreadSanitizer / AddressSanitizer, with the HIP runtime simulated on the host
// (tools/hipsim/) and fa_fold_f32 restated on the CPU (the same in-order
// left fold with separate roundings).  Many rounds on several pipes from
// several threads at once, random chunk sizes, slot counts, piece splits and
// scored / plain rows; every round is compared bit for bit with a direct CPU
// fold of the same rows.  Also: errors mid-round (a short row, mixed scores),
// a round abandoned with a chunk half filled and the pipe reused (bit-exact),
// destroy with copies possibly in flight, and finish with no rows.
//   tools/ingest_pipe_stress.sh   (builds with -fsanitize=thread, then address,undefined)
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <random>
#include <thread>
#include <vector>

#include "fedavg_hip.h"

#pragma clang fp contract(off)
#pragma GCC optimize("fp-contract=off")

static thread_local char g_msg[256] = "";
__attribute__((visibility("hidden"))) int fa_internal_fail(int code, const char* msg) {
    snprintf(g_msg, sizeof(g_msg), "%s", msg);
    return code;
}
extern "C" const char* fa_last_error(void) { return g_msg; }

// CPU restatement of fa_fold_f32 (fedavg_hip.h): acc = [acc_in +] t_0 + t_1 ...; optional divide
extern "C" int fa_fold_f32(const float* X, int64_t N, int64_t P, int64_t ldx, const float* a, const float* s,
                           const float* acc_in, float divisor, int finalize, float* out, void*) {
    for (int64_t p = 0; p < P; ++p) {
        float acc = 0.f;
        int64_t i = 0;
        if (acc_in) {
            acc = acc_in[p];
        } else if (N > 0) {
            float t = X[p] * a[0];
            if (s) t = t * s[0];
            acc = t;
            i = 1;
        }
        for (; i < N; ++i) {
            float t = X[i * ldx + p] * a[i];
            if (s) t = t * s[i];
            acc = acc + t;
        }
        out[p] = finalize ? acc / divisor : acc;
    }
    return FA_OK;
}

static std::atomic<int> g_fail{0};

static void check(bool ok, const char* what) {
    if (!ok) {
        fprintf(stderr, "FAIL: %s\n", what);
        g_fail.fetch_add(1);
    }
}

static void worker(int tid, int rounds) {
    std::mt19937_64 rng(1234 + tid);
    for (int r = 0; r < rounds; ++r) {
        const int64_t P = 1 + rng() % 70000;
        const int64_t N = 1 + rng() % 40;
        const int slots = 2 + rng() % 5;
        const int64_t ldx = (P + 63) / 64 * 64;
        const int64_t chunk = ldx * 4 * (1 + rng() % 6);
        const bool scored = rng() & 1;
        std::vector<float> X(N * P), a(N), s(N);
        for (auto& v : X) v = (float)((int64_t)(rng() % 2001) - 1000) / 1024.f;
        for (int64_t i = 0; i < N; ++i) {
            a[i] = (float)(1 + rng() % 600);
            s[i] = (float)(1 + rng() % 11) / 11.f;
        }
        fa_ingest* pipe = nullptr;
        check(fa_ingest_create(&pipe, P, chunk, slots, tid % 2) == FA_OK, "create");  // two devices: the pool grows
        std::vector<float> acc(P, -1.f);
        for (int rep = 0; rep < 2; ++rep) {  // the pipe is reused
            // the announced row count: unknown, exact, too high, too low (only the chunk sizes change)
            const int64_t guess[4] = {0, N, N + 3, N > 2 ? N - 2 : 1};
            check(fa_ingest_begin(pipe, acc.data(), nullptr, guess[rng() % 4]) == FA_OK, "begin");
            for (int64_t i = 0; i < N; ++i) {
                // the row in 1-4 pieces
                std::vector<const void*> src;
                std::vector<int64_t> sz;
                int64_t off = 0;
                const int parts = 1 + rng() % 4;
                for (int k = 0; k < parts; ++k) {
                    const int64_t len = k == parts - 1 ? P - off : (P - off) * (int64_t)(rng() % 100) / 100;
                    src.push_back(X.data() + i * P + off);
                    sz.push_back(len * 4);
                    off += len;
                }
                check(fa_ingest_add(pipe, src.data(), sz.data(), (int64_t)src.size(), a[i], s[i], scored) == FA_OK,
                      "add");
            }
            float total = 0.f;
            for (int64_t i = 0; i < N; ++i) total = total + a[i];  // exact: small integers
            check(fa_ingest_finish(pipe, total) == FA_OK, "finish");
            std::vector<float> exp(P);
            fa_fold_f32(X.data(), N, P, P, a.data(), scored ? s.data() : nullptr, nullptr, total, 1, exp.data(),
                        nullptr);
            check(memcmp(exp.data(), acc.data(), P * 4) == 0, "bit-exact");
        }
        // errors mid-round, then destroy with copies possibly in flight
        check(fa_ingest_begin(pipe, acc.data(), nullptr, 0) == FA_OK, "begin 2");
        const void* src0 = X.data();
        int64_t full = P * 4, shortb = (P - 1) * 4;
        check(fa_ingest_add(pipe, &src0, &full, 1, 1.f, 1.f, 0) == FA_OK, "add ok");
        check(fa_ingest_add(pipe, &src0, &shortb, 1, 1.f, 1.f, 0) == FA_ERR_SHAPE, "short row rejected");
        check(fa_ingest_add(pipe, &src0, &full, 1, 1.f, 0.5f, 1) == FA_ERR_SHAPE, "mixed scores rejected");
        // abandon that round with a chunk half filled (the second chunk ramps to 2 rows), then
        // reuse the pipe: the abandoned rows must not join the next round
        check(fa_ingest_add(pipe, &src0, &full, 1, 7.f, 1.f, 0) == FA_OK, "add ok 2");
        check(fa_ingest_begin(pipe, acc.data(), nullptr, 0) == FA_OK, "begin after an abandoned round");
        for (int64_t i = 0; i < N; ++i) {
            const void* src = X.data() + i * P;
            check(fa_ingest_add(pipe, &src, &full, 1, a[i], s[i], 0) == FA_OK, "add after abandon");
        }
        {
            float total = 0.f;
            for (int64_t i = 0; i < N; ++i) total = total + a[i];
            check(fa_ingest_finish(pipe, total) == FA_OK, "finish after abandon");
            std::vector<float> exp(P);
            fa_fold_f32(X.data(), N, P, P, a.data(), nullptr, nullptr, total, 1, exp.data(), nullptr);
            check(memcmp(exp.data(), acc.data(), P * 4) == 0, "bit-exact after an abandoned round");
        }
        // abandoned again, now with copies possibly in flight: destroy
        check(fa_ingest_begin(pipe, acc.data(), nullptr, 0) == FA_OK, "begin 4");
        for (int k = 0; k < 3; ++k) check(fa_ingest_add(pipe, &src0, &full, 1, 1.f, 1.f, 0) == FA_OK, "add 3");
        fa_ingest_destroy(pipe);
        fa_ingest* empty = nullptr;
        check(fa_ingest_create(&empty, P, chunk, slots, 0) == FA_OK, "create 2");
        check(fa_ingest_begin(empty, acc.data(), nullptr, 5) == FA_OK, "begin 3");
        check(fa_ingest_finish(empty, 1.f) == FA_ERR_NO_CLIENTS, "empty round");
        fa_ingest_destroy(empty);
    }
}

int main() {
    std::vector<std::thread> ts;
    for (int t = 0; t < 3; ++t) ts.emplace_back(worker, t, 12);
    for (auto& t : ts) t.join();
    if (g_fail.load()) {
        fprintf(stderr, "%d failures\n", g_fail.load());
        return 1;
    }
    printf("ingest_pipe_stress: ok\n");
    return 0;
}
