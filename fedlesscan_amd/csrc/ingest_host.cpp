// Host-side ingest helpers of libfedavg_hip.so (no GPU involved).
//
// Client updates reach the aggregator as uncompressed NPZ blobs
// (NpzWeightsSerializer, fedless/common/serialization.py:280-306; clients use
// compressed=False by default, client.py:186-199).  fa_npz_index locates every
// .npy member's raw payload inside the blob (zip / zip64 central directory ->
// local header -> .npy header), so the engine can copy payloads straight into
// pinned staging; fa_pack does that copy with several threads.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "fedavg_hip.h"
#include "host_copy.hpp"

namespace {

inline uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
inline uint32_t rd32(const uint8_t* p) { return (uint32_t)rd16(p) | ((uint32_t)rd16(p + 2) << 16); }
inline uint64_t rd64(const uint8_t* p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }

constexpr uint32_t kEOCD = 0x06054b50, kZ64Loc = 0x07064b50, kZ64EOCD = 0x06064b50;
constexpr uint32_t kCDir = 0x02014b50, kLocal = 0x04034b50;

// dtype code from a numpy descr string ("<f4", "|u1", ...); 0 = not supported
int dtype_code(const std::string& d, int* itemsize) {
    if (d.size() < 3) return 0;
    const char order = d[0];
    if (order == '>') return 0;  // big-endian payloads are not copied raw
    const std::string k = d.substr(1);
    struct E { const char* s; int code; int sz; };
    static const E table[] = {{"f4", FA_DT_F32, 4}, {"f8", FA_DT_F64, 8}, {"i4", FA_DT_I32, 4},
                              {"i8", FA_DT_I64, 8}, {"f2", FA_DT_F16, 2}, {"u1", FA_DT_U8, 1},
                              {"i1", FA_DT_I8, 1},  {"b1", FA_DT_BOOL, 1}};
    for (const E& e : table)
        if (k == e.s) {
            *itemsize = e.sz;
            return e.code;
        }
    return 0;
}

// Parse the python-dict header of a .npy file: {'descr': '<f4', 'fortran_order': False, 'shape': (3, 4), }
bool parse_npy_header(const char* h, size_t n, std::string* descr, bool* fortran, std::vector<int64_t>* shape) {
    std::string s(h, n);
    auto key = [&](const char* k) -> size_t {
        size_t p = s.find(std::string("'") + k + "'");
        return p == std::string::npos ? p : s.find(':', p);
    };
    size_t p = key("descr");
    if (p == std::string::npos) return false;
    size_t q0 = s.find('\'', p), q1 = q0 == std::string::npos ? q0 : s.find('\'', q0 + 1);
    if (q1 == std::string::npos) return false;
    *descr = s.substr(q0 + 1, q1 - q0 - 1);
    p = key("fortran_order");
    if (p == std::string::npos) return false;
    size_t v = s.find_first_not_of(" ", p + 1);
    if (v == std::string::npos) return false;
    *fortran = s.compare(v, 4, "True") == 0;
    p = key("shape");
    if (p == std::string::npos) return false;
    size_t a = s.find('(', p), b = a == std::string::npos ? a : s.find(')', a);
    if (b == std::string::npos) return false;
    shape->clear();
    const std::string dims = s.substr(a + 1, b - a - 1);
    size_t i = 0;
    while (i < dims.size()) {
        while (i < dims.size() && (dims[i] == ' ' || dims[i] == ',')) ++i;
        if (i >= dims.size()) break;
        if (dims[i] < '0' || dims[i] > '9') return false;
        int64_t x = 0;
        while (i < dims.size() && dims[i] >= '0' && dims[i] <= '9') x = x * 10 + (dims[i++] - '0');
        shape->push_back(x);
    }
    return true;
}

// Persistent host worker pool for fa_pack: creating threads per call cost
// more than the copies of a 128 MB chunk.  run(T, f) executes f(0..T-1) on the
// calling thread plus up to T-1 pool workers and returns when all are done.
class PackPool {
  public:
    static PackPool& get() {
        static PackPool pool;
        return pool;
    }
    void run(int T, const std::function<void(int)>& f) {
        std::unique_lock<std::mutex> call(call_mu_);  // one job at a time
        ensure_workers(T - 1);
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = &f;
            ntasks_ = T;
            next_ = 1;
            pending_ = T - 1;
            ++gen_;
        }
        cv_.notify_all();
        f(0);
        for (;;) {  // the caller helps drain the task list
            int t;
            {
                std::lock_guard<std::mutex> lk(mu_);
                if (next_ >= ntasks_) break;
                t = next_++;
            }
            f(t);
            std::lock_guard<std::mutex> lk(mu_);
            --pending_;
        }
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [&] { return pending_ == 0; });
        job_ = nullptr;
    }
    ~PackPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }

  private:
    void ensure_workers(int n) {
        while ((int)workers_.size() < n) workers_.emplace_back([this] { loop(); });
    }
    void loop() {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            while (job_ && next_ < ntasks_) {
                const int t = next_++;
                const std::function<void(int)>* f = job_;
                lk.unlock();
                (*f)(t);
                lk.lock();
                if (--pending_ == 0) done_cv_.notify_all();
            }
        }
    }
    std::mutex call_mu_, mu_;
    std::condition_variable cv_, done_cv_;
    std::vector<std::thread> workers_;
    const std::function<void(int)>* job_ = nullptr;
    int ntasks_ = 0, next_ = 0, pending_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

// ---- CRC-32 (ISO-HDLC / zlib: reflected polynomial 0xEDB88320) -------------
// The NPZ writer's member checksum (zipfile computes it with zlib.crc32 over
// the .npy header and payload).  Slicing-by-16 tables on each thread over its
// own byte range, then the ranges' CRCs are joined with the GF(2) "shift by
// n zero bytes" operator (the published zlib crc32_combine method: x^(8n)
// mod P by repeated squaring), so any thread count gives zlib's value.
constexpr uint32_t kCrcPoly = 0xEDB88320u;

struct CrcTables {
    uint32_t t[16][256];
    uint32_t x2n[32];  // x^(2^k) mod P
    CrcTables() {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kCrcPoly : c >> 1;
            t[0][i] = c;
        }
        for (uint32_t i = 0; i < 256; ++i)
            for (int s = 1; s < 16; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFF];
        uint32_t p = 1u << 30;  // x^1 (bit 31 is x^0 in the reflected order)
        x2n[0] = p;
        for (int k = 1; k < 32; ++k) x2n[k] = p = mult(p, p);
    }
    // a * b mod P, polynomials in the reflected bit order
    static uint32_t mult(uint32_t a, uint32_t b) {
        uint32_t m = 1u << 31, r = 0;
        for (;;) {
            if (a & m) {
                r ^= b;
                if ((a & (m - 1)) == 0) break;
            }
            m >>= 1;
            b = (b & 1) ? (b >> 1) ^ kCrcPoly : b >> 1;
        }
        return r;
    }
    // x^(8n) mod P
    uint32_t shift_bytes(uint64_t n) const {
        uint32_t p = 1u << 31;  // x^0
        int k = 3;              // 8 = 2^3
        while (n) {
            if (n & 1) p = mult(x2n[k & 31], p);
            n >>= 1;
            ++k;
        }
        return p;
    }
    // raw register update (no pre/post inversion)
    uint32_t update(uint32_t c, const uint8_t* p, size_t n) const {
        while (n && ((uintptr_t)p & 7)) {
            c = t[0][(c ^ *p++) & 0xFF] ^ (c >> 8);
            --n;
        }
        while (n >= 16) {
            uint32_t w0, w1, w2, w3;
            memcpy(&w0, p, 4);
            memcpy(&w1, p + 4, 4);
            memcpy(&w2, p + 8, 4);
            memcpy(&w3, p + 12, 4);
            w0 ^= c;
            c = t[15][w0 & 0xFF] ^ t[14][(w0 >> 8) & 0xFF] ^ t[13][(w0 >> 16) & 0xFF] ^ t[12][w0 >> 24] ^
                t[11][w1 & 0xFF] ^ t[10][(w1 >> 8) & 0xFF] ^ t[9][(w1 >> 16) & 0xFF] ^ t[8][w1 >> 24] ^
                t[7][w2 & 0xFF] ^ t[6][(w2 >> 8) & 0xFF] ^ t[5][(w2 >> 16) & 0xFF] ^ t[4][w2 >> 24] ^
                t[3][w3 & 0xFF] ^ t[2][(w3 >> 8) & 0xFF] ^ t[1][(w3 >> 16) & 0xFF] ^ t[0][w3 >> 24];
            p += 16;
            n -= 16;
        }
        while (n--) c = t[0][(c ^ *p++) & 0xFF] ^ (c >> 8);
        return c;
    }
};

const CrcTables& crc_tables() {
    static const CrcTables tables;
    return tables;
}

}  // namespace

// fa_last_error() text for the host entries (defined in fedavg.hip, hidden:
// not part of the exported ABI)
__attribute__((visibility("hidden"))) int fa_internal_fail(int code, const char* msg);

extern "C" {

static int npz_index_impl(const uint8_t* blob, int64_t len, int64_t* offsets, int64_t* counts, int32_t* dtypes,
                          int32_t* ndims, int64_t* shapes, int max_layers) {
    if (!blob || len < 22) return -1;
    // End of central directory: scan back over at most a 64 KiB comment
    int64_t eocd = -1;
    for (int64_t p = len - 22; p >= 0 && p >= len - 22 - 65535; --p)
        if (rd32(blob + p) == kEOCD) {
            eocd = p;
            break;
        }
    if (eocd < 0) return -1;
    uint64_t n_entries = rd16(blob + eocd + 10);
    uint64_t cd_off = rd32(blob + eocd + 16);
    if (eocd >= 20 && rd32(blob + eocd - 20) == kZ64Loc) {  // zip64
        uint64_t z = rd64(blob + eocd - 20 + 8);
        if (z + 56 > (uint64_t)len || rd32(blob + z) != kZ64EOCD) return -1;
        n_entries = rd64(blob + z + 32);
        cd_off = rd64(blob + z + 48);
    }
    if (n_entries > (uint64_t)max_layers) return -1;
    uint64_t p = cd_off;
    for (uint64_t e = 0; e < n_entries; ++e) {
        if (p + 46 > (uint64_t)len || rd32(blob + p) != kCDir) return -1;
        const uint16_t method = rd16(blob + p + 10);
        uint64_t csize = rd32(blob + p + 20), usize = rd32(blob + p + 24);
        const uint16_t nlen = rd16(blob + p + 28), xlen = rd16(blob + p + 30), clen = rd16(blob + p + 32);
        uint64_t lho = rd32(blob + p + 42);
        if (method != 0) return -1;  // compressed member: needs np.load
        // zip64 extra field (0x0001): fields present only where the 32-bit value is saturated
        uint64_t x = p + 46 + nlen, xend = x + xlen;
        while (x + 4 <= xend && xend <= (uint64_t)len) {
            const uint16_t id = rd16(blob + x), sz = rd16(blob + x + 2);
            if (id == 1) {
                uint64_t f = x + 4;
                if (usize == 0xFFFFFFFFu) { usize = rd64(blob + f); f += 8; }
                if (csize == 0xFFFFFFFFu) { csize = rd64(blob + f); f += 8; }
                if (lho == 0xFFFFFFFFu) { lho = rd64(blob + f); f += 8; }
            }
            x += 4 + sz;
        }
        if (lho + 30 > (uint64_t)len || rd32(blob + lho) != kLocal) return -1;
        const uint64_t data = lho + 30 + rd16(blob + lho + 26) + rd16(blob + lho + 28);
        if (data + 10 > (uint64_t)len || memcmp(blob + data, "\x93NUMPY", 6) != 0) return -1;
        const uint8_t major = blob[data + 6];
        uint64_t hlen, hstart;
        if (major == 1) { hlen = rd16(blob + data + 8); hstart = data + 10; }
        else if ((major == 2 || major == 3) && data + 12 <= (uint64_t)len) { hlen = rd32(blob + data + 8); hstart = data + 12; }
        else return -1;
        if (hstart + hlen > (uint64_t)len) return -1;
        std::string descr;
        bool fortran = false;
        std::vector<int64_t> shape;
        if (!parse_npy_header((const char*)blob + hstart, hlen, &descr, &fortran, &shape)) return -1;
        int itemsize = 0;
        const int code = dtype_code(descr, &itemsize);
        if (!code || fortran || shape.size() > 8) return -1;
        int64_t count = 1;
        for (int64_t d : shape) count *= d;
        const uint64_t payload = hstart + hlen;
        if (payload + (uint64_t)count * itemsize > data + csize || payload + (uint64_t)count * itemsize > (uint64_t)len)
            return -1;
        offsets[e] = (int64_t)payload;
        counts[e] = count;
        dtypes[e] = code;
        ndims[e] = (int32_t)shape.size();
        for (size_t k = 0; k < 8; ++k) shapes[e * 8 + k] = k < shape.size() ? shape[k] : 0;
        p += 46 + nlen + xlen + clen;
    }
    return (int)n_entries;
}

int fa_npz_index(const uint8_t* blob, int64_t len, int64_t* offsets, int64_t* counts, int32_t* dtypes,
                 int32_t* ndims, int64_t* shapes, int max_layers) {
    try {  // nothing may unwind across the C ABI
        return npz_index_impl(blob, len, offsets, counts, dtypes, ndims, shapes, max_layers);
    } catch (...) {
        return -1;
    }
}

int fa_pack(void* dst, const int64_t* dst_offsets, const void* const* srcs, const int64_t* sizes, int64_t n,
            int nthreads) {
    if (n < 0 || (n > 0 && (!dst || !dst_offsets || !srcs || !sizes)))
        return fa_internal_fail(FA_ERR_ARG, "fa_pack: bad arguments");
    // prefix sums of the source sizes: the work is split by bytes, not ranges
    std::vector<int64_t> off(n + 1, 0);
    for (int64_t i = 0; i < n; ++i) {
        if (sizes[i] < 0 || dst_offsets[i] < 0) return fa_internal_fail(FA_ERR_ARG, "fa_pack: negative size or offset");
        off[i + 1] = off[i] + sizes[i];
    }
    const int64_t total = off[n];
    if (total == 0) return FA_OK;
    int T = nthreads > 0 ? nthreads : (int)std::max(1u, std::thread::hardware_concurrency());
    T = (int)std::min<int64_t>(T, std::max<int64_t>(1, total >> 22));  // >= 4 MiB per thread
    auto work = [&](int t) {
        const int64_t b0 = total * t / T, b1 = total * (t + 1) / T;
        int64_t i = std::upper_bound(off.begin(), off.end(), b0) - off.begin() - 1;
        for (int64_t b = b0; b < b1 && i < n; ++i) {
            const int64_t s0 = std::max(b, off[i]), s1 = std::min(b1, off[i + 1]);
            if (s1 > s0)
                fa_host::pack_copy((uint8_t*)dst + dst_offsets[i] + (s0 - off[i]),
                                   (const uint8_t*)srcs[i] + (s0 - off[i]), (size_t)(s1 - s0));
            b = s1;
        }
    };
    if (T == 1) {
        work(0);
        return FA_OK;
    }
    try {
        PackPool::get().run(T, work);
    } catch (...) {  // e.g. thread creation failure: finish on this thread
        for (int t = 0; t < T; ++t) work(t);
    }
    return FA_OK;
}

int fa_crc32(const void* data, int64_t n, uint32_t crc_in, int nthreads, uint32_t* crc_out) {
    if (n < 0 || (n > 0 && !data) || !crc_out) return fa_internal_fail(FA_ERR_ARG, "fa_crc32: bad arguments");
    const CrcTables& K = crc_tables();
    const uint8_t* p = (const uint8_t*)data;
    int T = nthreads > 0 ? nthreads : (int)std::max(1u, std::thread::hardware_concurrency());
    T = (int)std::min<int64_t>(T, std::max<int64_t>(1, n >> 21));  // >= 2 MiB per thread
    if (T == 1) {
        *crc_out = ~K.update(~crc_in, p, (size_t)n);
        return FA_OK;
    }
    // thread t: the raw register over its range starting from 0; range 0 starts from ~crc_in
    std::vector<uint32_t> part(T, 0);
    auto work = [&](int t) {
        const int64_t b0 = n * t / T, b1 = n * (t + 1) / T;
        part[t] = K.update(t == 0 ? ~crc_in : 0u, p + b0, (size_t)(b1 - b0));
    };
    try {
        PackPool::get().run(T, work);
    } catch (...) {
        for (int t = 0; t < T; ++t) work(t);
    }
    // register after range t = (register after t-1) * x^(8 len_t) + part[t]  (CRC linearity)
    uint32_t c = part[0];
    for (int t = 1; t < T; ++t) {
        const int64_t len = n * (t + 1) / T - n * t / T;
        c = CrcTables::mult(K.shift_bytes((uint64_t)len), c) ^ part[t];
    }
    *crc_out = ~c;
    return FA_OK;
}

}  // extern "C"
