// host_copy.hpp — the host-side copy of the ingest packers (fa_pack,
// ingest_pipe.cpp): pageable client rows -> page-locked staging that the DMA
// engine reads next.  Large copies use non-temporal (streaming) stores: the
// staging is written once and read by the DMA engine, never by this CPU, so
// regular stores would only cost a read-for-ownership of every destination
// line and evict the source rows from the caches.  FEDAVG_PACK_NT=0 selects
// plain memcpy.  Runtime dispatch: AVX2 where the CPU has it, memcpy otherwise.
#pragma once
#include <immintrin.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

namespace fa_host {

__attribute__((target("avx2"))) inline void stream_copy_avx2(uint8_t* dst, const uint8_t* src, size_t n) {
    size_t head = (32 - ((uintptr_t)dst & 31)) & 31;
    if (head > n) head = n;
    memcpy(dst, src, head);
    dst += head;
    src += head;
    n -= head;
    size_t i = 0;
    for (; i + 128 <= n; i += 128) {
        const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i));
        const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 32));
        const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 64));
        const __m256i d = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 96));
        _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i), a);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 32), b);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 64), c);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 96), d);
    }
    memcpy(dst + i, src + i, n - i);
    _mm_sfence();  // the streaming stores are globally visible before the task reports done
}

inline bool stream_copy_enabled() {
    static const bool on = [] {
        const char* e = getenv("FEDAVG_PACK_NT");
        return !(e && e[0] == '0') && __builtin_cpu_supports("avx2");
    }();
    return on;
}

// Copy n bytes; streaming stores from 64 KiB up (below that the copy stays in cache anyway).
inline void pack_copy(void* dst, const void* src, size_t n) {
    if (n >= (64u << 10) && stream_copy_enabled())
        stream_copy_avx2(static_cast<uint8_t*>(dst), static_cast<const uint8_t*>(src), n);
    else
        memcpy(dst, src, n);
}

}  // namespace fa_host
