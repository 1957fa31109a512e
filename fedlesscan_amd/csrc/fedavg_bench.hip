// libfedavg_hip_bench.so — bench and tuning support, NOT the product ABI
// (include/fedavg_hip_bench.h): the integer-exact synthetic generator that
// fills HBM for bench.py and the GPU tests, the streaming-read calibration
// kernel, and the kernel-variant sweep entry points (variant 0 = the product's
// auto fold, the rest = alternatives kept for `bench.py --sweep`).  Shares the
// kernels of fold_kernels.hpp with libfedavg_hip.so.
#include "fold_kernels.hpp"
#include "fedavg_hip_bench.h"

namespace {

// Bijective blockIdx remap that gives each of the 8 XCDs (blocks b and b+8
// share one under round-robin dispatch) a contiguous range of column tiles.
// Placement is a speed hint only; any placement gives the same result.
__device__ __forceinline__ int64_t xcd_contiguous(int64_t b, int64_t n) {
    const int64_t q = n / 8, r = n % 8, x = b % 8, k = b / 8;
    return x * q + (x < r ? x : r) + k;
}

template <int U, int C, bool NT, bool SCORED, bool ACC, bool FIN, bool XR = false, bool NTS = false>
__global__ __launch_bounds__(kBlock) void k_fold_f32_v4(
    const float* __restrict__ X, int64_t N, int64_t P, int64_t ldx,
    const float* __restrict__ a, const float* __restrict__ s,
    const float* acc_in, float divisor, float* out) {  // acc_in may alias out
    const int64_t bid = XR ? xcd_contiguous(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
    fold_tile<U, C, NT, SCORED, ACC, FIN, NTS>(bid, X, N, P, ldx, a, s, acc_in, divisor, out);
}

// Balanced persistent form: the grid is the resident capacity (occupancy x
// CUs) and block b owns the contiguous quad range [b*per, (b+1)*per), per =
// ceil(nq / grid): every CU streams the same number of bytes, so there is no
// partly-filled last wave of blocks.  Inside its range a block walks tiles of
// C*kBlock quads; the same fold_quads body does the work.
template <int U, int C, bool NT, bool SCORED, bool ACC, bool FIN>
__global__ __launch_bounds__(kBlock) void k_fold_f32_balanced(
    const float* __restrict__ X, int64_t N, int64_t P, int64_t ldx,
    const float* __restrict__ a, const float* __restrict__ s,
    const float* acc_in, float divisor, float* out, int64_t per) {  // acc_in may alias out
    const int64_t nq = P >> 2;
    const int64_t ldq = ldx >> 2;
    const f32x4* X4 = reinterpret_cast<const f32x4*>(X);
    const f32x4* A4 = reinterpret_cast<const f32x4*>(acc_in);
    f32x4* O4 = reinterpret_cast<f32x4*>(out);
    const int64_t lo = (int64_t)blockIdx.x * per;
    const int64_t hi = lo + per < nq ? lo + per : nq;
    int64_t q0 = lo + threadIdx.x;
    for (; q0 + (int64_t)(C - 1) * kBlock < hi; q0 += (int64_t)C * kBlock)
        fold_quads<U, C, NT, SCORED, ACC, FIN>(X4 + q0, ldq, N, a, s, ACC ? A4 + q0 : nullptr, divisor, O4 + q0);
    for (; q0 < hi; q0 += kBlock)
        fold_quads<U, 1, NT, SCORED, ACC, FIN>(X4 + q0, ldq, N, a, s, ACC ? A4 + q0 : nullptr, divisor, O4 + q0);
    if ((P & 3) && blockIdx.x == gridDim.x - 1 && threadIdx.x == kBlock - 1) {
        for (int64_t col = nq * 4; col < P; ++col) {
            float acc;
            int64_t i = 0;
            if constexpr (ACC) {
                acc = acc_in[col];
            } else {
                acc = term1<SCORED>(X[col], a[0], SCORED ? s[0] : 1.0f);
                i = 1;
            }
            for (; i < N; ++i) acc = acc + term1<SCORED>(X[i * ldx + col], a[i], SCORED ? s[i] : 1.0f);
            if constexpr (FIN) acc = acc / divisor;
            out[col] = acc;
        }
    }
}

// ---------------------------------------------------------------------------
// synthetic generator (bit-identical to fedlesscan_amd/synth.py)
// ---------------------------------------------------------------------------
constexpr uint64_t kGolden = 0x9E3779B97F4A7C15ULL;
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
__device__ __forceinline__ float synth_value(uint64_t key, int64_t col) {
    uint64_t h = mix64(key + (uint64_t)(col + 1) * kGolden);
    int64_t v = (int64_t)(h & 0x1FFFFF) + (int64_t)((h >> 21) & 0x1FFFFF) +
                (int64_t)((h >> 42) & 0x1FFFFF) - 3 * (1 << 20);
    return (float)v * 0x1p-24f;
}

template <typename OutT>
__global__ __launch_bounds__(kBlock) void k_synth(OutT* __restrict__ X, int64_t nrows, int64_t ncols,
                                                   int64_t ldx, uint64_t seed, int64_t row0, int64_t col0) {
    const int64_t total = nrows * ncols;
    for (int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * kBlock) {
        const int64_t r = e / ncols;
        const int64_t c = e - r * ncols;
        const uint64_t key = mix64((seed * kGolden) ^ mix64((uint64_t)(row0 + r) + 1));
        const float v = synth_value(key, col0 + c);
        if constexpr (sizeof(OutT) == 4) X[r * ldx + c] = v;
        else X[r * ldx + c] = f2bf_rne(v);
    }
}

// Contiguous streaming read (calibration ceiling for the fold): block b reads
// its own contiguous 64 KiB chunk (16 independent 16-byte non-temporal loads
// per lane, all issued before the first use), the fastest pure-read pattern
// measured on MI355X (tools/hbm_probe.hip "chunk nt 64 KiB/block").
constexpr int kSweepQuads = 16 * kBlock;  // 64 KiB per block
__global__ __launch_bounds__(kBlock) void k_read_sweep(const f32x4* __restrict__ X, int64_t nq,
                                                        float* __restrict__ sink, int64_t sink_len) {
    const int64_t q0 = (int64_t)blockIdx.x * kSweepQuads + threadIdx.x;
    f32x4 v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int64_t q = q0 + (int64_t)k * kBlock;
        v[k] = q < nq ? __builtin_nontemporal_load(X + q) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    f32x4 acc = v[0];
#pragma unroll
    for (int k = 1; k < 16; ++k) acc = add4(acc, v[k]);
    float t = acc.x + acc.y + acc.z + acc.w;
    for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
    __shared__ float red[kBlock / 64];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0) sink[blockIdx.x % sink_len] = red[0] + red[1] + red[2] + red[3];
}

// Grid-stride copy on a fixed number of blocks (fa_bench_copy_f32).
__global__ __launch_bounds__(kBlock) void k_bench_copy(f32x4* __restrict__ dst, const f32x4* __restrict__ src,
                                                       int64_t nq) {
    for (int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x; q < nq; q += (int64_t)gridDim.x * kBlock)
        __builtin_nontemporal_store(__builtin_nontemporal_load(src + q), dst + q);
}

// Variant 0 is the product's auto fold (fold_f32_auto); the others are the
// alternatives whose sweeps chose it (profiles/r01_sweep_*.log).
// Names: u<rows ahead>c<quads per lane>, nt = non-temporal loads, _nts =
// non-temporal output stores; gs<k> grid-stride with k blocks per CU, gsbal
// balanced passes, gsq<n> n blocks, gsband<k> column bands of k passes;
// lds[2]_w<waves>r<rows per chunk>t<quads per block> LDS-staged (2 = two chunks
// in flight); bal_ balanced persistent grid; xcd_ XCD-contiguous block order.
constexpr const char* kVariants[] = {
    "auto",
    // one block per tile (the round-1 row-streaming kernel)
    "u8c4nt", "u4c1nt", "xcd_u8c4nt", "v4_pickq_nts", "bal_u4c4nt",
    // grid-stride over 16 KiB tiles
    "gs1_u8c4nt_nts", "gs2_u8c4nt_nts", "gs1_u4c8nt_nts", "gs1b512_u8c2nt_nts",
    "gsbal_u8c4nt_nts", "gsbal_u8c2nt_nts", "gsq192_u8c4nt_nts",
    "gsband2_u8c4nt_nts", "gsband3_u8c4nt_nts", "gsband4_u8c4nt_nts", "gsband6_u8c4nt_nts",
    // LDS-staged narrow folds
    "lds_w8r64t32", "lds_w4r64t64", "lds_w16r128t64",
    "lds2_w4r32t16", "lds2_w4r16t32", "lds2_w4r64t32", "lds2_w8r32t32", "lds2_w4r32t8", "lds2_w2r32t16",
    // LDS-DMA ring: ring_w<waves>r<rows per chunk>t<quads per block>s<slots>
    "ring_w4r32t16s4", "ring_w4r32t16s6", "ring_w4r32t16s8", "ring_w4r32t32s4", "ring_w4r32t32s6",
    "ring_w4r64t16s4", "ring_w4r16t32s8", "ring_w8r64t32s3", "ring_w4r32t8s8", "ring_w2r32t16s8",
    // register-staged LDS fold with <d> chunks in flight: lds<d>_w..r..t..
    "lds3_w4r32t16", "lds4_w4r32t16", "lds6_w4r32t16", "lds4_w4r16t32", "lds3_w4r16t32", "lds4_w2r32t16",
    "lds4_w4r32t8", "lds3_w8r32t32", "lds4_w4r64t32",
    // one-wave blocks, one quad per lane, U rows in flight in registers (gsw<threads>_u<rows>)
    "gsw64_u16c1", "gsw64_u32c1", "gsw64_u48c1", "gsw128_u32c1", "gsw64_u24c2",
    // non-power-of-two column tiles (more blocks per CU at the same row segment length)
    "lds2_w4r32t24", "lds2_w4r64t20", "lds2_w4r32t40", "lds2_w2r16t32", "lds2_w4r16t48", "lds2_w4r64t28",
    // the round-2 quad fold (wave 0 alone, lane = quad) of the product's LDS picks, for A/B
    "qf_lds4_w4r32t16", "qf_lds2_w4r32t16", "qf_lds2_w4r32t24", "qf_lds2_w4r16t32", "qf_lds2_w4r32t40",
    "qf_lds_w8r64t32",
    // column fold, more tile shapes (one column per lane)
    "lds4_w4r16t16", "lds4_w2r32t8", "lds4_w4r64t16", "lds6_w4r64t16", "lds4_w8r64t16", "lds2_w2r32t4",
    // loader A/B on the product picks: o<LOPT>[q]_... (bit 0: every lane loads a factor;
    // bit 1: a scheduling barrier after each stage's loads; q: quad fold)
    "o0q_lds4_w4r32t16", "o0q_lds2_w4r32t24", "o0q_lds2_w4r16t32", "o0q_lds2_w4r32t40",
    "o1_lds4_w4r32t16", "o1_lds2_w4r32t24", "o1_lds2_w4r16t32", "o1_lds2_w4r32t40",
    "o2_lds4_w4r32t16", "o2_lds2_w4r32t24", "o2_lds2_w4r16t32", "o2_lds2_w4r32t40",
    "o0_lds4_w4r32t16", "o0_lds2_w4r32t24", "o0_lds2_w4r16t32", "o0_lds2_w4r32t40",
    // 4-byte loads (rows not 16-B aligned; these also run on unaligned input), and
    // the per-column scalar fold the product used for such input in round 2
    "dw_lds4_w2r32t16", "dw_lds2_w4r32t24", "dw_lds2_w4r16t32", "dw_lds2_w4r32t40", "dw_lds2_w8r32t32",
    "dw_lds2_w4r64t32", "dw_lds3_w8r32t32", "scalar",
    // one block per tile (the product's few-client form, k_fold_f32_tile), more rows or quads per lane
    "tile_u8c1", "tile_u16c1", "tile_u8c2", "tile_u4c2", "tile_u8c1_nts", "tile_u4c1",
    // even split: one block per CU (g2: two) owning ceil(nq / blocks) contiguous quads,
    // auto = quads per lane from the range (k_fold_f32_even, round 3)
    "even_auto", "even_g2_auto", "even_u16c2", "even_u32c1", "even_u8c4", "even_u4c4", "even_g2_u8c2",
    "even_g4_auto",
    // one wave per 64 columns, LDS-DMA chunks, no barriers (k_fold_f32_w1, round 3): w1_r<rows>s<slots>
    "w1_r32s6", "w1_r64s4", "w1_r16s12", "w1_r32s8",
    // the column fold with the terms formed by the loaders (LOPT bit 3, k_fold_f32_lds, round 3):
    // the product's LDS picks, two deeper forms, and the 4-byte-load pick
    "pm_lds4_w2r32t16", "pm_lds2_w2r32t16", "pm_lds2_w4r32t24", "pm_lds2_w4r32t40", "pm_lds2_w2r16t32",
    "pm_lds1_w8r64t32", "pm_lds4_w4r32t16", "pm_lds6_w2r32t16", "pm_dw_lds4_w2r32t16",
    // more bytes in flight per block: deeper pipelines, 64-row chunks
    "pm_lds8_w2r32t16", "pm_lds10_w2r32t16", "pm_lds4_w2r64t16", "pm_lds6_w2r64t16",
    // the same with a scheduling barrier after each stage's loads (LOPT 8|2: exact wait counts)
    "pm_o2_lds6_w2r32t16", "pm_o2_lds4_w2r32t16", "pm_o2_lds4_w4r32t16", "pm_o2_lds8_w2r32t16",
};
constexpr int kFirstAnyAlign = 84;  // variants [kFirstAnyAlign, kEndAnyAlign) take any 4-B aligned layout
constexpr int kEndAnyAlign = 92;
constexpr int kPmDw = 118;  // and this one
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);
static_assert(kNumVariants > kPmDw, "pm_dw_lds4_w2r32t16 is variant 118");

// Quads per lane of the round-1 row-streaming policy (variant "v4_pickq_nts"):
// the widest per-block row run (C * 4 KiB) that still leaves >= ~1000 blocks.
inline int pick_quads(int64_t P) {
    const int64_t nq = P >> 2;
    if (nq / (4 * kBlock) >= 1000) return 4;
    if (nq / (2 * kBlock) >= 1000) return 2;
    return 1;
}

constexpr const char* kBf16Variants[] = {
    "bf16auto",
    // one block per tile, u<rows ahead>c<octets per lane>
    "bf16u8c1", "bf16u8c2", "bf16u2c8",
    // grid-stride (gs1: one block per CU; gsbal: balanced passes)
    "bf16gs1u8c2", "bf16gs1u8c4", "bf16gsbalu8c2", "bf16gsbalu2c8",
    // column bands of <k> passes
    "bf16band2u2c8", "bf16band4u2c8", "bf16band4u8c2",
    "bf16band4u16c2", "bf16band4u8c4", "bf16band4u4c4", "bf16band3u8c2", "bf16band4u16c1",
};
constexpr int kNumBf16Variants = sizeof(kBf16Variants) / sizeof(kBf16Variants[0]);
constexpr const char* kPtrsVariants[] = {
    "ptrs_o0_t16", "ptrs_o4_t16", "ptrs_o0_t24", "ptrs_o4_t24", "ptrs_o0_t32", "ptrs_o4_t32",
    "ptrs_o0_t40", "ptrs_o4_t40", "ptrs_o0q_t24", "ptrs_o4_t16d4", "ptrs_o0_t16d4",
    "ptrs_o0_w2t16d4", "ptrs_o4_w2t16d4", "ptrs_o0_w8r64t32",
    // any row alignment (4-byte loads / lane = column / the round-2 generic kernel)
    "ptrs_dw_w2t16d4", "ptrs_dw_t40", "ptrs_dw_t32", "ptrs_dw_t24", "ptrs_rows_scalar", "ptrs_generic",
    // two-wave forms of the stacked fold's 32K-256K picks (16-B aligned rows again)
    "ptrs_o0_w2t32", "ptrs_o4_w2t32", "ptrs_o0_w2t16d2", "ptrs_o4_w2t16d2",
    // the loaders form the terms (LOPT bit 3), with and without the pointer ring (round 3)
    "ptrs_o12_w2t16d4", "ptrs_o12_w2t16d6", "ptrs_o8_w2t16d6", "ptrs_o8_w2t16d4",
    // with a scheduling barrier per stage (bit 1: exact stash waits)
    "ptrs_o14_w2t16d6", "ptrs_o6_w2t16d4", "ptrs_o14_w2t16d4",
};
constexpr int kNumPtrsVariants = sizeof(kPtrsVariants) / sizeof(kPtrsVariants[0]);


// Resident blocks of one balanced-kernel instantiation on the current device
// (occupancy API x CU count), cached per (instantiation, device).  The guide
// notes the API can over-report by one block per CU for SGPR-heavy 256-thread
// kernels; for a plain (non-cooperative) launch that only costs balance.
template <int U, int C, bool NT, bool SC, bool ACC, bool FIN>
int resident_blocks() {
    static thread_local int cache[16] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) dev = 0;
    if (cache[dev] > 0) return cache[dev];
    int cus = 256, per_cu = 4;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_fold_f32_balanced<U, C, NT, SC, ACC, FIN>, kBlock,
                                                     0) != hipSuccess ||
        per_cu < 1)
        per_cu = 4;
    cache[dev] = cus * per_cu;
    return cache[dev];
}

template <int U, int C, bool NT, bool SC, bool ACC, bool FIN>
void launch_balanced(hipStream_t st, const float* X, int64_t N, int64_t P, int64_t ldx, const float* a,
                     const float* s, const float* acc_in, float d, float* out) {
    auto kern = k_fold_f32_balanced<U, C, NT, SC, ACC, FIN>;
    const int64_t nq = P >> 2;
    int64_t grid = resident_blocks<U, C, NT, SC, ACC, FIN>();
    const int64_t tiles = (nq + kBlock - 1) / kBlock;  // never more blocks than 256-quad tiles
    if (grid > tiles) grid = tiles > 0 ? tiles : 1;
    const int64_t per = grid > 0 ? (nq + grid - 1) / grid : 0;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kBlock), 0, st, X, N, P, ldx, a, s, acc_in, d, out, per);
}

template <int U, int C, bool NT, bool SC, bool ACC, bool FIN, bool XR = false, bool NTS = false>
void launch_v4(hipStream_t st, const float* X, int64_t N, int64_t P, int64_t ldx, const float* a,
               const float* s, const float* acc_in, float d, float* out) {
    const int64_t per_block = (int64_t)kBlock * C, units = (P >> 2) + ((P & 3) ? 1 : 0);
    const dim3 grid((unsigned)((units + per_block - 1) / per_block));  // incl. the column-tail lane
    hipLaunchKernelGGL((k_fold_f32_v4<U, C, NT, SC, ACC, FIN, XR, NTS>), grid, dim3(kBlock), 0,
                       st, X, N, P, ldx, a, s, acc_in, d, out);
}

template <int U, int C, bool NT, bool BAL = false, bool XR = false, bool NTS = false>
void launch_v4_flags(hipStream_t st, bool sc, bool acc, bool fin, const float* X, int64_t N, int64_t P,
                     int64_t ldx, const float* a, const float* s, const float* acc_in, float d, float* out) {
#define FA_V4(SC, ACC, FIN)                                                                   \
    do {                                                                                      \
        if constexpr (BAL) launch_balanced<U, C, NT, SC, ACC, FIN>(st, X, N, P, ldx, a, s, acc_in, d, out); \
        else launch_v4<U, C, NT, SC, ACC, FIN, XR, NTS>(st, X, N, P, ldx, a, s, acc_in, d, out); \
    } while (0)
    // tuning variants only: a plain fold with the divide (see launch_gs_flags)
    (void)acc;
    (void)fin;
    if (sc) FA_V4(true, false, true); else FA_V4(false, false, true);
#undef FA_V4
}

int fold_f32_variant(const float* X, int64_t N, int64_t P, int64_t ldx, const float* a, const float* s,
                     float divisor, float* out, void* stream, int variant) {
    if (variant < 0 || variant >= kNumVariants) return fail(FA_ERR_ARG, "unknown variant %d", variant);
    if (variant == 0) return fold_f32_auto(X, N, P, ldx, a, s, nullptr, divisor, 1, out, stream);
    int rc = check_common(N, P, ldx, X, a, out);
    if (rc) return rc;
    if (P == 0) { g_err[0] = 0; return FA_OK; }
    // unaligned layouts take the product's fold, except the any-alignment variants
    if ((variant < kFirstAnyAlign || variant >= kEndAnyAlign) && variant != kPmDw &&
        (!aligned16(X) || (ldx % 4) || !aligned16(out)))
        return fold_f32_auto(X, N, P, ldx, a, s, nullptr, divisor, 1, out, stream);
    hipStream_t st = (hipStream_t)stream;
    const bool sc = s != nullptr, acc = false, fin = true;
    const float* acc_in = nullptr;
#define FA_VF(U, C) launch_v4_flags<U, C, true>(st, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out)
#define FA_VB(U, C) launch_v4_flags<U, C, true, true>(st, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out)
#define FA_VX(U, C) \
    launch_v4_flags<U, C, true, false, true>(st, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out)
#define FA_VS(U, C) \
    launch_v4_flags<U, C, true, false, false, true>(st, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out)
#define FA_VG(K, U, C) launch_gs_flags<U, C, true>(st, K, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out)
#define FA_VGB(K, U, C, B) \
    launch_gs_flags<U, C, true, B>(st, K, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out)
#define FA_VBAND(K, U, C) launch_gs_bands<U, C, true>(st, K, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out)
#define FA_VL(NW, R, TQ, D) \
    launch_lds_flags<NW, R, TQ, D>(st, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out)
    switch (variant) {  // must match kVariants[]
        case 1: FA_VF(8, 4); break;
        case 2: FA_VF(4, 1); break;
        case 3: FA_VX(8, 4); break;
        case 4:  // v4_pickq_nts: the round-1 policy
            switch (pick_quads(P)) {
                case 4: FA_VS(8, 4); break;
                case 2: FA_VS(4, 2); break;
                default: FA_VS(4, 1); break;
            }
            break;
        case 5: FA_VB(4, 4); break;
        case 6: FA_VG(1, 8, 4); break;
        case 7: FA_VG(2, 8, 4); break;
        case 8: FA_VG(1, 4, 8); break;
        case 9: FA_VGB(1, 8, 2, 512); break;
        case 10: FA_VG(-1, 8, 4); break;
        case 11: FA_VG(-1, 8, 2); break;
        case 12: FA_VG(1192, 8, 4); break;
        case 13: FA_VBAND(2, 8, 4); break;
        case 14: FA_VBAND(3, 8, 4); break;
        case 15: FA_VBAND(4, 8, 4); break;
        case 16: FA_VBAND(6, 8, 4); break;
        case 17: rc = FA_VL(8, 64, 32, 1); break;
        case 18: rc = FA_VL(4, 64, 64, 1); break;
        case 19: rc = FA_VL(16, 128, 64, 1); break;
        case 20: rc = FA_VL(4, 32, 16, 2); break;
        case 21: rc = FA_VL(4, 16, 32, 2); break;
        case 22: rc = FA_VL(4, 64, 32, 2); break;
        case 23: rc = FA_VL(8, 32, 32, 2); break;
        case 24: rc = FA_VL(4, 32, 8, 2); break;
        case 25: rc = FA_VL(2, 32, 16, 2); break;
#define FA_VR(NW, R, TQ, S) launch_ring_flags<NW, R, TQ, S>(st, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out)
        case 26: rc = FA_VR(4, 32, 16, 4); break;
        case 27: rc = FA_VR(4, 32, 16, 6); break;
        case 28: rc = FA_VR(4, 32, 16, 8); break;
        case 29: rc = FA_VR(4, 32, 32, 4); break;
        case 30: rc = FA_VR(4, 32, 32, 6); break;
        case 31: rc = FA_VR(4, 64, 16, 4); break;
        case 32: rc = FA_VR(4, 16, 32, 8); break;
        case 33: rc = FA_VR(8, 64, 32, 3); break;
        case 34: rc = FA_VR(4, 32, 8, 8); break;
        case 35: rc = FA_VR(2, 32, 16, 8); break;
#undef FA_VR
        case 36: rc = FA_VL(4, 32, 16, 3); break;
        case 37: rc = FA_VL(4, 32, 16, 4); break;
        case 38: rc = FA_VL(4, 32, 16, 6); break;
        case 39: rc = FA_VL(4, 16, 32, 4); break;
        case 40: rc = FA_VL(4, 16, 32, 3); break;
        case 41: rc = FA_VL(2, 32, 16, 4); break;
        case 42: rc = FA_VL(4, 32, 8, 4); break;
        case 43: rc = FA_VL(8, 32, 32, 3); break;
        case 44: rc = FA_VL(4, 64, 32, 4); break;
        case 45: FA_VGB(8, 16, 1, 64); break;
        case 46: FA_VGB(8, 32, 1, 64); break;
        case 47: FA_VGB(8, 48, 1, 64); break;
        case 48: FA_VGB(8, 32, 1, 128); break;
        case 49: FA_VGB(8, 24, 2, 64); break;
        case 50: rc = FA_VL(4, 32, 24, 2); break;
        case 51: rc = FA_VL(4, 64, 20, 2); break;
        case 52: rc = FA_VL(4, 32, 40, 2); break;
        case 53: rc = FA_VL(2, 16, 32, 2); break;
        case 54: rc = FA_VL(4, 16, 48, 2); break;
        case 55: rc = FA_VL(4, 64, 28, 2); break;
#define FA_VQ(NW, R, TQ, D) \
    launch_lds_flags<NW, R, TQ, D, false, false, false>(st, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out)
        case 56: rc = FA_VQ(4, 32, 16, 4); break;
        case 57: rc = FA_VQ(4, 32, 16, 2); break;
        case 58: rc = FA_VQ(4, 32, 24, 2); break;
        case 59: rc = FA_VQ(4, 16, 32, 2); break;
        case 60: rc = FA_VQ(4, 32, 40, 2); break;
        case 61: rc = FA_VQ(8, 64, 32, 1); break;
#undef FA_VQ
        case 62: rc = FA_VL(4, 16, 16, 4); break;
        case 63: rc = FA_VL(2, 32, 8, 4); break;
        case 64: rc = FA_VL(4, 64, 16, 4); break;
        case 65: rc = FA_VL(4, 64, 16, 6); break;
        case 66: rc = FA_VL(8, 64, 16, 4); break;
        case 67: rc = FA_VL(2, 32, 4, 2); break;
#define FA_VO(NW, R, TQ, D, CF, O) \
    launch_lds_flags<NW, R, TQ, D, false, false, CF, O>(st, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out)
        case 68: rc = FA_VO(4, 32, 16, 4, false, 0); break;
        case 69: rc = FA_VO(4, 32, 24, 2, false, 0); break;
        case 70: rc = FA_VO(4, 16, 32, 2, false, 0); break;
        case 71: rc = FA_VO(4, 32, 40, 2, false, 0); break;
        case 72: rc = FA_VO(4, 32, 16, 4, true, 1); break;
        case 73: rc = FA_VO(4, 32, 24, 2, true, 1); break;
        case 74: rc = FA_VO(4, 16, 32, 2, true, 1); break;
        case 75: rc = FA_VO(4, 32, 40, 2, true, 1); break;
        case 76: rc = FA_VO(4, 32, 16, 4, true, 2); break;
        case 77: rc = FA_VO(4, 32, 24, 2, true, 2); break;
        case 78: rc = FA_VO(4, 16, 32, 2, true, 2); break;
        case 79: rc = FA_VO(4, 32, 40, 2, true, 2); break;
        case 80: rc = FA_VO(4, 32, 16, 4, true, 0); break;
        case 81: rc = FA_VO(4, 32, 24, 2, true, 0); break;
        case 82: rc = FA_VO(4, 16, 32, 2, true, 0); break;
        case 83: rc = FA_VO(4, 32, 40, 2, true, 0); break;
#undef FA_VO
#define FA_VD(NW, R, TQ, D) \
    launch_lds_flags<NW, R, TQ, D, false, false, true, 0, true>(st, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out)
        case 84: rc = FA_VD(2, 32, 16, 4); break;
        case 85: rc = FA_VD(4, 32, 24, 2); break;
        case 86: rc = FA_VD(4, 16, 32, 2); break;
        case 87: rc = FA_VD(4, 32, 40, 2); break;
        case 88: rc = FA_VD(8, 32, 32, 2); break;
        case 89: rc = FA_VD(4, 64, 32, 2); break;
        case 90: rc = FA_VD(8, 32, 32, 3); break;
#undef FA_VD
        case 91:
            if (sc) launch_scalar<true, false, true>(st, X, N, P, ldx, a, s, acc_in, divisor, out);
            else launch_scalar<false, false, true>(st, X, N, P, ldx, a, s, acc_in, divisor, out);
            break;
#define FA_VT(U, C, NTS) launch_tile_flags<U, C, NTS>(st, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out)
        case 92: rc = FA_VT(8, 1, false); break;
        case 93: rc = FA_VT(16, 1, false); break;
        case 94: rc = FA_VT(8, 2, false); break;
        case 95: rc = FA_VT(4, 2, false); break;
        case 96: rc = FA_VT(8, 1, true); break;
        case 97: rc = FA_VT(4, 1, false); break;
#undef FA_VT
#define FA_VE(G, U, C) launch_even_flags<U, C>(st, G, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out)
        case 98: launch_even_auto(st, cu_count(), sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out); break;
        case 99: launch_even_auto(st, 2 * cu_count(), sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out); break;
        case 100: FA_VE(cu_count(), 16, 2); break;
        case 101: FA_VE(cu_count(), 32, 1); break;
        case 102: FA_VE(cu_count(), 8, 4); break;
        case 103: FA_VE(cu_count(), 4, 4); break;
        case 104: FA_VE(2 * cu_count(), 8, 2); break;
        case 105: launch_even_auto(st, 4 * cu_count(), sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out); break;
        case 106: rc = launch_w1<32, 6>(st, sc, X, N, P, ldx, a, s, divisor, out); break;
        case 107: rc = launch_w1<64, 4>(st, sc, X, N, P, ldx, a, s, divisor, out); break;
        case 108: rc = launch_w1<16, 12>(st, sc, X, N, P, ldx, a, s, divisor, out); break;
        case 109: rc = launch_w1<32, 8>(st, sc, X, N, P, ldx, a, s, divisor, out); break;
#undef FA_VE
#define FA_VP(NW, R, TQ, D, DW) \
    launch_lds_flags<NW, R, TQ, D, false, false, true, 8, DW>(st, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out)
        case 110: rc = FA_VP(2, 32, 16, 4, false); break;
        case 111: rc = FA_VP(2, 32, 16, 2, false); break;
        case 112: rc = FA_VP(4, 32, 24, 2, false); break;
        case 113: rc = FA_VP(4, 32, 40, 2, false); break;
        case 114: rc = FA_VP(2, 16, 32, 2, false); break;
        case 115: rc = FA_VP(8, 64, 32, 1, false); break;
        case 116: rc = FA_VP(4, 32, 16, 4, false); break;
        case 117: rc = FA_VP(2, 32, 16, 6, false); break;
        case kPmDw: rc = FA_VP(2, 32, 16, 4, true); break;
        case 119: rc = FA_VP(2, 32, 16, 8, false); break;
        case 120: rc = FA_VP(2, 32, 16, 10, false); break;
        case 121: rc = FA_VP(2, 64, 16, 4, false); break;
        case 122: rc = FA_VP(2, 64, 16, 6, false); break;
#define FA_VP2(NW, R, TQ, D) \
    launch_lds_flags<NW, R, TQ, D, false, false, true, 10>(st, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out)
        case 123: rc = FA_VP2(2, 32, 16, 6); break;
        case 124: rc = FA_VP2(2, 32, 16, 4); break;
        case 125: rc = FA_VP2(4, 32, 16, 4); break;
        case 126: rc = FA_VP2(2, 32, 16, 8); break;
#undef FA_VP2
#undef FA_VP
        default: return fail(FA_ERR_ARG, "unknown variant %d", variant);
    }
#undef FA_VF
#undef FA_VB
#undef FA_VX
#undef FA_VS
#undef FA_VG
#undef FA_VGB
#undef FA_VBAND
#undef FA_VL
    if (rc) return rc;
    return check_launch("fold_f32_variant");
}

}  // namespace

extern "C" {

const char* fa_bench_last_error(void) { return g_err; }
int fa_num_variants(void) { return kNumVariants; }
const char* fa_f32_pick_name(int64_t N, int64_t P, int64_t cus) {
    if (N < 1 || P < 1) return "";
    return f32_pick_name(pick_f32(N, P, cus));
}
int fa_num_f32_forms(void) { return kNumF32Picks; }
const char* fa_f32_form_name(int form) { return (form >= 0 && form < kNumF32Picks) ? f32_pick_name((F32Pick)form) : ""; }
int fa_fedavg_f32_form(const float* X, int64_t N, int64_t P, int64_t ldx, const float* a, const float* s,
                       float divisor, float* out, void* stream, int form) {
    if (form < 0 || form >= kNumF32Picks) return fail(FA_ERR_ARG, "unknown fp32 form %d", form);
    int rc = check_common(N, P, ldx, X, a, out);
    if (rc) return rc;
    if (P == 0) { g_err[0] = 0; return FA_OK; }
    if (!aligned16(X) || (ldx % 4) || !aligned16(out)) return fail(FA_ERR_ARG, "the vector forms need 16-B rows");
    StreamDevice on_stream_device(stream);
    rc = launch_f32_pick((F32Pick)form, (hipStream_t)stream, s != nullptr, false, true, X, N, P, ldx, a, s, nullptr,
                         divisor, out);
    if (rc) return rc;
    return check_launch("fa_fedavg_f32_form");
}
int fa_num_ptrs_forms(void) { return kNumPtrsForms; }
const char* fa_ptrs_form_name(int form) {
    return (form >= 0 && form < kNumPtrsForms) ? ptrs_form_name((PtrsForm)form) : "";
}
int fa_fedavg_f32_ptrs_form(const float* const* xi, int64_t N, int64_t P, const float* a, const float* s,
                            float divisor, float* out, void* stream, int form) {
    if (form < 0 || form >= kNumPtrsForms) return fail(FA_ERR_ARG, "unknown pointer-table form %d", form);
    int rc = check_common(N, P, P, xi, a, out);
    if (rc) return rc;
    if (P == 0) { g_err[0] = 0; return FA_OK; }
    if (!aligned16(out)) return fail(FA_ERR_ARG, "needs a 16-B aligned out");
    StreamDevice on_stream_device(stream);
    rc = launch_ptrs_form((PtrsForm)form, (hipStream_t)stream, xi, N, P, a, s, divisor, out);
    if (rc) return rc;
    return check_launch("fa_fedavg_f32_ptrs_form");
}
int fa_num_step_forms(void) { return kNumStepForms; }
const char* fa_step_form_name(int form) { return step_form_name(form); }

int fa_bench_rounds_create(void** r, int device) {
    if (!r) return fail(FA_ERR_ARG, "null handle");
    *r = nullptr;
    RoundsState* o = new RoundsState();
    const int rc = rounds_state_init(*o, device);
    if (rc) {
        delete o;
        return rc;
    }
    *r = o;
    return FA_OK;
}

int fa_bench_rounds_destroy(void* r) {
    RoundsState* o = static_cast<RoundsState*>(r);
    if (!o) return FA_OK;
    rounds_state_free(*o);
    delete o;
    return FA_OK;
}

int fa_fedavg_rounds_form(void* r, int form, const void* X, int64_t N, int64_t ldx, const float* a, const float* s,
                          float divisor, float* out, uint16_t* out_bf16, int rounds, const int64_t* offsets,
                          void* stream) {
    if (!r) return fail(FA_ERR_ARG, "null rounds state");
    if (form < 0 || form >= kNumStepForms) return fail(FA_ERR_ARG, "unknown step form %d", form);
    StreamDevice on_stream_device(stream);
    return launch_step(*static_cast<RoundsState*>(r), form, (hipStream_t)stream, X, N, ldx, a, s, divisor, out,
                       kStepSpecs[form].bf16 ? out_bf16 : nullptr, rounds, offsets);
}

int fa_bench_rounds_wait(void* r, int round, void* stream) {
    RoundsState* o = static_cast<RoundsState*>(r);
    if (!o) return fail(FA_ERR_ARG, "null rounds state");
    StreamDevice on_stream_device(stream);
    return rounds_wait(*o, round, (hipStream_t)stream);
}

int fa_bench_rounds_set_sys(void* r, int sys) {
    RoundsState* o = static_cast<RoundsState*>(r);
    if (!o) return fail(FA_ERR_ARG, "null rounds state");
    if (sys < 0 || sys > 2) return fail(FA_ERR_ARG, "sys must be 0, 1 or 2");
    o->sys = sys;
    return FA_OK;
}

int fa_num_bf16_forms(void) { return kNumBf16Forms; }
const char* fa_bf16_form_name(int form) {
    return (form >= 0 && form < kNumBf16Forms) ? bf16_form_name((Bf16Form)form) : "";
}
int fa_fedavg_bf16_form(const uint16_t* X, int64_t N, int64_t P, int64_t ldx, const float* a, const float* s,
                        float divisor, float* out_f32, uint16_t* out_bf16, void* stream, int form) {
    if (form < 0 || form >= kNumBf16Forms) return fail(FA_ERR_ARG, "unknown bf16 form %d", form);
    int rc = check_common(N, P, ldx, X, a, bf16_any_out(out_f32, out_bf16));
    if (rc) return rc;
    if (P == 0) { g_err[0] = 0; return FA_OK; }
    if (!aligned16(X) || (ldx % 8) || !aligned16(out_f32) || (out_bf16 && !aligned16(out_bf16)))
        return fail(FA_ERR_ARG, "the vector forms need 16-B rows");
    StreamDevice on_stream_device(stream);
    launch_bf16_form((Bf16Form)form, (hipStream_t)stream, X, N, P, ldx, a, s, divisor, out_f32, out_bf16);
    return check_launch("fa_fedavg_bf16_form");
}
const char* fa_variant_name(int variant) {
    return (variant >= 0 && variant < kNumVariants) ? kVariants[variant] : "";
}

int fa_fedavg_f32_variant(const float* X, int64_t N, int64_t P, int64_t ldx, const float* a,
                          const float* s, float divisor, float* out, void* stream, int variant) {
    return fold_f32_variant(X, N, P, ldx, a, s, divisor, out, stream, variant);
}

int fa_fedavg_bf16_variant(const uint16_t* X, int64_t N, int64_t P, int64_t ldx, const float* a,
                           const float* s, float divisor, float* out_f32, uint16_t* out_bf16, void* stream,
                           int variant) {
    if (variant < 0 || variant >= kNumBf16Variants) return fail(FA_ERR_ARG, "unknown bf16 variant %d", variant);
    if (variant == 0) return bf16_auto(X, N, P, ldx, a, s, divisor, out_f32, out_bf16, stream);
    int rc = check_common(N, P, ldx, X, a, bf16_any_out(out_f32, out_bf16));
    if (rc) return rc;
    if (P == 0) { g_err[0] = 0; return FA_OK; }
    if (!aligned16(X) || (ldx % 8) || !aligned16(out_f32) || (out_bf16 && !aligned16(out_bf16)))
        return bf16_auto(X, N, P, ldx, a, s, divisor, out_f32, out_bf16, stream);
    hipStream_t st = (hipStream_t)stream;
#define FA_BF(U, C)                                                                                         \
    {                                                                                                       \
        const int64_t per_block = (int64_t)kBlock * (C), units = (P >> 3) + ((P & 7) ? 1 : 0);            \
        const dim3 grid((unsigned)((units + per_block - 1) / per_block));                                   \
        if (s)                                                                                              \
            hipLaunchKernelGGL((k_fedavg_bf16_v8<U, C, true>), grid, dim3(kBlock), 0, st, X, N, P, ldx, a, s, \
                               divisor, out_f32, out_bf16);                                                 \
        else                                                                                                \
            hipLaunchKernelGGL((k_fedavg_bf16_v8<U, C, false>), grid, dim3(kBlock), 0, st, X, N, P, ldx, a,  \
                               s, divisor, out_f32, out_bf16);                                              \
    }
    switch (variant) {  // must match kBf16Variants[]
        case 1: FA_BF(8, 1); break;
        case 2: FA_BF(8, 2); break;
        case 3: FA_BF(2, 8); break;
        case 4: launch_bf16_gs<8, 2>(st, 1, X, N, P, ldx, a, s, divisor, out_f32, out_bf16); break;
        case 5: launch_bf16_gs<8, 4>(st, 1, X, N, P, ldx, a, s, divisor, out_f32, out_bf16); break;
        case 6: launch_bf16_gs<8, 2>(st, -1, X, N, P, ldx, a, s, divisor, out_f32, out_bf16); break;
        case 7: launch_bf16_gs<2, 8>(st, -1, X, N, P, ldx, a, s, divisor, out_f32, out_bf16); break;
        case 8: launch_bf16_bands<2, 8>(st, 2, X, N, P, ldx, a, s, divisor, out_f32, out_bf16); break;
        case 9: launch_bf16_bands<2, 8>(st, 4, X, N, P, ldx, a, s, divisor, out_f32, out_bf16); break;
        case 10: launch_bf16_bands<8, 2>(st, 4, X, N, P, ldx, a, s, divisor, out_f32, out_bf16); break;
        case 11: launch_bf16_bands<16, 2>(st, 4, X, N, P, ldx, a, s, divisor, out_f32, out_bf16); break;
        case 12: launch_bf16_bands<8, 4>(st, 4, X, N, P, ldx, a, s, divisor, out_f32, out_bf16); break;
        case 13: launch_bf16_bands<4, 4>(st, 4, X, N, P, ldx, a, s, divisor, out_f32, out_bf16); break;
        case 14: launch_bf16_bands<8, 2>(st, 3, X, N, P, ldx, a, s, divisor, out_f32, out_bf16); break;
        default: launch_bf16_bands<16, 1>(st, 4, X, N, P, ldx, a, s, divisor, out_f32, out_bf16); break;
    }
#undef FA_BF
    return check_launch("fedavg_bf16_variant");
}

// LDS-staged pointer-table fold (fa_fedavg_f32_ptrs_aligned's narrow picks)
// with an explicit tile and loader: ptrs_o<LOPT>[q]_t<TQ> (see k_fold_f32_lds).
int fa_fedavg_f32_ptrs_variant(const float* const* xi, int64_t N, int64_t P, const float* a, const float* s,
                               float divisor, float* out, void* stream, int variant) {
    int rc = check_common(N, P, P, xi, a, out);
    if (rc) return rc;
    if (P == 0) { g_err[0] = 0; return FA_OK; }
    if ((variant < 14 || variant >= 20) && !aligned16(out)) return fail(FA_ERR_ARG, "needs a 16-B aligned out");
    hipStream_t st = (hipStream_t)stream;
    const float* X = (const float*)xi;
    const bool sc = s != nullptr;
#define FA_PV(R, TQ, D, CF, O) \
    launch_lds_flags<4, R, TQ, D, false, true, CF, O>(st, sc, false, true, X, N, P, P, a, s, nullptr, divisor, out)
#define FA_PW(NW, R, TQ, D, O) \
    launch_lds_flags<NW, R, TQ, D, false, true, true, O>(st, sc, false, true, X, N, P, P, a, s, nullptr, divisor, out)
    switch (variant) {  // must match kPtrsVariants[]
        case 0: rc = FA_PV(32, 16, 2, true, 0); break;
        case 1: rc = FA_PV(32, 16, 2, true, 4); break;
        case 2: rc = FA_PV(32, 24, 2, true, 0); break;
        case 3: rc = FA_PV(32, 24, 2, true, 4); break;
        case 4: rc = FA_PV(16, 32, 2, true, 0); break;
        case 5: rc = FA_PV(16, 32, 2, true, 4); break;
        case 6: rc = FA_PV(32, 40, 2, true, 0); break;
        case 7: rc = FA_PV(32, 40, 2, true, 4); break;
        case 8: rc = FA_PV(32, 24, 2, false, 0); break;
        case 9: rc = FA_PV(32, 16, 4, true, 4); break;
        case 10: rc = FA_PV(32, 16, 4, true, 0); break;
        case 11: rc = FA_PW(2, 32, 16, 4, 0); break;
        case 12: rc = FA_PW(2, 32, 16, 4, 4); break;
        case 13: rc = FA_PW(8, 64, 32, 1, 0); break;
#define FA_PD(NW, R, TQ, D, O) \
    launch_lds_flags<NW, R, TQ, D, false, true, true, O, true>(st, sc, false, true, X, N, P, P, a, s, nullptr, divisor, \
                                                              out)
        case 14: rc = FA_PD(2, 32, 16, 4, 4); break;
        case 15: rc = FA_PD(4, 32, 40, 2, 0); break;
        case 16: rc = FA_PD(4, 16, 32, 2, 0); break;
        case 17: rc = FA_PD(4, 32, 24, 2, 0); break;
#undef FA_PD
        case 18:
            if (sc) hipLaunchKernelGGL(k_fold_f32_rows_scalar<true>, grid_for(P), dim3(kBlock), 0, st, xi, N, P, a, s,
                                       divisor, out);
            else hipLaunchKernelGGL(k_fold_f32_rows_scalar<false>, grid_for(P), dim3(kBlock), 0, st, xi, N, P, a, s,
                                    divisor, out);
            break;
        case 19:
            if (sc) hipLaunchKernelGGL((k_fedavg_f32_ptrs<8, true>), grid_for((P + 3) / 4), dim3(kBlock), 0, st, xi, N,
                                       P, a, s, divisor, out);
            else hipLaunchKernelGGL((k_fedavg_f32_ptrs<8, false>), grid_for((P + 3) / 4), dim3(kBlock), 0, st, xi,
                                    N, P, a, s, divisor, out);
            break;
        case 20: rc = FA_PW(2, 16, 32, 2, 0); break;
        case 21: rc = FA_PW(2, 16, 32, 2, 4); break;
        case 22: rc = FA_PW(2, 32, 16, 2, 0); break;
        case 23: rc = FA_PW(2, 32, 16, 2, 4); break;
        case 24: rc = FA_PW(2, 32, 16, 4, 12); break;
        case 25: rc = FA_PW(2, 32, 16, 6, 12); break;
        case 26: rc = FA_PW(2, 32, 16, 6, 8); break;
        case 27: rc = FA_PW(2, 32, 16, 4, 8); break;
        case 28: rc = FA_PW(2, 32, 16, 6, 14); break;
        case 29: rc = FA_PW(2, 32, 16, 4, 6); break;
        case 30: rc = FA_PW(2, 32, 16, 4, 14); break;
        default: return fail(FA_ERR_ARG, "unknown pointer variant %d", variant);
    }
#undef FA_PV
#undef FA_PW
    if (rc) return rc;
    return check_launch("fa_fedavg_f32_ptrs_variant");
}
int fa_num_ptrs_variants(void) { return kNumPtrsVariants; }
const char* fa_ptrs_variant_name(int variant) {
    return (variant >= 0 && variant < kNumPtrsVariants) ? kPtrsVariants[variant] : "";
}

int fa_num_bf16_variants(void) { return kNumBf16Variants; }
const char* fa_bf16_variant_name(int variant) {
    return (variant >= 0 && variant < kNumBf16Variants) ? kBf16Variants[variant] : "";
}

int fa_synth_f32(float* X, int64_t nrows, int64_t ncols, int64_t ldx, uint64_t seed, int64_t row0,
                 int64_t col0, void* stream) {
    if (nrows < 0 || ncols < 0 || ldx < ncols) return fail(FA_ERR_ARG, "bad synth shape");
    if (nrows == 0 || ncols == 0) { g_err[0] = 0; return FA_OK; }
    if (!X) return fail(FA_ERR_ARG, "null X");
    hipLaunchKernelGGL(k_synth<float>, dim3(8192), dim3(kBlock), 0, (hipStream_t)stream, X, nrows, ncols, ldx,
                       seed, row0, col0);
    return check_launch("k_synth<f32>");
}

int fa_synth_bf16(uint16_t* X, int64_t nrows, int64_t ncols, int64_t ldx, uint64_t seed, int64_t row0,
                  int64_t col0, void* stream) {
    if (nrows < 0 || ncols < 0 || ldx < ncols) return fail(FA_ERR_ARG, "bad synth shape");
    if (nrows == 0 || ncols == 0) { g_err[0] = 0; return FA_OK; }
    if (!X) return fail(FA_ERR_ARG, "null X");
    hipLaunchKernelGGL(k_synth<uint16_t>, dim3(8192), dim3(kBlock), 0, (hipStream_t)stream, X, nrows, ncols,
                       ldx, seed, row0, col0);
    return check_launch("k_synth<bf16>");
}

int fa_bench_copy_f32(float* dst, const float* src, int64_t n, int blocks, void* stream) {
    if (n < 0 || blocks < 1 || (n > 0 && (!dst || !src)) || !aligned16(dst) || !aligned16(src) || (n & 3))
        return fail(FA_ERR_ARG, "bench copy needs 16-B aligned buffers, n %% 4 == 0, blocks >= 1");
    if (n == 0) { g_err[0] = 0; return FA_OK; }
    hipLaunchKernelGGL(k_bench_copy, dim3((unsigned)blocks), dim3(kBlock), 0, (hipStream_t)stream,
                       reinterpret_cast<f32x4*>(dst), reinterpret_cast<const f32x4*>(src), n >> 2);
    return check_launch("k_bench_copy");
}

int fa_bench_stream_cu_mask(int device, const uint32_t* mask, int words, void** stream) {
    if (!mask || words < 1 || !stream) return fail(FA_ERR_ARG, "bad CU mask arguments");
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess) {
        (void)hipGetLastError();
        return fail(FA_ERR_HIP, "cannot select device %d", device);
    }
    hipStream_t st = nullptr;
    const hipError_t e = hipExtStreamCreateWithCUMask(&st, (uint32_t)words, mask);
    (void)hipSetDevice(prev);
    if (e != hipSuccess) return fail(FA_ERR_HIP, "hipExtStreamCreateWithCUMask: %s", hipGetErrorString(e));
    *stream = st;
    g_err[0] = 0;
    return FA_OK;
}
int fa_bench_stream_destroy(void* stream) {
    if (stream && hipStreamDestroy((hipStream_t)stream) != hipSuccess) return fail(FA_ERR_HIP, "hipStreamDestroy");
    return FA_OK;
}

int fa_read_sweep_f32(const float* X, int64_t n, float* sink, int64_t sink_len, void* stream) {
    if (n < 0 || !X || !sink || sink_len <= 0 || !aligned16(X) || (n & 3))
        return fail(FA_ERR_ARG, "read sweep needs 16-B aligned X, n %% 4 == 0, sink_len > 0");
    const int64_t nq = n >> 2, grid = (nq + kSweepQuads - 1) / kSweepQuads;
    if (grid > 0x7FFFFFFF) return fail(FA_ERR_ARG, "read sweep too large");
    if (grid == 0) { g_err[0] = 0; return FA_OK; }
    hipLaunchKernelGGL(k_read_sweep, dim3((unsigned)grid), dim3(kBlock), 0, (hipStream_t)stream,
                       reinterpret_cast<const f32x4*>(X), nq, sink, sink_len);
    return check_launch("k_read_sweep");
}

}  // extern "C"
