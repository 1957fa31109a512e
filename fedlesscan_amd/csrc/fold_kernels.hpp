// fold_kernels.hpp — device code shared by libfedavg_hip.so (the product,
// fedavg.hip) and libfedavg_hip_bench.so (kernel variants, input generator and
// read-sweep calibration for bench.py / the sweeps, fedavg_bench.hip).
//
// Hot path replaced (reference, all numpy on one CPU core):
//   fedless/aggregator/fed_avg_aggregator.py:24-42        FedAvgAggregator._aggregate
//   fedless/aggregator/stall_aware_aggregation.py:42-67   StallAwareAggregator._aggregate
//
// The op is a bandwidth-bound weighted column reduction over a row-stacked
// [N clients][ldx] matrix: 2-3 FLOP per 4-byte element, far below any MFMA
// ridge, so it runs on the VALU and the design goal is HBM read bandwidth.
//
// Bit-exactness contract: every output column is owned by
// ONE lane, which folds clients 0..N-1 strictly in order with a separate
// multiply and add (no FMA: these TUs are compiled with fp-contract off) and
// finishes with an IEEE divide.  No split-N, tree or atomic reassociation on
// any default path (the opt-in fa_fedavg_f32_splitn is the one exception).
//
// Parallelism comes from the columns: lane = 4 consecutive fp32 columns
// (one 16-byte global_load_dwordx4 per client row).  Memory-level
// parallelism comes from U independent client-row loads in flight ahead of
// the in-order adds (the loads are independent, only the adds are ordered).
// Kernel families (fold_f32_auto picks one by shape, pick_f32):
//   k_fold_f32_gs    grid-stride over 16 KiB column tiles, ~1 block per CU,
//                    balanced passes, launched per column band (large models)
//   k_fold_f32_tile  one block per tile, same tile body (few clients)
//   k_fold_f32_lds   LDS-staged: all waves stream client-row chunks of a
//                    narrow column tile into LDS, then every wave folds its
//                    share of the tile's columns from LDS (narrow models)
// Everything here sits in an anonymous namespace: each library gets its own
// copy, and templates are instantiated only where a TU launches them.
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "fedavg_hip.h"
#include "tuner.hpp"

#pragma clang fp contract(off)

namespace {

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(FA_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
    g_err[0] = 0;
    return FA_OK;
}

constexpr int kBlock = 256;

typedef float f32x4 __attribute__((ext_vector_type(4)));
// f32x4 in the global address space: loads through pointers read from memory
// (row tables) are global_load, not flat_load
typedef __attribute__((address_space(1))) const f32x4 gf32x4;
typedef __attribute__((address_space(1))) const float gf32;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__host__ __device__ inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
// [a, a + na) and [b, b + nb) share a byte
inline bool overlaps(const void* a, size_t na, const void* b, size_t nb) {
    const uintptr_t x = reinterpret_cast<uintptr_t>(a), y = reinterpret_cast<uintptr_t>(b);
    return x < y + nb && y < x + na;
}

// ---------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------
template <bool NT>
__device__ __forceinline__ f32x4 ld4(const f32x4* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

__device__ __forceinline__ f32x4 scale4(f32x4 x, float a) { return x * a; }
__device__ __forceinline__ f32x4 add4(f32x4 x, f32x4 y) { return x + y; }
__device__ __forceinline__ f32x4 div4(f32x4 x, float d) { return x / d; }

// t_i = fl(fl(x*a) * s): two roundings, left-to-right like `layer * n * s`.
template <bool SCORED>
__device__ __forceinline__ f32x4 term4(f32x4 x, float a, float s) {
    f32x4 t = scale4(x, a);
    if constexpr (SCORED) t = scale4(t, s);
    return t;
}
template <bool SCORED>
__device__ __forceinline__ float term1(float x, float a, float s) {
    float t = x * a;
    if constexpr (SCORED) t = t * s;
    return t;
}

// ---------------------------------------------------------------------------
// Write-through (sc1) 16-byte stores for the one-launch step (round 5): the
// line goes to memory, not only the XCD's L2, so a block that publishes a
// round needs no L2 write-back (an agent release fence per block and round
// cost the C4 rank step 3.5 %, tools/step_probe.hip).  A raw buffer store
// over a wave-uniform base (the tile's first octet: readfirstlane of a value
// every lane shares) with a small per-lane offset; cache-policy operand 16 =
// sc1 on gfx950.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wt_rsrc(const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, -1, 0x00020000);
}
__device__ __forceinline__ int64_t uniform64(int64_t v) {
    const uint64_t u = (uint64_t)v;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u), hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
// WT (the tile functions' template argument): 0 plain stores; kWtAgent sc1
// (write-through to memory: the one-launch step on this GPU); kWtSystem sc0
// sc1 (system-coherent: a peer exchange's step, whose rounds other GPUs' copy
// engines read).  Cache-policy operand: sc0 = 1, sc1 = 16 on gfx950.
constexpr int kWtAgent = 1, kWtSystem = 2;
template <int WT>
__device__ __forceinline__ void st16_wt(__amdgpu_buffer_rsrc_t r, int byte_off, u32x4 v) {
    static_assert(WT == kWtAgent || WT == kWtSystem, "write-through flavour");
    __builtin_amdgcn_raw_buffer_store_b128(v, r, byte_off, 0, WT == kWtSystem ? 17 : 16);
}
// After a tile's few plain tail stores: write them back before the block
// publishes (the wide stores are write-through already).
template <int WT>
__device__ __forceinline__ void wt_tail_release() {
    if constexpr (WT == kWtSystem) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    else if constexpr (WT == kWtAgent) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
}

// fp32 fold over a stacked matrix, 16 B per lane per client row.
//   X viewed as [N][ldq] f32x4 (ldq = ldx/4), 16-byte aligned rows.
//   A lane owns C quads spaced kBlock apart (a block covers C*kBlock quads =
//   C*4 KiB of every client row); nq = P/4 full quads, and the trailing P%4
//   columns are folded by the lane whose first quad index == nq.
// Template: U = client rows loaded ahead of the ordered adds; C = quads per
// lane; NT = non-temporal (read-once) loads; SCORED = stall-aware second
// multiply; ACC = continue a fold from acc_in; FIN = divide at the end.
// ---------------------------------------------------------------------------
template <int U, int C, bool NT, bool SCORED, bool ACC, bool FIN, bool NTS = false, int B = kBlock, int WT = 0>
__device__ __forceinline__ void fold_quads(const f32x4* __restrict__ p, int64_t ldq, int64_t N,
                                           const float* __restrict__ a, const float* __restrict__ s,
                                           const f32x4* acc_in, float divisor, f32x4* out) {
    f32x4 acc[C];
    int64_t i = 0;
    if constexpr (ACC) {
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] = acc_in[c * B];
    } else {
        const float a0 = a[0], s0 = SCORED ? s[0] : 1.0f;
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] = term4<SCORED>(ld4<NT>(p + c * B), a0, s0);
        i = 1;
    }
    for (; i + U <= N; i += U) {
        f32x4 v[U][C];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int c = 0; c < C; ++c) v[u][c] = ld4<NT>(p + (i + u) * ldq + c * B);
        // deep unrolls (one-wave blocks): keep every load of the group issued
        // before the first add (the scheduler would otherwise sink them)
        if constexpr (U >= 16) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float ai = a[i + u], si = SCORED ? s[i + u] : 1.0f;
#pragma unroll
            for (int c = 0; c < C; ++c) acc[c] = add4(acc[c], term4<SCORED>(v[u][c], ai, si));
        }
    }
    for (; i < N; ++i) {
        const float ai = a[i], si = SCORED ? s[i] : 1.0f;
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] = add4(acc[c], term4<SCORED>(ld4<NT>(p + i * ldq + c * B), ai, si));
    }
    if constexpr (WT) {  // write-through over the lane's tile base (out - threadIdx.x, shared by every lane)
        const __amdgpu_buffer_rsrc_t rs = wt_rsrc(reinterpret_cast<const void*>(
            (uintptr_t)uniform64((int64_t)(uintptr_t)(out - threadIdx.x))));
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const f32x4 r = FIN ? div4(acc[c], divisor) : acc[c];
            st16_wt<WT>(rs, (int)(16 * ((int)threadIdx.x + c * B)), __builtin_bit_cast(u32x4, r));
        }
        return;
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const f32x4 r = FIN ? div4(acc[c], divisor) : acc[c];
        if constexpr (NTS) __builtin_nontemporal_store(r, out + c * B);
        else out[c * B] = r;
    }
}
// One tile: C*kBlock quads of every client row (tile index bid).
template <int U, int C, bool NT, bool SCORED, bool ACC, bool FIN, bool NTS, int B = kBlock, int WT = 0>
__device__ __forceinline__ void fold_tile(int64_t bid, const float* __restrict__ X, int64_t N, int64_t P,
                                          int64_t ldx, const float* __restrict__ a, const float* __restrict__ s,
                                          const float* acc_in, float divisor, float* out) {
    const int64_t nq = P >> 2;
    const int64_t ldq = ldx >> 2;
    const int64_t q0 = bid * (B * C) + threadIdx.x;
    const f32x4* X4 = reinterpret_cast<const f32x4*>(X);
    const f32x4* A4 = reinterpret_cast<const f32x4*>(acc_in);
    f32x4* O4 = reinterpret_cast<f32x4*>(out);
    if (q0 + (int64_t)(C - 1) * B < nq) {
        // every quad of this lane is in range (all blocks but the last)
        fold_quads<U, C, NT, SCORED, ACC, FIN, NTS, B, WT>(X4 + q0, ldq, N, a, s, ACC ? A4 + q0 : nullptr, divisor,
                                                        O4 + q0);
        return;
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int64_t q = q0 + (int64_t)c * B;
        if (q < nq)
            fold_quads<U, 1, NT, SCORED, ACC, FIN, false, B, WT>(X4 + q, ldq, N, a, s, ACC ? A4 + q : nullptr, divisor,
                                                             O4 + q);
    }
    // column tail: at most 3 columns, folded by the lane that would own quad
    // index nq under the C-quads-per-lane mapping (scalar loads, same order)
    const int64_t tb = nq / (B * C), tl = (nq % (B * C)) % B;
    if ((P & 3) && bid == tb && (int64_t)threadIdx.x == tl) {
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
        // WT: these few plain stores are written back before the block publishes
        wt_tail_release<WT>();
    }
}

// Grid-stride form: a small grid (about one block per CU) walks the tiles in
// order, tile = blockIdx.x + k*gridDim.x, so at any moment the running blocks
// stream ADJACENT column tiles of the same client rows (one contiguous band,
// rows visited in near lock-step) and each block streams many rows per tile.
// On MI355X this reads HBM faster than one block per tile with several
// resident per CU.
template <int U, int C, bool NT, bool SCORED, bool ACC, bool FIN, bool NTS, int B = kBlock>
__global__ __launch_bounds__(B) void k_fold_f32_gs(
    const float* __restrict__ X, int64_t N, int64_t P, int64_t ldx,
    const float* __restrict__ a, const float* __restrict__ s,
    const float* acc_in, float divisor, float* out, int64_t ntiles) {  // acc_in may alias out
    for (int64_t bid = blockIdx.x; bid < ntiles; bid += gridDim.x)
        fold_tile<U, C, NT, SCORED, ACC, FIN, NTS, B>(bid, X, N, P, ldx, a, s, acc_in, divisor, out);
}

// One block per tile (few clients: more blocks in flight than the grid-stride
// form, each with a short row run).
template <int U, int C, bool NT, bool SCORED, bool ACC, bool FIN, bool NTS>
__global__ __launch_bounds__(kBlock) void k_fold_f32_tile(
    const float* __restrict__ X, int64_t N, int64_t P, int64_t ldx,
    const float* __restrict__ a, const float* __restrict__ s,
    const float* acc_in, float divisor, float* out) {  // acc_in may alias out
    fold_tile<U, C, NT, SCORED, ACC, FIN, NTS>(blockIdx.x, X, N, P, ldx, a, s, acc_in, divisor, out);
}

// Narrow models: LDS-staged client rows.
//   When P is small (a few hundred thousand parameters: the MNIST CNN, the
//   speech CNN, a 1M-param bucket), one lane per quad gives too few lanes to
//   keep enough bytes in flight on 256 CUs.  Here a block owns only TQ quads
//   (TQ*16 B of every client row) and ALL its NW waves load: each chunk of R
//   client rows is read with R*TQ/(NW*64) independent 16-byte loads per lane
//   and parked in LDS; wave 0 then folds the chunk from LDS in client order
//   (lane = one quad) while the next chunk's loads are already in flight.  The
//   adds stay one lane per column, strictly in row order: bit-identical to
//   every other fold.  Per-chunk factors a[], s[] are staged in LDS too.
//
//   Every block that owns full quads runs the pipelined loop, the last one
//   too: its quad indices past the end are clamped to the last full quad (a
//   valid address; the value is never stored), so no load carries a branch.
//   (A checked, unpipelined last block used to be the straggler of the whole
//   launch: one dependent HBM round trip per chunk, 64 of them at N = 1024.)
//   The P%4 tail columns get one extra block of their own: every thread
//   loads one row's tail elements and forms its term (elementwise, as in the
//   fold), NT rows in flight per pass, and thread 0 adds the pass in row order.
//
//   ROWS: X is really `const float* const* xi`, a device table of N row
//   pointers (separately allocated client rows, every row 16-B aligned;
//   fa_fedavg_f32_ptrs_aligned); ldx is unused.
//
//   COLF (the default): the staged chunk is folded by ALL waves, one column per
//   lane: wave w owns columns [w*CPW, (w+1)*CPW) of the block's TQ*4, CPW =
//   TQ*4/NW.  Per row a lane issues one 4-byte LDS read, a multiply and an add,
//   and the NW waves fold side by side on their own SIMDs.  The quad fold
//   (COLF = false, wave 0 alone, lane = quad: two packed multiplies and two
//   packed adds per row with TQ of 64 lanes active) kept the other waves at the
//   barrier for most of each chunk when a CU holds only one block (1024 x 16K:
//   ~0.5 us of fold per 8 KB chunk).  Per column the arithmetic is the same.
//
//   DW: 4-byte loads (lane = one float of a row segment) instead of 16-byte
//   quads, for rows that are not 16-B aligned (a row pitch that is not a
//   multiple of 4 floats: a torch.stack of an odd-sized model, or separately
//   allocated rows at any 4-B offset).  Consecutive lanes still read
//   consecutive floats of one row, so every wave-load is one contiguous
//   256-byte run; the tile in LDS and the fold are the same.
template <int NW, int R, int TQ, bool SCORED, bool ACC, bool FIN, int DEPTH = 1, bool ROWS = false,
          bool COLF = true, int LOPT = 0, bool DW = false>
__global__ __launch_bounds__(NW * 64) void k_fold_f32_lds(
    const float* __restrict__ X, int64_t N, int64_t P, int64_t ldx,
    const float* __restrict__ a, const float* __restrict__ s,
    const float* acc_in, float divisor, float* out) {  // acc_in may alias out
    constexpr int NT = NW * 64;
    constexpr int LQ = R * TQ / NT;  // quads each thread loads per chunk
    static_assert(TQ <= 64 && (R * TQ) % NT == 0 && R <= NT, "tile shape");
    __shared__ f32x4 tile[R * TQ];
    __shared__ float fa[R], fs[SCORED ? R : 1];
    const int64_t nq = P >> 2;                     // full quads
    const int64_t nbq = (nq + TQ - 1) / TQ;        // blocks over the full quads
    const int t = threadIdx.x;
    const int64_t ldq = ldx >> 2;
    const float* const* __restrict__ xi = reinterpret_cast<const float* const*>(X);
    auto rowf = [&](int64_t row) -> const float* {
        if constexpr (ROWS) return xi[row];
        else return X + row * ldx;
    };

    if ((int64_t)blockIdx.x >= nbq) {
        // ---- the P%4 tail columns (block-uniform branch: this block only) ----
        const int w4 = (int)(P & 3);
        const int64_t col0 = nq * 4;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        if (ACC && t == 0)
            for (int k = 0; k < w4; ++k) acc[k] = acc_in[col0 + k];
        for (int64_t r0 = 0; r0 < N; r0 += NT) {
            const int64_t row = r0 + t;
            if (row < N) {
                const float* rp = rowf(row);
                f32x4 x = {0.f, 0.f, 0.f, 0.f};
                for (int k = 0; k < w4; ++k) x[k] = rp[col0 + k];
                tile[t] = term4<SCORED>(x, a[row], SCORED ? s[row] : 1.0f);
            }
            __syncthreads();
            if (t == 0) {
                const int rows = (N - r0) < NT ? (int)(N - r0) : NT;
                int i = 0;
                if (!ACC && r0 == 0) {
                    acc = tile[0];
                    i = 1;
                }
                for (; i + 8 <= rows; i += 8) {
                    f32x4 v[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) v[k] = tile[i + k];
#pragma unroll
                    for (int k = 0; k < 8; ++k) acc = add4(acc, v[k]);
                }
                for (; i < rows; ++i) acc = add4(acc, tile[i]);
            }
            __syncthreads();
        }
        if (t == 0) {
            const f32x4 res = FIN ? div4(acc, divisor) : acc;
            for (int k = 0; k < w4; ++k) out[col0 + k] = res[k];
        }
        return;
    }

    // ---- full quads [q0, q0 + tq) ----
    const int64_t q0 = (int64_t)blockIdx.x * TQ;
    const int tq = (int)((nq - q0) < TQ ? (nq - q0) : TQ);
    // this lane's quad within the tile for its j-th load, clamped to the last
    // full quad (the last block's lanes past the end re-read a valid quad)
    auto qof = [&](int j) -> int64_t {
        const int64_t q = q0 + (t + j * NT) % TQ;
        return q < nq ? q : nq - 1;
    };
    // one chunk in registers: its LQ quads per lane and (lanes < R) its
    // factors; ROWS with the pointer ring: also the row pointers of the chunk
    // this stage loads next
    constexpr bool PRING = ROWS && (LOPT & 4);
    constexpr bool PRE = (LOPT & 8) != 0;
    static_assert(!PRE || COLF, "premultiplied stash: column fold only");
    constexpr int LU = DW ? 4 * LQ : LQ;  // loads per thread per chunk
    constexpr int RW = DW ? 4 * TQ : TQ;  // load units per row of the tile
    struct Stage {
        f32x4 v[DW ? 1 : LQ];
        float vf[DW ? LU : 1];
        float fv, sv;
        const float* p[PRING ? LU : 1];
        float pa[PRE ? LU : 1], ps[PRE && SCORED ? LU : 1];  // PRE: the factors of each load's row
    };
    // DW: this lane's float of the tile for its j-th load, clamped to the last
    // column of the full quads
    auto fof = [&](int j) -> int64_t {
        const int64_t col = q0 * 4 + (t + j * NT) % RW;
        return col < nq * 4 ? col : nq * 4 - 1;
    };
    Stage st[DEPTH > 1 ? DEPTH : 1];
    const int64_t nfull = N / R;  // chunks taken by the pipelined loop
    // ROWS: each lane reads its own rows' pointers from the table (8 B, a
    // cache-resident line shared by the lanes of a row), with vector loads: a
    // scalar load would share lgkmcnt with the fold's LDS reads and, returning
    // out of order, force the fold to wait for it.  Two schedules:
    //   next-chunk (LOPT bit 2 clear): the pointers of chunk c+1 are fetched
    //     right behind chunk c's data loads; issuing chunk c+1 then waits for
    //     them, and so (waits count loads in issue order) for chunk c's data;
    //   pointer ring (bit 2 set): chunk c always goes through stage c % DEPTH,
    //     which right after its data fetches the pointers of chunk c + dist
    //     (dist = stages in flight), the next chunk it loads; that wait falls
    //     after chunk c has been stashed anyway.
    // Loader options (LOPT, measured with the tuning variants o<LOPT>_*):
    //   bit 0: every lane loads a factor (lanes >= R a duplicate) instead of
    //     `if (t < R)`.  Whole waves skip the guarded load, so the compiler
    //     cannot count a stage's loads and waits for more than the oldest
    //     stage before a stash (down to vmcnt(0)): the guarded form keeps
    //     fewer bytes in flight per block;
    //   bit 1: a scheduling barrier after each stage's loads, so the
    //     prologue's factor loads are not sunk behind later stages' data (the
    //     loop-carried wait counts would merge to the worst case).
    //   Bits 0+1 give exact waits (all DEPTH stages in flight) -- and ran
    //   SLOWER where several blocks share a CU: 1024 x 67K, 24-quad tiles,
    //   bit 0 alone 47.3 us against 45.0 with neither (the same sweep,
    //   profiles/r02_lds/loader_ab_sweep.log); both bits were slower still in
    //   a first run of it.  The shallower effective pipeline of the guarded
    //   loader is the better one there.  The product uses LOPT 0, and 4 (the
    //   pointer ring) only for the pointer-table form of the narrowest pick,
    //   one block per CU (1024 x 16K rows: 20.3 against 26.1 us; 1024 x 67K,
    //   24-quad tiles: 57.3 against 53.8 us, profiles/r02_lds/ptrs_variants.log).
    //   bit 3 (PRE, column fold only): the loaders form the terms.  Each lane
    //     also loads its rows' factors and stashes t = fl(fl(x*a)*s) instead of
    //     x, with all 64 lanes busy, so the fold's per-row chain is one LDS read
    //     and one add (the same products and the same ordered adds: the same
    //     bits).  Without it the fold lanes (CPW of 64 per wave) also read the
    //     factors and multiply, row by row.
    const float* nxt[ROWS && !PRING ? LU : 1];
    auto fetch_ptrs = [&](int64_t c, Stage& g) {  // chunk index clamped, no branch
        if constexpr (ROWS) {
            const int64_t cc = c < nfull ? c : nfull - 1;
#pragma unroll
            for (int j = 0; j < LU; ++j) {
                const float* p = xi[cc * R + (t + j * NT) / RW];
                if constexpr (PRING) g.p[j] = p;
                else nxt[j] = p;
            }
        }
    };
    // Full chunks stream through loops whose loads carry no checks and no
    // control flow: a branch between a load and its use makes the compiler
    // wait for the load right after issuing it, which would serialise the
    // chunk loads with the fold.
    auto load_full = [&](int64_t c, Stage& g, int dist) {  // chunk c: rows [c*R, c*R + R)
        if constexpr (ROWS) {
#pragma unroll
            for (int j = 0; j < LU; ++j) {  // a global (not flat) load: the table holds device pointers
                const float* p;
                if constexpr (PRING) p = g.p[j];
                else p = nxt[j];
                if constexpr (DW) g.vf[j] = __builtin_nontemporal_load((const gf32*)p + fof(j));
                else g.v[j] = __builtin_nontemporal_load((const gf32x4*)p + qof(j));
            }
        } else if constexpr (DW) {
#pragma unroll
            for (int j = 0; j < LU; ++j)
                g.vf[j] = __builtin_nontemporal_load(X + (c * R + (t + j * NT) / RW) * ldx + fof(j));
        } else {
            const f32x4* X4 = reinterpret_cast<const f32x4*>(X);
#pragma unroll
            for (int j = 0; j < LQ; ++j)
                g.v[j] = __builtin_nontemporal_load(X4 + (c * R + (t + j * NT) / TQ) * ldq + qof(j));
        }
        if constexpr (PRE) {
#pragma unroll
            for (int j = 0; j < LU; ++j) {
                const int64_t row = c * R + (t + j * NT) / RW;
                g.pa[j] = a[row];
                if constexpr (SCORED) g.ps[j] = s[row];
            }
        } else if constexpr (LOPT & 1) {
            g.fv = a[c * R + t % R];
            if constexpr (SCORED) g.sv = s[c * R + t % R];
        } else if (t < R) {
            g.fv = a[c * R + t];
            if constexpr (SCORED) g.sv = s[c * R + t];
        }
        if constexpr (PRING) fetch_ptrs(c + dist, g);
        else if (c + 1 < nfull) fetch_ptrs(c + 1, g);
        if constexpr ((LOPT & 2) != 0) __builtin_amdgcn_sched_barrier(0);
    };
    auto load_rows_checked = [&](int64_t c, Stage& g) {  // the last, partial chunk: rows < N only
#pragma unroll
        for (int j = 0; j < LU; ++j) {
            const int64_t row = c * R + (t + j * NT) / RW;
            if (row < N) {
                if constexpr (DW) g.vf[j] = __builtin_nontemporal_load((const gf32*)rowf(row) + fof(j));
                else g.v[j] = __builtin_nontemporal_load((const gf32x4*)rowf(row) + qof(j));
                if constexpr (PRE) {
                    g.pa[j] = a[row];
                    if constexpr (SCORED) g.ps[j] = s[row];
                }
            }
        }
        if (!PRE && t < R && c * R + t < N) {
            g.fv = a[c * R + t];
            if constexpr (SCORED) g.sv = s[c * R + t];
        }
    };
    auto stash = [&](const Stage& g) {
        if constexpr (DW) {
            float* tw = reinterpret_cast<float*>(tile);  // [R][TQ*4] floats, the quad layout's bytes
#pragma unroll
            for (int j = 0; j < LU; ++j) {
                if constexpr (PRE) tw[t + j * NT] = term1<SCORED>(g.vf[j], g.pa[j], SCORED ? g.ps[j] : 1.0f);
                else tw[t + j * NT] = g.vf[j];
            }
        } else {
#pragma unroll
            for (int j = 0; j < LQ; ++j) {
                if constexpr (PRE) tile[t + j * NT] = term4<SCORED>(g.v[j], g.pa[j], SCORED ? g.ps[j] : 1.0f);
                else tile[t + j * NT] = g.v[j];
            }
        }
        if (!PRE && t < R) {
            fa[t] = g.fv;
            if constexpr (SCORED) fs[t] = g.sv;
        }
    };
    // column fold: this lane's column of the block (COLF)
    constexpr int TC = TQ * 4, CPW = (TC + NW - 1) / NW;
    static_assert(!COLF || CPW <= 64, "column fold: at most one column per lane");
    const int ccol = (t >> 6) * CPW + (t & 63);
    const bool cfold = (t & 63) < CPW && ccol < tq * 4;
    const float* tilef = reinterpret_cast<const float*>(tile);
    float acc1 = 0.f;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if constexpr (ACC) {
        if constexpr (COLF) {
            if (cfold) acc1 = acc_in[q0 * 4 + ccol];
        } else {
            if (t < tq) acc = reinterpret_cast<const f32x4*>(acc_in)[q0 + t];
        }
    }
    // fold the staged chunk c (rows valid rows) in client order
    auto fold = [&](int64_t c, int rows) {
        if constexpr (PRE) {  // the tile holds the terms
            if (cfold) {
                int r = 0;
                if (!ACC && c == 0) {
                    acc1 = tilef[ccol];
                    r = 1;
                }
                for (; r + 8 <= rows; r += 8) {
                    float x[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) x[k] = tilef[(r + k) * TC + ccol];
#pragma unroll
                    for (int k = 0; k < 8; ++k) acc1 = acc1 + x[k];
                }
                for (; r < rows; ++r) acc1 = acc1 + tilef[r * TC + ccol];
            }
        } else if constexpr (COLF) {
            if (cfold) {
                int r = 0;
                if (!ACC && c == 0) {
                    acc1 = term1<SCORED>(tilef[ccol], fa[0], SCORED ? fs[0] : 1.0f);
                    r = 1;
                }
                for (; r + 8 <= rows; r += 8) {
                    float x[8], f[8], g[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        x[k] = tilef[(r + k) * TC + ccol];
                        f[k] = fa[r + k];
                        g[k] = SCORED ? fs[r + k] : 1.0f;
                    }
#pragma unroll
                    for (int k = 0; k < 8; ++k) acc1 = acc1 + term1<SCORED>(x[k], f[k], g[k]);
                }
                for (; r < rows; ++r)
                    acc1 = acc1 + term1<SCORED>(tilef[r * TC + ccol], fa[r], SCORED ? fs[r] : 1.0f);
            }
        } else if (t < tq) {  // lane = quad, wave 0 only
            int r = 0;
            if (!ACC && c == 0) {
                acc = term4<SCORED>(tile[t], fa[0], SCORED ? fs[0] : 1.0f);
                r = 1;
            }
            // 8 LDS reads in flight ahead of the ordered adds (the reads are
            // independent, only the adds are ordered)
            for (; r + 8 <= rows; r += 8) {
                f32x4 x[8];
                float f[8], g[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    x[k] = tile[(r + k) * TQ + t];
                    f[k] = fa[r + k];
                    g[k] = SCORED ? fs[r + k] : 1.0f;
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) acc = add4(acc, term4<SCORED>(x[k], f[k], g[k]));
            }
            for (; r < rows; ++r) acc = add4(acc, term4<SCORED>(tile[r * TQ + t], fa[r], SCORED ? fs[r] : 1.0f));
        }
    };
    int64_t c = 0;  // next chunk to fold
    if (DEPTH >= 2 && nfull > DEPTH) {
        // DEPTH chunks in flight: LDS holds chunk c, stage st[(c+i) % DEPTH]
        // holds chunk c+i (i = 1..DEPTH), loading.  Stage indices are static
        // after unrolling (c stays a multiple of DEPTH at the loop head), so the
        // stages live in registers; the steady-state loop has no conditional load.
#pragma unroll
        for (int k = 0; k < (PRING ? DEPTH : 1); ++k) fetch_ptrs(k, st[k]);
        load_full(0, st[0], DEPTH);
        stash(st[0]);
        __syncthreads();
#pragma unroll
        for (int k = 1; k <= DEPTH; ++k) load_full(k, st[k % DEPTH], DEPTH);
        for (; c + 2 * DEPTH < nfull; c += DEPTH) {
#pragma unroll
            for (int k = 0; k < DEPTH; ++k) {
                fold(c + k, R);
                __syncthreads();                    // chunk c+k consumed
                stash(st[(k + 1) % DEPTH]);         // waits for that stage only
                __syncthreads();                    // chunk c+k+1 staged
                load_full(c + k + 1 + DEPTH, st[(k + 1) % DEPTH], DEPTH);
            }
        }
        // drain: LDS = c, stages = c+1 .. c+DEPTH (all < nfull), c+2*DEPTH >= nfull
#pragma unroll
        for (int k = 0; k < 2 * DEPTH; ++k) {
            const int64_t cc = c + k;
            if (cc < nfull) {
                fold(cc, R);
                __syncthreads();
                if (cc + 1 < nfull) {
                    stash(st[(k + 1) % DEPTH]);
                    __syncthreads();
                    if (cc + 1 + DEPTH < nfull) load_full(cc + 1 + DEPTH, st[(k + 1) % DEPTH], DEPTH);
                }
            }
        }
        c = nfull;
    } else if (nfull > 0) {
        fetch_ptrs(0, st[0]);
        load_full(0, st[0], 1);
        stash(st[0]);
        __syncthreads();
        for (; c + 1 < nfull; ++c) {
            load_full(c + 1, st[0], 1);  // in flight while chunk c is folded
            fold(c, R);
            __syncthreads();  // chunk c consumed
            stash(st[0]);
            __syncthreads();  // chunk c+1 staged
        }
        fold(c, R);
        __syncthreads();
        ++c;
    }
    if (c * R < N) {  // the last, partial chunk
        load_rows_checked(c, st[0]);
        stash(st[0]);
        __syncthreads();
        fold(c, (int)(N - c * R));
        __syncthreads();
    }
    if constexpr (COLF) {
        if (cfold) __builtin_nontemporal_store(FIN ? acc1 / divisor : acc1, out + q0 * 4 + ccol);
    } else if (t < tq) {
        const f32x4 res = FIN ? div4(acc, divisor) : acc;
        __builtin_nontemporal_store(res, reinterpret_cast<f32x4*>(out) + q0 + t);
    }
}

// ---------------------------------------------------------------------------
// TUNING VARIANT ONLY (measured and rejected, DESIGN.md 5 "LDS-DMA ring"):
// the product never launches it; it stays in libfedavg_hip_bench.so as the
// measured answer to the "deeper LDS ring" idea.
// Narrow models, deep ring: LDS-DMA (global_load_lds) into an S-slot ring.
//   Same tile as k_fold_f32_lds with the round-1 quad fold (a block owns TQ
//   quads of every row; wave 0 folds each R-row chunk from LDS in client
//   order, one lane per quad),
//   but the chunks are copied HBM -> LDS by global_load_lds_dwordx4, which
//   needs no VGPRs: S - 1 chunks stay in flight per block (the register-staged
//   fold holds two), which was the hypothesis for narrow models (it measured
//   slower everywhere).  Counters on
//   1024 x 16K / 67K (profiles/r02_narrow/SUMMARY.md): SQ_WAIT_ANY = 72-80 %
//   of the wave cycles with at most two chunks in flight, i.e. latency-bound.
//   Synchronisation per chunk: each wave's counted `s_waitcnt vmcnt` retires
//   its own copies of chunk c (later chunks stay in flight), then a raw
//   s_barrier makes everyone's copies visible and tells the loaders that wave
//   0 has finished the chunk before (whose slot the next copy reuses).  No
//   ordinary global load sits inside the ring (hipcc would drain the ring at
//   its first use), and all LDS is one __shared__ array.
//   The factors of a chunk travel the same way (4-byte copies, lanes < R).
//   The last partial chunk (N % R rows) and the P%4 tail columns take the
//   register paths of k_fold_f32_lds after the ring has drained.
// ---------------------------------------------------------------------------
template <int N_>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N_ >= 0 && N_ < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N_ & 0xF) | ((N_ >> 4) << 14) | 0x70 | 0xF00);  // vmcnt(N_) only
}

__device__ __forceinline__ void glds16(const void* src, void* lds) {
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}
__device__ __forceinline__ void glds4(const void* src, void* lds) {
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)lds, 4, 0, 0);
}

template <int NW, int R, int TQ, int S, bool SCORED, bool ACC, bool FIN>
__global__ __launch_bounds__(NW * 64) void k_fold_f32_ring(
    const float* __restrict__ X, int64_t N, int64_t P, int64_t ldx,
    const float* __restrict__ a, const float* __restrict__ s,
    const float* acc_in, float divisor, float* out) {  // acc_in may alias out
    constexpr int NT = NW * 64;
    constexpr int LQ = R * TQ / NT;                 // 16-B copies per thread per chunk
    constexpr int F = SCORED ? 2 : 1;               // factor copies per chunk (wave 0)
    constexpr int TILE_B = R * TQ * 16;
    constexpr int SLOT_B = TILE_B + ((F * R * 4 + 15) / 16) * 16;
    static_assert(TQ <= 64 && 64 % TQ == 0 && (R * TQ) % NT == 0 && R <= 64 && S >= 3, "ring shape");
    static_assert((S - 2) * (LQ + F) < 64, "vmcnt range");
    __shared__ __attribute__((aligned(16))) char smem[S * SLOT_B];
    const int t = threadIdx.x;
    const int lane = t & 63;
    const int w = __builtin_amdgcn_readfirstlane(t >> 6);
    const int64_t nq = P >> 2;
    const int64_t nbq = (nq + TQ - 1) / TQ;
    const int64_t ldq = ldx >> 2;
    const f32x4* X4 = reinterpret_cast<const f32x4*>(X);
    f32x4* tile0 = reinterpret_cast<f32x4*>(smem);

    if ((int64_t)blockIdx.x >= nbq) {
        // ---- the P%4 tail columns: row-parallel terms, thread 0 adds in order ----
        const int w4 = (int)(P & 3);
        const int64_t col0 = nq * 4;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        if (ACC && t == 0)
            for (int k = 0; k < w4; ++k) acc[k] = acc_in[col0 + k];
        for (int64_t r0 = 0; r0 < N; r0 += NT) {
            const int64_t row = r0 + t;
            if (row < N) {
                f32x4 x = {0.f, 0.f, 0.f, 0.f};
                for (int k = 0; k < w4; ++k) x[k] = X[row * ldx + col0 + k];
                tile0[t] = term4<SCORED>(x, a[row], SCORED ? s[row] : 1.0f);
            }
            __syncthreads();
            if (t == 0) {
                const int rows = (N - r0) < NT ? (int)(N - r0) : NT;
                int i = 0;
                if (!ACC && r0 == 0) {
                    acc = tile0[0];
                    i = 1;
                }
                for (; i < rows; ++i) acc = add4(acc, tile0[i]);
            }
            __syncthreads();
        }
        if (t == 0) {
            const f32x4 res = FIN ? div4(acc, divisor) : acc;
            for (int k = 0; k < w4; ++k) out[col0 + k] = res[k];
        }
        return;
    }

    const int64_t q0 = (int64_t)blockIdx.x * TQ;
    const int tq = (int)((nq - q0) < TQ ? (nq - q0) : TQ);
    auto qof = [&](int j) -> int64_t {  // clamped: the last block's lanes past the end re-read a valid quad
        const int64_t q = q0 + (t + j * NT) % TQ;
        return q < nq ? q : nq - 1;
    };
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if constexpr (ACC) {
        if (t < tq) acc = reinterpret_cast<const f32x4*>(acc_in)[q0 + t];
        wait_vmcnt<0>();  // before the ring: no ordinary load may be pending inside it
    }
    const int64_t nfull = N / R;
    auto issue = [&](int64_t c) {  // copy chunk c into slot c % S (every wave its share)
        char* slot = smem + (int)(c % S) * SLOT_B;
#pragma unroll
        for (int j = 0; j < LQ; ++j)
            glds16(X4 + (c * R + (t + j * NT) / TQ) * ldq + qof(j), slot + (j * NT + w * 64) * 16);
        if (w == 0 && lane < R) {
            glds4(a + c * R + lane, slot + TILE_B);
            if constexpr (SCORED) glds4(s + c * R + lane, slot + TILE_B + R * 4);
        }
    };
    auto fold = [&](const char* slot, int rows, bool first) {
        const f32x4* tile = reinterpret_cast<const f32x4*>(slot);
        const float* fa = reinterpret_cast<const float*>(slot + TILE_B);
        const float* fs = fa + R;
        if (t < tq) {
            int r = 0;
            if (first) {
                acc = term4<SCORED>(tile[t], fa[0], SCORED ? fs[0] : 1.0f);
                r = 1;
            }
            for (; r + 8 <= rows; r += 8) {
                f32x4 x[8];
                float f[8], g[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    x[k] = tile[(r + k) * TQ + t];
                    f[k] = fa[r + k];
                    g[k] = SCORED ? fs[r + k] : 1.0f;
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) acc = add4(acc, term4<SCORED>(x[k], f[k], g[k]));
            }
            for (; r < rows; ++r) acc = add4(acc, term4<SCORED>(tile[r * TQ + t], fa[r], SCORED ? fs[r] : 1.0f));
        }
    };
    const int64_t pre = nfull < S - 1 ? nfull : S - 1;
    for (int64_t c = 0; c < pre; ++c) issue(c);
    for (int64_t c = 0; c < nfull; ++c) {
        // retire this wave's copies of chunk c; chunks c+1 .. c+S-2 stay in flight
        if (c + S - 2 < nfull) {
            if (w == 0) wait_vmcnt<(S - 2) * (LQ + F)>();
            else wait_vmcnt<(S - 2) * LQ>();
        } else {
            wait_vmcnt<0>();
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // everyone's copies of c landed; wave 0 is done with c-1
        if (c + S - 1 < nfull) issue(c + S - 1);
        if (w == 0) fold(smem + (int)(c % S) * SLOT_B, R, !ACC && c == 0);
    }
    wait_vmcnt<0>();
    __syncthreads();
    if (nfull * R < N) {  // the last, partial chunk: register path through slot 0
        const int64_t c = nfull;
        f32x4* tile = tile0;
        float* fa = reinterpret_cast<float*>(smem + TILE_B);
#pragma unroll
        for (int j = 0; j < LQ; ++j) {
            const int64_t row = c * R + (t + j * NT) / TQ;
            if (row < N) tile[t + j * NT] = __builtin_nontemporal_load(X4 + row * ldq + qof(j));
        }
        if (t < R && c * R + t < N) {
            fa[t] = a[c * R + t];
            if constexpr (SCORED) fa[R + t] = s[c * R + t];
        }
        __syncthreads();
        if (w == 0) fold(smem, (int)(N - c * R), !ACC && c == 0);
        __syncthreads();
    }
    if (t < tq) {
        const f32x4 res = FIN ? div4(acc, divisor) : acc;
        __builtin_nontemporal_store(res, reinterpret_cast<f32x4*>(out) + q0 + t);
    }
}

template <int NW, int R, int TQ, int S, bool ALLF = false>
int launch_ring_flags(hipStream_t st, bool sc, bool acc, bool fin, const float* X, int64_t N, int64_t P,
                      int64_t ldx, const float* a, const float* s, const float* acc_in, float d, float* out) {
    const int64_t blocks = ((P >> 2) + TQ - 1) / TQ + ((P & 3) ? 1 : 0);
    if (blocks * NW * 64 > (int64_t)0xFFFFFFFF)
        return fail(FA_ERR_ARG, "P=%lld too large for a ring launch", (long long)P);
    const dim3 grid((unsigned)blocks), block(NW * 64);
#define FA_RG(SC, ACC, FIN) \
    hipLaunchKernelGGL((k_fold_f32_ring<NW, R, TQ, S, SC, ACC, FIN>), grid, block, 0, st, X, N, P, ldx, a, s, \
                       acc_in, d, out)
    if constexpr (!ALLF) {
        if (sc) FA_RG(true, false, true); else FA_RG(false, false, true);
    } else if (sc) {
        if (acc) { if (fin) FA_RG(true, true, true); else FA_RG(true, true, false); }
        else     { if (fin) FA_RG(true, false, true); else FA_RG(true, false, false); }
    } else {
        if (acc) { if (fin) FA_RG(false, true, true); else FA_RG(false, true, false); }
        else     { if (fin) FA_RG(false, false, true); else FA_RG(false, false, false); }
    }
#undef FA_RG
    return FA_OK;
}

// ---------------------------------------------------------------------------
// One-wave LDS-DMA fold for narrow models (k_fold_f32_w1, round 3; measured
// and NOT adopted: tuning variants w1_* only).  1024 x 16K: 21.3 us (64-row
// chunks, 3 in flight) against 18.6 us for the two-wave LDS pick; 1024 x 67K
// 0.065 against 0.045 ms; 16-row chunks 32.5 us: the per-chunk wait / issue
// cadence of one wave, not the barriers, bounds it
// (profiles/r03_w1_rejected/).  A block is ONE wave owning 64 columns
// (16 quads): every chunk of R client rows is copied HBM -> LDS with
// global_load_lds_dwordx4 (a wave-instruction moves 4 rows x 256 B), S-1
// chunks in flight, and the same wave folds each landed chunk with one column
// per lane (all 64 lanes, a 4-byte LDS read, a multiply and an add per row),
// strictly in row order.  One wave needs no s_barrier: the chunk's vmcnt
// retires its copies, and a slot is refilled only after the wave has folded
// it (its reads were consumed by the adds).  The multi-wave LDS forms pay two
// barriers per chunk and fold with half the lanes idle at 16K params (two
// waves over 64 columns, CPW = 32).  The last partial chunk (N % R rows) and
// the P%4 tail columns take register paths, as k_fold_f32_ring.
// ---------------------------------------------------------------------------
template <int R, int S, bool SCORED>
__global__ __launch_bounds__(64) void k_fold_f32_w1(
    const float* __restrict__ X, int64_t N, int64_t P, int64_t ldx,
    const float* __restrict__ a, const float* __restrict__ s, float divisor, float* out) {
    constexpr int TQ = 16;                                   // quads per block: 64 columns
    constexpr int LQ = R * TQ / 64;                          // 16-B copies per lane per chunk
    constexpr int F = SCORED ? 2 : 1;                        // factor copies per chunk
    constexpr int TILE_B = R * TQ * 16;                      // R rows x 256 B
    constexpr int SLOT_B = TILE_B + ((F * R * 4 + 15) / 16) * 16;
    static_assert(R % 4 == 0 && R <= 64 && S >= 3, "w1 shape");
    static_assert((S - 2) * (LQ + F) < 64, "vmcnt range");
    __shared__ __attribute__((aligned(16))) char smem[S * SLOT_B];
    const int t = threadIdx.x;
    const int64_t nq = P >> 2;
    const int64_t nbq = (nq + TQ - 1) / TQ;
    const int64_t ldq = ldx >> 2;
    const f32x4* X4 = reinterpret_cast<const f32x4*>(X);

    if ((int64_t)blockIdx.x >= nbq) {
        // ---- the P%4 tail columns: row-parallel terms, lane 0 adds in order ----
        f32x4* tile0 = reinterpret_cast<f32x4*>(smem);
        const int w4 = (int)(P & 3);
        const int64_t col0 = nq * 4;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        for (int64_t r0 = 0; r0 < N; r0 += 64) {
            const int64_t row = r0 + t;
            if (row < N) {
                f32x4 x = {0.f, 0.f, 0.f, 0.f};
                for (int k = 0; k < w4; ++k) x[k] = X[row * ldx + col0 + k];
                tile0[t] = term4<SCORED>(x, a[row], SCORED ? s[row] : 1.0f);
            }
            __syncthreads();
            if (t == 0) {
                const int rows = (N - r0) < 64 ? (int)(N - r0) : 64;
                int i = 0;
                if (r0 == 0) {
                    acc = tile0[0];
                    i = 1;
                }
                for (; i < rows; ++i) acc = add4(acc, tile0[i]);
            }
            __syncthreads();
        }
        if (t == 0) {
            const f32x4 res = div4(acc, divisor);
            for (int k = 0; k < w4; ++k) out[col0 + k] = res[k];
        }
        return;
    }

    const int64_t q0 = (int64_t)blockIdx.x * TQ;
    const int tq = (int)((nq - q0) < TQ ? (nq - q0) : TQ);
    // the quad this lane copies (the same for every copy: 16 lanes per row), clamped
    // for the last block's lanes past the end (a valid address whose value is never stored)
    const int64_t myq = (q0 + (t % TQ)) < nq ? q0 + (t % TQ) : nq - 1;
    const int rsub = t / TQ;  // this lane's row within each 4-row copy
    float acc = 0.f;
    const int64_t nfull = N / R;
    auto issue = [&](int64_t c) {
        char* slot = smem + (int)(c % S) * SLOT_B;
#pragma unroll
        for (int j = 0; j < LQ; ++j) glds16(X4 + (c * R + 4 * j + rsub) * ldq + myq, slot + j * 1024);
        if (t < R) {
            glds4(a + c * R + t, slot + TILE_B);
            if constexpr (SCORED) glds4(s + c * R + t, slot + TILE_B + R * 4);
        }
    };
    auto fold = [&](const char* slot, int rows, bool first) {
        const float* tile = reinterpret_cast<const float*>(slot);  // [rows][64] floats
        const float* fa = reinterpret_cast<const float*>(slot + TILE_B);
        const float* fs = fa + R;
        int r = 0;
        if (first) {
            acc = term1<SCORED>(tile[t], fa[0], SCORED ? fs[0] : 1.0f);
            r = 1;
        }
        for (; r + 8 <= rows; r += 8) {
            float x[8], f[8], g[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                x[k] = tile[(r + k) * 64 + t];
                f[k] = fa[r + k];
                g[k] = SCORED ? fs[r + k] : 1.0f;
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) acc = acc + term1<SCORED>(x[k], f[k], g[k]);
        }
        for (; r < rows; ++r) acc = acc + term1<SCORED>(tile[r * 64 + t], fa[r], SCORED ? fs[r] : 1.0f);
    };
    const int64_t pre = nfull < S - 1 ? nfull : S - 1;
    for (int64_t c = 0; c < pre; ++c) issue(c);
    for (int64_t c = 0; c < nfull; ++c) {
        // chunk c landed; chunks c+1 .. c+S-2 stay in flight
        if (c + S - 2 < nfull) wait_vmcnt<(S - 2) * (LQ + F)>();
        else wait_vmcnt<0>();
        // slot (c-1) % S was folded in the previous iteration: its LDS reads
        // are complete before the copies into it are issued; the "memory"
        // clobber also keeps the compiler from moving chunk c's LDS reads above
        // the vmcnt wait
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (c + S - 1 < nfull) issue(c + S - 1);
        fold(smem + (int)(c % S) * SLOT_B, R, c == 0);
    }
    wait_vmcnt<0>();
    if (nfull * R < N) {  // the last, partial chunk: register path through slot 0
        const int64_t c = nfull;
        f32x4* tile = reinterpret_cast<f32x4*>(smem);
        float* fa = reinterpret_cast<float*>(smem + TILE_B);
#pragma unroll
        for (int j = 0; j < LQ; ++j) {
            const int64_t row = c * R + 4 * j + rsub;
            if (row < N) tile[j * 64 + t] = __builtin_nontemporal_load(X4 + row * ldq + myq);
        }
        if (t < R && c * R + t < N) {
            fa[t] = a[c * R + t];
            if constexpr (SCORED) fa[R + t] = s[c * R + t];
        }
        __syncthreads();
        fold(smem, (int)(N - c * R), c == 0);
    }
    if (t < 4 * tq) __builtin_nontemporal_store(acc / divisor, out + q0 * 4 + t);
}

template <int R, int S>
int launch_w1(hipStream_t st, bool sc, const float* X, int64_t N, int64_t P, int64_t ldx, const float* a,
              const float* s, float d, float* out) {
    const int64_t blocks = ((P >> 2) + 15) / 16 + ((P & 3) ? 1 : 0);
    if (blocks > (int64_t)0x7FFFFFFF) return fail(FA_ERR_ARG, "P=%lld too large for a w1 launch", (long long)P);
    if (sc)
        hipLaunchKernelGGL((k_fold_f32_w1<R, S, true>), dim3((unsigned)blocks), dim3(64), 0, st, X, N, P, ldx, a, s,
                           d, out);
    else
        hipLaunchKernelGGL((k_fold_f32_w1<R, S, false>), dim3((unsigned)blocks), dim3(64), 0, st, X, N, P, ldx, a, s,
                           d, out);
    return FA_OK;
}

// Split-client fold (opt-in, NOT bit-exact; fa_fedavg_f32_splitn).
//   For models too narrow to fill the chip even with LDS staging, the
//   clients of every column are cut into S = 4*NW contiguous slices.  A block
//   owns 16 quads (64 columns); lane l of wave w folds quad l%16 over slice
//   4*w + l/16, in client order, 8 rows ahead.  The S partial sums are then
//   combined in a FIXED pairwise tree -- two wavefront shuffles (slice pairs,
//   then pairs of pairs), then the waves' partials through LDS -- so the
//   result is deterministic run to run, but it is a different association
//   than the reference's left fold: it differs in the last bits (normwise
//   error measured in tests/test_gpu_parity.py and DESIGN.md 5).
template <int NW, bool SCORED>
__global__ __launch_bounds__(NW * 64) void k_fold_f32_splitn(
    const float* __restrict__ X, int64_t N, int64_t P, int64_t ldx,
    const float* __restrict__ a, const float* __restrict__ s, float divisor, float* __restrict__ out) {
    constexpr int S = 4 * NW;  // client slices
    constexpr int U = 8;
    __shared__ f32x4 part[NW][16];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int qq = lane & 15, slice = 4 * w + (lane >> 4);
    const int64_t nq = P >> 2, q = (int64_t)blockIdx.x * 16 + qq;
    const int64_t ns = (N + S - 1) / S;
    const int64_t r0 = slice * ns < N ? slice * ns : N, r1 = r0 + ns < N ? r0 + ns : N;
    const int64_t ldq = ldx >> 2;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if ((int64_t)blockIdx.x * 16 + 16 <= nq) {  // block-uniform: 16 full quads, no checks in the loop
        const f32x4* p = reinterpret_cast<const f32x4*>(X) + q;
        int64_t i = r0;
        if (i < r1) {
            acc = term4<SCORED>(__builtin_nontemporal_load(p + i * ldq), a[i], SCORED ? s[i] : 1.0f);
            ++i;
        }
        for (; i + U <= r1; i += U) {
            f32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(p + (i + u) * ldq);
#pragma unroll
            for (int u = 0; u < U; ++u) acc = add4(acc, term4<SCORED>(v[u], a[i + u], SCORED ? s[i + u] : 1.0f));
        }
        for (; i < r1; ++i)
            acc = add4(acc, term4<SCORED>(__builtin_nontemporal_load(p + i * ldq), a[i], SCORED ? s[i] : 1.0f));
    } else if (q * 4 < P) {  // last block: full and partial quads, element loads
        const int w4 = (P - q * 4) < 4 ? (int)(P - q * 4) : 4;
        for (int64_t i = r0; i < r1; ++i) {
            f32x4 x = {0.f, 0.f, 0.f, 0.f};
            for (int k = 0; k < w4; ++k) x[k] = X[i * ldx + q * 4 + k];
            const f32x4 t = term4<SCORED>(x, a[i], SCORED ? s[i] : 1.0f);
            acc = i == r0 ? t : add4(acc, t);
        }
    }
    // fixed tree: slice pairs (xor 16), pairs of pairs (xor 32); fp add is
    // commutative, so both lanes of a pair hold the same bits
#pragma unroll
    for (int off = 16; off <= 32; off <<= 1) {
        f32x4 o;
        o.x = __shfl_xor(acc.x, off);
        o.y = __shfl_xor(acc.y, off);
        o.z = __shfl_xor(acc.z, off);
        o.w = __shfl_xor(acc.w, off);
        acc = add4(acc, o);
    }
    if (lane < 16) part[w][qq] = acc;
    __syncthreads();
    if (w == 0 && lane < 16 && q * 4 < P) {
        f32x4 t[NW];
#pragma unroll
        for (int k = 0; k < NW; ++k) t[k] = part[k][qq];
#pragma unroll
        for (int stride = 1; stride < NW; stride <<= 1)  // ((p0+p1)+(p2+p3))+...
#pragma unroll
            for (int k = 0; k + stride < NW; k += 2 * stride) t[k] = add4(t[k], t[k + stride]);
        const f32x4 r = div4(t[0], divisor);
        if (q < nq) {
            __builtin_nontemporal_store(r, reinterpret_cast<f32x4*>(out) + q);
        } else {
            for (int k = 0; k < (int)(P & 3); ++k) out[q * 4 + k] = r[k];
        }
    }
}

// One column per lane, any alignment / stride (fallback for unaligned input).
template <bool SCORED, bool ACC, bool FIN>
__global__ __launch_bounds__(kBlock) void k_fold_f32_scalar(
    const float* __restrict__ X, int64_t N, int64_t P, int64_t ldx,
    const float* __restrict__ a, const float* __restrict__ s,
    const float* acc_in, float divisor, float* out) {  // acc_in may alias out
    const int64_t c = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (c >= P) return;
    float acc;
    int64_t i = 0;
    if constexpr (ACC) {
        acc = acc_in[c];
    } else {
        acc = term1<SCORED>(X[c], a[0], SCORED ? s[0] : 1.0f);
        i = 1;
    }
#pragma unroll 8
    for (; i < N; ++i) acc = acc + term1<SCORED>(X[i * ldx + c], a[i], SCORED ? s[i] : 1.0f);
    if constexpr (FIN) acc = acc / divisor;
    out[c] = acc;
}

// ---------------------------------------------------------------------------
// Even split: a persistent grid of G blocks (one per CU) where block b owns
// the contiguous quad range [b*per, min((b+1)*per, nq)), per = ceil(nq / G).
// Every block streams the same bytes (to one quad per row), so the launch
// ends when every CU ends: no partly-filled last round of blocks, no idle CUs
// (the tile launches leave 20-30 % of the CUs idle at 0.7-0.9 tiles per CU).
// Inside its range a block walks chunks of C*kBlock quads, lane l taking quads
// chunk + l + kBlock*c (every wave-load one contiguous 1 KiB run).  A lane
// whose quad lies past the range loads the range's last quad instead (a valid
// address the wave's other lanes already read: one merged cache line) and
// never stores it, so the loads carry no branch.  Rows go U at a time with
// every row index clamped to N-1 and the adds of rows past N skipped (a
// wave-uniform test after the loads), so the client tail is pipelined too.
// Same per-column in-order fold as every other kernel (bit-identical).
// The P%4 tail columns are folded by the last lane of the last block.
// ---------------------------------------------------------------------------
template <int U, int C, bool SCORED, bool ACC, bool FIN>
__global__ __launch_bounds__(kBlock) void k_fold_f32_even(
    const float* __restrict__ X, int64_t N, int64_t P, int64_t ldx,
    const float* __restrict__ a, const float* __restrict__ s,
    const float* acc_in, float divisor, float* out, int64_t per) {  // acc_in may alias out
    const int64_t nq = P >> 2, ldq = ldx >> 2;
    const f32x4* X4 = reinterpret_cast<const f32x4*>(X);
    const int64_t lo = (int64_t)blockIdx.x * per;
    const int64_t hi = lo + per < nq ? lo + per : nq;
    for (int64_t base = lo; base < hi; base += (int64_t)C * kBlock) {
        int64_t q[C];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int64_t qq = base + threadIdx.x + (int64_t)c * kBlock;
            q[c] = qq < hi ? qq : hi - 1;
        }
        f32x4 acc[C];
        int64_t i0;
        if constexpr (ACC) {
#pragma unroll
            for (int c = 0; c < C; ++c) acc[c] = reinterpret_cast<const f32x4*>(acc_in)[q[c]];
            i0 = 0;
        } else {
            const float a0 = a[0], s0 = SCORED ? s[0] : 1.0f;
#pragma unroll
            for (int c = 0; c < C; ++c) acc[c] = term4<SCORED>(__builtin_nontemporal_load(X4 + q[c]), a0, s0);
            i0 = 1;
        }
        for (int64_t i = i0; i < N; i += U) {
            f32x4 v[U][C];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t r = i + u < N ? i + u : N - 1;
#pragma unroll
                for (int c = 0; c < C; ++c) v[u][c] = __builtin_nontemporal_load(X4 + r * ldq + q[c]);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (i + u < N) {  // wave-uniform
                    const float ai = a[i + u], si = SCORED ? s[i + u] : 1.0f;
#pragma unroll
                    for (int c = 0; c < C; ++c) acc[c] = add4(acc[c], term4<SCORED>(v[u][c], ai, si));
                }
            }
        }
#pragma unroll
        for (int c = 0; c < C; ++c) {
            if (base + threadIdx.x + (int64_t)c * kBlock < hi) {
                const f32x4 r = FIN ? div4(acc[c], divisor) : acc[c];
                __builtin_nontemporal_store(r, reinterpret_cast<f32x4*>(out) + q[c]);
            }
        }
    }
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
#pragma unroll 8
            for (; i < N; ++i) acc = acc + term1<SCORED>(X[i * ldx + col], a[i], SCORED ? s[i] : 1.0f);
            if constexpr (FIN) acc = acc / divisor;
            out[col] = acc;
        }
    }
}

// List-of-rows form: xi[i] = device pointer to client i's P floats.  A lane
// owns 4 columns; U rows are loaded ahead of the ordered adds.  The row
// alignment test is wave-uniform (every lane reads the same pointer).
__device__ __forceinline__ f32x4 load_row4(const float* row, int64_t c0, int w) {
    if (w == 4 && aligned16(row)) return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(row + c0));
    f32x4 x = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < w; ++k) x[k] = row[c0 + k];
    return x;
}

template <int U, bool SCORED>
__global__ __launch_bounds__(kBlock) void k_fedavg_f32_ptrs(
    const float* const* __restrict__ xi, int64_t N, int64_t P,
    const float* __restrict__ a, const float* __restrict__ s, float divisor,
    float* __restrict__ out) {
    const int64_t c0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * 4;
    if (c0 >= P) return;
    const int w = (P - c0) >= 4 ? 4 : (int)(P - c0);
    f32x4 acc = term4<SCORED>(load_row4(xi[0], c0, w), a[0], SCORED ? s[0] : 1.0f);
    int64_t i = 1;
    for (; i + U <= N; i += U) {
        f32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = load_row4(xi[i + u], c0, w);
#pragma unroll
        for (int u = 0; u < U; ++u) acc = add4(acc, term4<SCORED>(v[u], a[i + u], SCORED ? s[i + u] : 1.0f));
    }
    for (; i < N; ++i) acc = add4(acc, term4<SCORED>(load_row4(xi[i], c0, w), a[i], SCORED ? s[i] : 1.0f));
    acc = div4(acc, divisor);
    if (w == 4 && aligned16(out + c0)) {
        *reinterpret_cast<f32x4*>(out + c0) = acc;
    } else {
        for (int k = 0; k < w; ++k) out[c0 + k] = acc[k];
    }
}

// List-of-rows form, rows at any 4-B offset, large models: lane = one column,
// row i's base a wave-uniform load from the table, 8 rows of loads ahead of the
// ordered adds.  Consecutive lanes read consecutive floats of a row: every
// wave-load is one contiguous 256-byte run, whatever the row's alignment.
template <bool SCORED>
__global__ __launch_bounds__(kBlock) void k_fold_f32_rows_scalar(
    const float* const* __restrict__ xi, int64_t N, int64_t P,
    const float* __restrict__ a, const float* __restrict__ s, float divisor, float* __restrict__ out) {
    const int64_t c = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (c >= P) return;
    float acc = term1<SCORED>(((const gf32*)xi[0])[c], a[0], SCORED ? s[0] : 1.0f);
    int64_t i = 1;
    for (; i + 8 <= N; i += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load((const gf32*)xi[i + u] + c);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc = acc + term1<SCORED>(v[u], a[i + u], SCORED ? s[i + u] : 1.0f);
    }
    for (; i < N; ++i) acc = acc + term1<SCORED>(((const gf32*)xi[i])[c], a[i], SCORED ? s[i] : 1.0f);
    out[c] = acc / divisor;
}

// List-of-rows form with every row 16-B aligned (fa_fedavg_f32_ptrs_aligned):
// the tile structure of the stacked fold (C quads per lane, U rows ahead) with
// row i's base read from xi[i] (a wave-uniform scalar load).  No branch sits
// between the loads and their use.
template <int U, int C, bool SCORED>
__device__ __forceinline__ void fold_quads_rows(const float* const* __restrict__ xi, int64_t q0, int64_t N,
                                                const float* __restrict__ a, const float* __restrict__ s,
                                                float divisor, f32x4* __restrict__ out) {
    f32x4 acc[C];
    {
        const f32x4* r = reinterpret_cast<const f32x4*>(xi[0]) + q0;
        const float a0 = a[0], s0 = SCORED ? s[0] : 1.0f;
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] = term4<SCORED>(__builtin_nontemporal_load(r + c * kBlock), a0, s0);
    }
    int64_t i = 1;
    for (; i + U <= N; i += U) {
        f32x4 v[U][C];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const f32x4* r = reinterpret_cast<const f32x4*>(xi[i + u]) + q0;
#pragma unroll
            for (int c = 0; c < C; ++c) v[u][c] = __builtin_nontemporal_load(r + c * kBlock);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float ai = a[i + u], si = SCORED ? s[i + u] : 1.0f;
#pragma unroll
            for (int c = 0; c < C; ++c) acc[c] = add4(acc[c], term4<SCORED>(v[u][c], ai, si));
        }
    }
    for (; i < N; ++i) {
        const f32x4* r = reinterpret_cast<const f32x4*>(xi[i]) + q0;
        const float ai = a[i], si = SCORED ? s[i] : 1.0f;
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] = add4(acc[c], term4<SCORED>(__builtin_nontemporal_load(r + c * kBlock), ai, si));
    }
#pragma unroll
    for (int c = 0; c < C; ++c) __builtin_nontemporal_store(div4(acc[c], divisor), out + c * kBlock);
}

template <int U, int C, bool SCORED>
__global__ __launch_bounds__(kBlock) void k_fold_f32_rows_gs(
    const float* const* __restrict__ xi, int64_t N, int64_t P, const float* __restrict__ a,
    const float* __restrict__ s, float divisor, float* __restrict__ out, int64_t ntiles) {
    const int64_t nq = P >> 2;
    f32x4* O4 = reinterpret_cast<f32x4*>(out);
    for (int64_t bid = blockIdx.x; bid < ntiles; bid += gridDim.x) {
        const int64_t q0 = bid * (kBlock * C) + threadIdx.x;
        if (q0 + (int64_t)(C - 1) * kBlock < nq) {
            fold_quads_rows<U, C, SCORED>(xi, q0, N, a, s, divisor, O4 + q0);
        } else {
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const int64_t q = q0 + (int64_t)c * kBlock;
                if (q < nq) fold_quads_rows<U, 1, SCORED>(xi, q, N, a, s, divisor, O4 + q);
            }
            const int64_t tb = nq / (kBlock * C), tl = (nq % (kBlock * C)) % kBlock;
            if ((P & 3) && bid == tb && (int64_t)threadIdx.x == tl) {
                for (int64_t col = nq * 4; col < P; ++col) {
                    float acc = term1<SCORED>(xi[0][col], a[0], SCORED ? s[0] : 1.0f);
                    for (int64_t i = 1; i < N; ++i) acc = acc + term1<SCORED>(xi[i][col], a[i], SCORED ? s[i] : 1.0f);
                    out[col] = acc / divisor;
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// bf16: 8 columns per lane (one 16-byte load per row), exact upcast, f32 fold.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float bf2f(uint32_t bits16) { return __uint_as_float(bits16 << 16); }

__device__ __forceinline__ uint16_t f2bf_rne(float f) {
    uint32_t u = __float_as_uint(f);
    if (f != f) return (uint16_t)((u >> 16) | 0x40u);
    return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}

// A 16-byte load holds 8 bf16 = 4 words; the low half of word k is column 2k,
// the high half column 2k+1.  Exact upcast = the half moved to the top of an
// f32, so the 8 columns fold as two f32x4 (even / odd columns).
__device__ __forceinline__ void unpack_bf16x8(u32x4 w, f32x4& even, f32x4& odd) {
    even = __builtin_bit_cast(f32x4, w << 16);
    odd = __builtin_bit_cast(f32x4, w & 0xFFFF0000u);
}

// A 16-byte non-temporal output store
__device__ __forceinline__ void st16(void* p, u32x4 v) { __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p)); }


// One row group of U rows x C octets: loaded (ld) and folded in row order (add)
template <int U, int C>
__device__ __forceinline__ void octets_ld(u32x4 (&v)[U][C], const u32x4* __restrict__ p, int64_t i, int64_t ldo) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int c = 0; c < C; ++c) v[u][c] = __builtin_nontemporal_load(p + (i + u) * ldo + c * kBlock);
}
template <int U, int C, bool SCORED>
__device__ __forceinline__ void octets_add(f32x4 (&ev)[C], f32x4 (&od)[C], const u32x4 (&v)[U][C],
                                           const float* __restrict__ a, const float* __restrict__ s, int64_t i) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const float ai = a[i + u], si = SCORED ? s[i + u] : 1.0f;
#pragma unroll
        for (int c = 0; c < C; ++c) {
            f32x4 e, o;
            unpack_bf16x8(v[u][c], e, o);
            ev[c] = add4(ev[c], term4<SCORED>(e, ai, si));
            od[c] = add4(od[c], term4<SCORED>(o, ai, si));
        }
    }
}

template <int U, int C, bool SCORED, int B = kBlock, int WT = 0>
__device__ __forceinline__ void fold_octets(const u32x4* __restrict__ p, int64_t ldo, int64_t N,
                                            const float* __restrict__ a, const float* __restrict__ s,
                                            float divisor, float* __restrict__ out, uint16_t* __restrict__ outb,
                                            int64_t o0) {
    static_assert(B == kBlock, "octet tiles are kBlock lanes wide");
    f32x4 ev[C], od[C];
    {
        const float a0 = a[0], s0 = SCORED ? s[0] : 1.0f;
#pragma unroll
        for (int c = 0; c < C; ++c) {
            f32x4 e, o;
            unpack_bf16x8(__builtin_nontemporal_load(p + c * B), e, o);
            ev[c] = term4<SCORED>(e, a0, s0);
            od[c] = term4<SCORED>(o, a0, s0);
        }
    }
    int64_t i = 1;
    for (; i + U <= N; i += U) {
        u32x4 v[U][C];
        octets_ld<U, C>(v, p, i, ldo);
        // deep unrolls: every load of the group issued before the first add
        if constexpr (U >= 16) __builtin_amdgcn_sched_barrier(0);
        octets_add<U, C, SCORED>(ev, od, v, a, s, i);
    }
    for (; i < N; ++i) {
        const float ai = a[i], si = SCORED ? s[i] : 1.0f;
#pragma unroll
        for (int c = 0; c < C; ++c) {
            f32x4 e, o;
            unpack_bf16x8(__builtin_nontemporal_load(p + i * ldo + c * B), e, o);
            ev[c] = add4(ev[c], term4<SCORED>(e, ai, si));
            od[c] = add4(od[c], term4<SCORED>(o, ai, si));
        }
    }
    // WT: the stores' base is the first octet of the lane's tile, shared by
    // every lane (o0 - threadIdx.x), so the per-lane offsets stay small
    const int64_t ob = WT ? uniform64(o0 - (int64_t)threadIdx.x) : 0;
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const f32x4 e = div4(ev[c], divisor), o = div4(od[c], divisor);
        const int64_t oc = o0 + (int64_t)c * B;
        // out (fp32) and outb (RNE bf16) are each optional, one of them given
        // (ABI 5): a step that exchanges only the bf16 copy stores no fp32
        if (out) {
            const u32x4 lo = __builtin_bit_cast(u32x4, f32x4{e.x, o.x, e.y, o.y});
            const u32x4 hi = __builtin_bit_cast(u32x4, f32x4{e.z, o.z, e.w, o.w});
            if constexpr (WT) {
                const __amdgpu_buffer_rsrc_t r = wt_rsrc(out + 8 * ob);
                st16_wt<WT>(r, (int)(32 * (oc - ob)), lo);
                st16_wt<WT>(r, (int)(32 * (oc - ob)) + 16, hi);
            } else {
                f32x4* o4 = reinterpret_cast<f32x4*>(out) + 2 * oc;
                st16(o4, lo);
                st16(o4 + 1, hi);
            }
        }
        if (outb) {
            u32x4 b;
            b.x = (uint32_t)f2bf_rne(e.x) | ((uint32_t)f2bf_rne(o.x) << 16);
            b.y = (uint32_t)f2bf_rne(e.y) | ((uint32_t)f2bf_rne(o.y) << 16);
            b.z = (uint32_t)f2bf_rne(e.z) | ((uint32_t)f2bf_rne(o.z) << 16);
            b.w = (uint32_t)f2bf_rne(e.w) | ((uint32_t)f2bf_rne(o.w) << 16);
            if constexpr (WT) st16_wt<WT>(wt_rsrc(outb + 8 * ob), (int)(16 * (oc - ob)), b);
            else st16(reinterpret_cast<u32x4*>(outb) + oc, b);
        }
    }
}

// bf16 rows: a lane owns C octets (8 columns, one 16-byte load per row each)
// spaced kBlock apart; the trailing P%8 columns go to the lane with o0 == P/8.
template <int U, int C, bool SCORED, int B = kBlock, int WT = 0>
__device__ __forceinline__ void bf16_tile(int64_t bid, const uint16_t* __restrict__ X, int64_t N, int64_t P,
                                          int64_t ldx, const float* __restrict__ a, const float* __restrict__ s,
                                          float divisor, float* __restrict__ out, uint16_t* __restrict__ outb) {
    const int64_t no = P >> 3;  // full octets
    const int64_t ldo = ldx >> 3;
    const int64_t o0 = bid * (B * C) + threadIdx.x;
    const u32x4* X8 = reinterpret_cast<const u32x4*>(X);
    if (o0 + (int64_t)(C - 1) * B < no) {
        fold_octets<U, C, SCORED, B, WT>(X8 + o0, ldo, N, a, s, divisor, out, outb, o0);
        return;
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int64_t o = o0 + (int64_t)c * B;
        if (o < no) fold_octets<U, 1, SCORED, B, WT>(X8 + o, ldo, N, a, s, divisor, out, outb, o);
    }
    const int64_t tb = no / (B * C), tl = (no % (B * C)) % B;
    if ((P & 7) && bid == tb && (int64_t)threadIdx.x == tl) {
        for (int64_t col = no * 8; col < P; ++col) {
            float acc = term1<SCORED>(bf2f(X[col]), a[0], SCORED ? s[0] : 1.0f);
            for (int64_t i = 1; i < N; ++i)
                acc = acc + term1<SCORED>(bf2f(X[i * ldx + col]), a[i], SCORED ? s[i] : 1.0f);
            acc = acc / divisor;
            if (out) out[col] = acc;
            if (outb) outb[col] = f2bf_rne(acc);
        }
        // WT: these few plain stores are written back before the block publishes
        wt_tail_release<WT>();
    }
}

template <int U, int C, bool SCORED>
__global__ __launch_bounds__(kBlock) void k_fedavg_bf16_v8(
    const uint16_t* __restrict__ X, int64_t N, int64_t P, int64_t ldx,
    const float* __restrict__ a, const float* __restrict__ s, float divisor,
    float* __restrict__ out, uint16_t* __restrict__ outb) {
    bf16_tile<U, C, SCORED>(blockIdx.x, X, N, P, ldx, a, s, divisor, out, outb);
}

// grid-stride over octet tiles, as k_fold_f32_gs
template <int U, int C, bool SCORED>
__global__ __launch_bounds__(kBlock) void k_fedavg_bf16_gs(
    const uint16_t* __restrict__ X, int64_t N, int64_t P, int64_t ldx,
    const float* __restrict__ a, const float* __restrict__ s, float divisor,
    float* __restrict__ out, uint16_t* __restrict__ outb, int64_t ntiles) {
    for (int64_t bid = blockIdx.x; bid < ntiles; bid += gridDim.x)
        bf16_tile<U, C, SCORED>(bid, X, N, P, ldx, a, s, divisor, out, outb);
}

// ---------------------------------------------------------------------------
// One launch per exchange step (round 4, fa_fedavg_*_rounds).  Per-round
// dynamic launches pay a tile-time of tail per round (the last tiles of a
// round run on a few blocks while the others idle; measured: 256 x the C4
// rank's slots, 1.12 ms per step with 8 KiB dynamic tiles against 0.96 static,
// profiles/r04_dyn/), and the overlapped exchange needs the rounds' results in
// order, not each round's fold in its own kernel.  So one launch folds every
// round's slot, taking the tiles of round 0, then round 1, ... from one
// counter: a round's last tiles overlap the next round's first ones (no tail
// until the step's end), slowed blocks fold fewer tiles, and when a round's
// last tile is done the block that finished it raises the round's flag to
// the launch's epoch.  The exchange of round k is issued behind
// k_wait_round on another stream (a one-lane kernel that polls the flag and
// returns), so it starts mid-launch, as soon as round k is complete.
//   Publication is per block and round, not per tile: when a block's next
//   tile belongs to a later round, every wave waits for its stores, and one
//   lane writes the XCD's L2 back (agent-scope release), waits for that, and
//   adds the block's tile count of the round to the round's counter; the add
//   that completes the round stores the epoch into the round's flag (an
//   agent-scope atomic).  A release per tile cost 0.3-0.6 ms per C4 rank step
//   (profiles/r04_step/).  The waiter polls the flag with relaxed agent-scope
//   loads; the exchange kernels behind it read the results after their own
//   launch acquire.  A waiter gives up after `max_ticks` of the device wall
//   clock (never an endless spin), counting a timeout in the signal words.
// ---------------------------------------------------------------------------
constexpr int kMaxRounds = 8, kMaxSegs = 3 * kMaxRounds;
// The launch's tiles, in column order: segment g covers local columns
// [col0[g], col0[g] + width[g]) of round round[g] with wide tiles (small[g] = 0)
// or narrow ones (1); its tiles are [seg_end[g-1], seg_end[g]) of the launch.
// Tiles [0, static_tiles) are dealt statically -- block b folds b, b + G, ...
// (G blocks: every block's share of every round, rounds in order, blocks in
// lock-step over adjacent tiles as in the grid-stride forms) -- and the rest,
// the step's last columns in narrow tiles, go to whichever block asks the
// counter next.  A block that lags (it shares its CU with other kernels)
// finishes its static share late and takes few or none of the dynamic tiles.
struct StepTable {
    int64_t seg_end[kMaxSegs];
    int64_t col0[kMaxSegs];
    int64_t ocol0[kMaxSegs];  // the output column of segment g's first column: col0[g], or where the caller
                              // maps its round (out_offsets: a rank's slots straight into the gathered model)
    int64_t width[kMaxSegs];
    int32_t round[kMaxSegs];
    int32_t small[kMaxSegs];
    int64_t round_tiles[kMaxRounds];
    int64_t static_tiles;
    int32_t segs;
    int32_t rounds;
    int32_t sys;    // publish the rounds at system scope: other GPUs read them (fa_peers, the peer exchange)
    int32_t wt;     // the tiles' output stores are write-through: no per-block L2 write-back
    int32_t sysfence;  // sys with sc1 tile stores: a system release fence per block and round (round 5's
                       // publication; bench-library A/B only: the product's sys launches store sc0 sc1)
    int64_t stride[kMaxSegs];  // balanced rounds (step_tiles_bal): static segment g dealt over stride[g] blocks
};
// signal words: [0] next dynamic tile, [1] blocks done, [2, 2+R) tiles done per round,
// [2+R, 2+2R) round flags (the epoch of the launch that completed the round), [2+2R] waits timed out
constexpr int kSigDone = 2, kSigFlag = 2 + kMaxRounds, kSigTimeout = 2 + 2 * kMaxRounds, kSigWords = 3 + 2 * kMaxRounds;
constexpr int kStatusWords = kMaxRounds;  // a timeout record per round

// A block leaves round k (its tiles come in round order): publish its cnt
// tiles of the round once.  Every storing wave waits for its stores
// (vmcnt(0)), a barrier, then one lane counts the block's tiles with an
// agent-scope add; the block whose add completes the round raises the round's
// flag with a release store (after an acquire fence, one per round: it cost
// nothing measurable, profiles/r05_step/, where an acq_rel add in every block
// cost ~4 %).
// Which stores make that a hand-off:
//   !T.wt: plain tile stores, so the lane first writes the XCD's L2 back
//     (agent release fence) -- MI355X_MICROARCH.md's first valid producer
//     form, ordered by the memory model (every block's release, the last
//     block's acquire);
//   T.wt (the step kernels, round 5): the tiles are stored write-through
//     (sc1; the tail's few plain stores behind their own release,
//     wt_tail_release), so once every storing wave's vmcnt(0) wait has
//     returned the bytes are in memory and the block adds with no fence --
//     the per-block release cost 3.5 % of the C4 rank step
//     (tools/step_probe.hip).  The non-completing blocks' relaxed adds carry
//     no release, so this guarantee is ISA-level (MI355X_MICROARCH.md, "Valid
//     forms": sc1 stores, vmcnt(0), a barrier, one lane's agent-scope add;
//     the consumers load behind a kernel boundary), not the HIP memory
//     model's;
//   T.sys (a peer exchange's state, read by other GPUs' copy engines over
//     xGMI): the same at system scope -- the tiles stored sc0 sc1 (system
//     coherent, kWtSystem) and the flag's release store system-scope; round
//     5 kept a system release fence per block instead (T.sysfence, sc1 tile
//     stores: now only the bench library's A/B, fa_bench_rounds_set_sys).
// Block-uniform arguments (every thread calls it).
__device__ __forceinline__ void step_publish(const StepTable& T, unsigned int* sig, unsigned int epoch, int k,
                                             unsigned int cnt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        if (T.sysfence) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        else if (!T.wt) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned int nk = (unsigned int)T.round_tiles[k];
        if (__hip_atomic_fetch_add(&sig[kSigDone + k], cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + cnt ==
            nk) {  // the round's last tiles
            __hip_atomic_store(&sig[kSigDone + k], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (T.sys) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
                __hip_atomic_store(&sig[kSigFlag + k], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            } else {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                __hip_atomic_store(&sig[kSigFlag + k], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

// The last block out resets the dynamic-tile counters for the next launch.
__device__ __forceinline__ void step_reset(unsigned int* sig) {
    if (threadIdx.x == 0) {
        if (atomicAdd(&sig[1], 1u) == gridDim.x - 1) {
            atomicExch(&sig[0], 0u);
            atomicExch(&sig[1], 0u);
        }
    }
}

// Balanced rounds (round 5): every static segment -- a round's wide tiles --
// is dealt over its own stride[g] blocks, the fewest that still fold it in
// the same number of passes (block b < stride[g] folds tiles b, b + stride[g],
// ...), as the per-round band launches' balanced grids do; the blocks past the
// stride go straight on to the next round.  So no round ends in a partial
// pass, without a launch boundary between rounds.  Then the dynamic pool (the
// last round's last columns), a tile fetched ahead as in step_tiles.  The
// static segments are wide tiles and the pool's narrow (build_step_table), so
// each call site inlines one tile body.
template <class Wide, class Narrow>
__device__ __forceinline__ void step_tiles_bal(const StepTable& T, unsigned int* sig, unsigned int epoch,
                                               Wide wide, Narrow narrow) {
    __shared__ unsigned int nxt[2];
    const int64_t b = blockIdx.x;
    const int64_t ntiles = T.seg_end[T.segs - 1];
    const int64_t Ts = T.static_tiles;
    int k = -1;
    unsigned int cnt = 0;
    int g = 0;
    for (; g < T.segs; ++g) {
        const int64_t lo = g ? T.seg_end[g - 1] : 0;
        if (lo >= Ts) break;
        if (T.round[g] != k) {
            if (k >= 0 && cnt) step_publish(T, sig, epoch, k, cnt);
            k = T.round[g];
            cnt = 0;
        }
        const int64_t n = T.seg_end[g] - lo, S = T.stride[g];
        for (int64_t i = b; b < S && i < n; i += S) {
            wide(g, i);
            ++cnt;
        }
    }
    if (Ts < ntiles) {  // the dynamic pool
        int p = 0;
        if (threadIdx.x == 0) nxt[p] = atomicAdd(&sig[0], 1u);
        __syncthreads();
        int64_t t = Ts + nxt[p];
        p ^= 1;
        while (t < ntiles) {
            while (g + 1 < T.segs && t >= T.seg_end[g]) ++g;
            if (T.round[g] != k) {
                if (k >= 0 && cnt) step_publish(T, sig, epoch, k, cnt);
                k = T.round[g];
                cnt = 0;
            }
            unsigned int nx = 0;
            if (threadIdx.x == 0) nx = atomicAdd(&sig[0], 1u);  // fetched a tile ahead
            narrow(g, t - (g ? T.seg_end[g - 1] : 0));
            ++cnt;
            if (threadIdx.x == 0) nxt[p] = nx;
            __syncthreads();
            t = Ts + nxt[p];
            p ^= 1;
        }
    }
    if (k >= 0 && cnt) step_publish(T, sig, epoch, k, cnt);
    step_reset(sig);
}

template <class Tile>
__device__ __forceinline__ void step_tiles(const StepTable& T, unsigned int* sig, unsigned int epoch, Tile tile) {
    __shared__ unsigned int nxt[2];
    const int64_t ntiles = T.seg_end[T.segs - 1];
    const int64_t Ts = T.static_tiles;
    const int64_t G = gridDim.x;
    int p = 0;
    int64_t t = blockIdx.x;
    if (t >= Ts) {  // no static tile for this block: its first tile from the counter
        if (threadIdx.x == 0) nxt[p] = atomicAdd(&sig[0], 1u);
        __syncthreads();
        t = Ts + nxt[p];
        p ^= 1;
    }
    int g = 0;
    while (g + 1 < T.segs && t >= T.seg_end[g]) ++g;
    int k = T.round[g];
    unsigned int cnt = 0;  // this block's tiles of round k so far
    while (t < ntiles) {
        const bool dyn_next = t + G >= Ts;  // the next tile comes from the counter
        unsigned int nx = 0;
        if (dyn_next && threadIdx.x == 0) nx = atomicAdd(&sig[0], 1u);  // fetched a tile ahead
        tile(g, t - (g ? T.seg_end[g - 1] : 0));
        ++cnt;
        int64_t tn = t + G;
        if (dyn_next) {
            if (threadIdx.x == 0) nxt[p] = nx;
            __syncthreads();
            tn = Ts + nxt[p];
            p ^= 1;
        }
        int gn = g;
        while (gn < T.segs && tn >= T.seg_end[gn]) ++gn;  // T.segs: no tile left
        const int kn = gn < T.segs ? T.round[gn] : kMaxRounds;
        if (kn != k) {
            step_publish(T, sig, epoch, k, cnt);
            cnt = 0;
            k = kn;
        }
        t = tn;
        g = gn < T.segs ? gn : g;
    }
    step_reset(sig);
}

// wide tiles: UB rows ahead x CB octets (quads) per lane; narrow: US x CS;
// BAL: balanced rounds (step_tiles_bal).  One schedule per instantiation: both
// inlined into one kernel made it ~4 % slower (code size: the unrolled tile
// body four times over; profiles/r05_step/)
template <int UB, int CB, int US, int CS, bool SCORED, int B, bool BAL = false, int WTM = kWtAgent>
__global__ __launch_bounds__(B) void k_fedavg_bf16_step(
    const uint16_t* __restrict__ X, int64_t N, int64_t ldx, const float* __restrict__ a,
    const float* __restrict__ s, float divisor, float* __restrict__ out, uint16_t* __restrict__ outb, StepTable T,
    unsigned int* sig, unsigned int epoch) {
    auto wide = [&](int g, int64_t bid) {
        const int64_t c0 = T.col0[g], o0 = T.ocol0[g];
        bf16_tile<UB, CB, SCORED, B, WTM>(bid, X + c0, N, T.width[g], ldx, a, s, divisor, out ? out + o0 : nullptr,
                                          outb ? outb + o0 : nullptr);
    };
    auto narrow = [&](int g, int64_t bid) {
        const int64_t c0 = T.col0[g], o0 = T.ocol0[g];
        bf16_tile<US, CS, SCORED, B, WTM>(bid, X + c0, N, T.width[g], ldx, a, s, divisor, out ? out + o0 : nullptr,
                                          outb ? outb + o0 : nullptr);
    };
    if constexpr (BAL) {
        step_tiles_bal(T, sig, epoch, wide, narrow);
    } else {
        step_tiles(T, sig, epoch, [&](int g, int64_t bid) {
            if (T.small[g]) narrow(g, bid);
            else wide(g, bid);
        });
    }
}

template <int UB, int CB, int US, int CS, bool SCORED, int B, bool BAL = false, int WTM = kWtAgent>
__global__ __launch_bounds__(B) void k_fold_f32_step(
    const float* __restrict__ X, int64_t N, int64_t ldx, const float* __restrict__ a, const float* __restrict__ s,
    float divisor, float* __restrict__ out, StepTable T, unsigned int* sig, unsigned int epoch) {
    auto wide = [&](int g, int64_t bid) {
        const int64_t c0 = T.col0[g];
        fold_tile<UB, CB, true, SCORED, false, true, true, B, WTM>(bid, X + c0, N, T.width[g], ldx, a, s, nullptr,
                                                                   divisor, out + T.ocol0[g]);
    };
    auto narrow = [&](int g, int64_t bid) {
        const int64_t c0 = T.col0[g];
        fold_tile<US, CS, true, SCORED, false, true, true, B, WTM>(bid, X + c0, N, T.width[g], ldx, a, s, nullptr,
                                                                   divisor, out + T.ocol0[g]);
    };
    if constexpr (BAL) {
        step_tiles_bal(T, sig, epoch, wide, narrow);
    } else {
        step_tiles(T, sig, epoch, [&](int g, int64_t bid) {
            if (T.small[g]) narrow(g, bid);
            else wide(g, bid);
        });
    }
}

// Poll round flag `flag` until it reaches `epoch` (wrapping compare), then
// return: the kernel a stream runs before an exchange that needs the round.
// A waiter that sees no completion within max_ticks of the device wall clock
// returns anyway (no launch can hang a stream), counts the timeout in device
// memory and stores the launch's epoch into `status`, a word of page-locked
// host memory mapped into the device: the host reads it without a HIP call
// once the wait has run, and the caller raises instead of handing on an
// exchange that read an unfinished round (ShardedAggregator, fa_rounds_check).
__global__ __launch_bounds__(64) void k_wait_round(const unsigned int* flag, unsigned int epoch, unsigned int* timeouts,
                                                   unsigned int* status, long long max_ticks) {
    if (threadIdx.x != 0) return;
    const long long t0 = wall_clock64();
    // relaxed agent-scope (L2-served) polls: the exchange kernels that follow
    // this one read the round's results after their own launch acquire
    while ((int)(__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - epoch) < 0) {
        if (wall_clock64() - t0 > max_ticks) {
            atomicAdd(timeouts, 1u);
            if (status) __hip_atomic_store(status, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        __builtin_amdgcn_s_sleep(4);
    }
}

template <bool SCORED>
__global__ __launch_bounds__(kBlock) void k_fedavg_bf16_scalar(
    const uint16_t* __restrict__ X, int64_t N, int64_t P, int64_t ldx,
    const float* __restrict__ a, const float* __restrict__ s, float divisor,
    float* __restrict__ out, uint16_t* __restrict__ outb) {
    const int64_t c = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (c >= P) return;
    float acc = term1<SCORED>(bf2f(X[c]), a[0], SCORED ? s[0] : 1.0f);
    for (int64_t i = 1; i < N; ++i)
        acc = acc + term1<SCORED>(bf2f(X[i * ldx + c]), a[i], SCORED ? s[i] : 1.0f);
    acc = acc / divisor;
    if (out) out[c] = acc;
    if (outb) outb[c] = f2bf_rne(acc);
}

// ---------------------------------------------------------------------------
// float64 and integer folds: one column per lane, coalesced 8-byte loads.
// ---------------------------------------------------------------------------
typedef double f64x2 __attribute__((ext_vector_type(2)));

// float64: a lane owns 2 columns (one 16-byte load per row), U rows ahead;
// the odd last column (P % 2) goes to the lane with q == P/2.
template <int U, bool SCORED>
__global__ __launch_bounds__(kBlock) void k_fedavg_f64_v2(
    const double* __restrict__ X, int64_t N, int64_t P, int64_t ldx,
    const double* __restrict__ a, const double* __restrict__ s, double divisor,
    double* __restrict__ out) {
    const int64_t nq = P >> 1, ldq = ldx >> 1;
    const int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (q < nq) {
        const f64x2* p = reinterpret_cast<const f64x2*>(X) + q;
        f64x2 acc = __builtin_nontemporal_load(p) * a[0];
        if constexpr (SCORED) acc = acc * s[0];
        int64_t i = 1;
        for (; i + U <= N; i += U) {
            f64x2 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(p + (i + u) * ldq);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                f64x2 t = v[u] * a[i + u];
                if constexpr (SCORED) t = t * s[i + u];
                acc = acc + t;
            }
        }
        for (; i < N; ++i) {
            f64x2 t = __builtin_nontemporal_load(p + i * ldq) * a[i];
            if constexpr (SCORED) t = t * s[i];
            acc = acc + t;
        }
        __builtin_nontemporal_store(acc / divisor, reinterpret_cast<f64x2*>(out) + q);
    } else if (q == nq && (P & 1)) {
        const int64_t c = P - 1;
        double acc = X[c] * a[0];
        if constexpr (SCORED) acc = acc * s[0];
        for (int64_t i = 1; i < N; ++i) {
            double t = X[i * ldx + c] * a[i];
            if constexpr (SCORED) t = t * s[i];
            acc = acc + t;
        }
        out[c] = acc / divisor;
    }
}

// float64, one column per lane, any alignment / stride.
template <bool SCORED>
__global__ __launch_bounds__(kBlock) void k_fedavg_f64(
    const double* __restrict__ X, int64_t N, int64_t P, int64_t ldx,
    const double* __restrict__ a, const double* __restrict__ s, double divisor,
    double* __restrict__ out) {
    const int64_t c = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (c >= P) return;
    double acc = X[c] * a[0];
    if constexpr (SCORED) acc = acc * s[0];
#pragma unroll 8
    for (int64_t i = 1; i < N; ++i) {
        double t = X[i * ldx + c] * a[i];
        if constexpr (SCORED) t = t * s[i];
        acc = acc + t;
    }
    out[c] = acc / divisor;
}

// numpy integer semantics: product and fold in the input dtype with
// two's-complement wrap (computed unsigned to avoid C++ UB), then
// true_divide -> float64(acc) / float64(total).
template <typename T, typename UT>
__global__ __launch_bounds__(kBlock) void k_fedavg_int(
    const T* __restrict__ X, int64_t N, int64_t P, int64_t ldx,
    const int64_t* __restrict__ a, double divisor, double* __restrict__ out) {
    const int64_t c = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (c >= P) return;
    UT acc = 0;
    for (int64_t i = 0; i < N; ++i) {
        UT t = (UT)X[i * ldx + c] * (UT)(T)a[i];
        acc = (i == 0) ? t : (UT)(acc + t);
    }
    out[c] = (double)(T)acc / divisor;
}

// ---------------------------------------------------------------------------
// host-side dispatch
// ---------------------------------------------------------------------------
inline dim3 grid_for(int64_t lanes) { return dim3((unsigned)((lanes + kBlock - 1) / kBlock)); }

// The output a bf16 fold's pointer checks look at: out_f32 and out_bf16 are
// each optional (ABI 5), one of them required.
inline const void* bf16_any_out(const float* out_f32, const uint16_t* out_bf16) {
    return out_f32 ? static_cast<const void*>(out_f32) : static_cast<const void*>(out_bf16);
}

int check_common(int64_t N, int64_t P, int64_t ldx, const void* X, const void* a, const void* out) {
    if (N < 0 || P < 0) return fail(FA_ERR_ARG, "negative size (N=%lld, P=%lld)", (long long)N, (long long)P);
    if (N == 0) return fail(FA_ERR_NO_CLIENTS, "no client results to aggregate (N == 0)");
    if (ldx < P) return fail(FA_ERR_SHAPE, "row pitch ldx=%lld < P=%lld", (long long)ldx, (long long)P);
    if (P > 0 && (!X || !a || !out)) return fail(FA_ERR_ARG, "null X/a/out pointer");
    if ((P + 4 * (int64_t)kBlock) / (4 * (int64_t)kBlock) > (int64_t)0x7FFFFFFF)
        return fail(FA_ERR_ARG, "P too large for one launch");
    return FA_OK;
}

// Make the device that owns `stream` current for the duration of one C-ABI
// call, and restore the caller's device afterwards.  Every allocation (the
// host-factor ring's device slots), every CU-count lookup (the fold policy) and
// every launch then belongs to the stream's GPU, whatever device the calling
// thread has current: a fold of tensors on cuda:1 issued from a thread whose
// current device is 0 reads its factors from cuda:1's memory and is picked for
// cuda:1's CU count.  A NULL stream means the caller's current device.
struct StreamDevice {
    int prev = -1;
    explicit StreamDevice(void* stream) {
        if (!stream) return;
        int cur = 0;
        hipDevice_t d = 0;
        if (hipGetDevice(&cur) != hipSuccess || hipStreamGetDevice((hipStream_t)stream, &d) != hipSuccess) {
            (void)hipGetLastError();
            return;
        }
        if ((int)d != cur && hipSetDevice((int)d) == hipSuccess) prev = cur;
    }
    ~StreamDevice() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    StreamDevice(const StreamDevice&) = delete;
    StreamDevice& operator=(const StreamDevice&) = delete;
};

// Compute units of the current device (cached per device).
int cu_count() {
    static thread_local int cache[16] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) dev = 0;
    if (cache[dev] > 0) return cache[dev];
    int cus = 256;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
    cache[dev] = cus;
    return cus;
}

// The "auto" fp32 fold, from variant sweeps (interleaved, shuffled order) over
// model sizes x client counts on MI355X (profiles/r01_sweep_shapes.log,
// profiles/r01_sweep_balanced.log).  tiles4 = 16 KiB column tiles (4 quads per lane):
//   P < 32K params                     LDS-staged, 2 waves, 32-row chunks of 16-quad tiles,
//                                      four chunks in flight per block
//   32K <= P < 80K                     LDS-staged, two chunks in flight: 4 waves over 24- or
//                                      40-quad tiles, or 2 waves over 16-quad tiles where
//                                      32-quad ones would fill the CUs best (pick_lds_tile)
//   80K <= P < 256K                    LDS-staged, 2 waves, two 16-row chunks of 32-quad tiles
//   N >= 256, tiles4 < 0.7 x CUs       LDS-staged, 8 waves, 64-row chunks, 32-quad tiles
//   48 <= N < 112, tiles4 < 3/5 CUs    one lane per column (k_fold_f32_scalar); 48 <= N < 80:
//                                      up to 0.9 x CUs
//   tiles4 < 0.7 x CUs (0.9 x CUs for  one block per 4 KiB tile, 4 rows x 1 quad (4x the
//     N < 112, 1 x CUs for N < 64)     blocks of the grid-stride fold)
//   N >= 112, 0.7-0.9 x CUs            grid-stride, balanced passes, 8 rows x 2 quads
//   N < 24, tiles4 >= CUs              one block per 16 KiB tile, 8 rows x 4 quads
//   CUs < tiles4 < 2 x CUs             grid-stride, balanced passes, 8 rows x 2 quads
//   otherwise (C2, C3, C5, ...)        grid-stride, balanced passes, 8 rows x 4 quads,
//                                      in column bands of <= 3 passes x CUs tiles
// with non-temporal output stores (plain ones in the 4 KiB tile and column forms).
enum class F32Pick { kLdsW2T16, kLdsW2T16D4, kLdsW2T16D2, kLdsW2T32, kLdsW4T24, kLdsW4T40, kLdsW8, kColumn, kTileC1, kTileC4,
                     kTileC4Plain, kGsBalC2, kGsBalC4,
                     // forms only the tuner (below) chooses: plain one-shot folds (no accumulator in, divide)
                     kGsBands6, kGs1C4, kTileU8C2, kEvenU4C4, kLdsQfW4T32 };
constexpr int kNumF32Picks = (int)F32Pick::kLdsQfW4T32 + 1;
inline bool f32_tuning_only(F32Pick p) { return (int)p >= (int)F32Pick::kGsBands6; }
inline const char* f32_pick_name(F32Pick p) {
    switch (p) {
        case F32Pick::kLdsW2T16: return "lds_w2_t16";
        case F32Pick::kLdsW2T16D4: return "lds_w2_t16_d4";
        case F32Pick::kLdsW2T16D2: return "lds_w2_t16_d2";
        case F32Pick::kLdsW2T32: return "lds_w2_t32";
        case F32Pick::kLdsW4T24: return "lds_w4_t24";
        case F32Pick::kLdsW4T40: return "lds_w4_t40";
        case F32Pick::kLdsW8: return "lds_w8_t32";
        case F32Pick::kColumn: return "column";
        case F32Pick::kTileC1: return "tile_4k";
        case F32Pick::kTileC4: return "tile_16k";
        case F32Pick::kTileC4Plain: return "tile_16k_ps";
        case F32Pick::kGsBalC2: return "gs_bal_8k";
        case F32Pick::kGsBalC4: return "gs_bands_16k";
        case F32Pick::kGsBands6: return "gs_bands6_16k";
        case F32Pick::kGs1C4: return "gs1_16k";
        case F32Pick::kTileU8C2: return "tile_8k";
        case F32Pick::kEvenU4C4: return "even_u4c4";
        case F32Pick::kLdsQfW4T32: return "lds_qf_w4_t32";
    }
    return "";
}
// bf16 fold forms (the vector path: 16-B aligned rows, ldx % 8 == 0).
enum class Bf16Form { kV8U2C8, kV8U4C4, kV8U8C2, kV8U8C1, kBandsU8C4, kBandsU8C2, kBandsU2C8, kBandsU4C4,
                      kBandsU16C2, kGsBalU8C2, kGs1U8C4 };
constexpr int kNumBf16Forms = (int)Bf16Form::kGs1U8C4 + 1;
inline const char* bf16_form_name(Bf16Form f) {
    switch (f) {
        case Bf16Form::kV8U2C8: return "bf16_tile_u2c8";
        case Bf16Form::kV8U4C4: return "bf16_tile_u4c4";
        case Bf16Form::kV8U8C2: return "bf16_tile_u8c2";
        case Bf16Form::kV8U8C1: return "bf16_tile_u8c1";
        case Bf16Form::kBandsU8C4: return "bf16_bands4_u8c4";
        case Bf16Form::kBandsU8C2: return "bf16_bands4_u8c2";
        case Bf16Form::kBandsU2C8: return "bf16_bands2_u2c8";
        case Bf16Form::kBandsU4C4: return "bf16_bands4_u4c4";
        case Bf16Form::kBandsU16C2: return "bf16_bands4_u16c2";
        case Bf16Form::kGsBalU8C2: return "bf16_gsbal_u8c2";
        case Bf16Form::kGs1U8C4: return "bf16_gs1_u8c4";
    }
    return "";
}

// Column tile of the LDS fold for 32K-256K params: the launch is ~2-8 blocks
// per CU, so how evenly the blocks fill the CUs decides the time (a scan over
// P at 1024 clients: 768 blocks of 32 quads ran at 7.17 TB/s, 526 blocks at
// 5.9).  Of 24-, 32- and 40-quad tiles take the one whose block count wastes
// the least of the last round of CUs (ties: 32).
inline F32Pick pick_lds_tile(int64_t P, int64_t cus) {
    const int64_t nq = P >> 2, tail = (P & 3) ? 1 : 0;
    auto waste = [&](int64_t tq) {
        const int64_t b = (nq + tq - 1) / tq + tail;
        return (double)(((b + cus - 1) / cus) * cus) / (double)b;
    };
    const double w24 = waste(24), w32 = waste(32), w40 = waste(40);
    // where 32-quad tiles fill the CUs best, two-wave blocks over 16-quad tiles
    // (twice the blocks, same waves per CU) instead: the 4-wave 32-quad form
    // ran 10-60 % behind at 256-1024 x 32K/57K/65K (profiles/r02_lds/range_32k_256k/)
    if (w32 <= w24 && w32 <= w40) return F32Pick::kLdsW2T16D2;
    return w24 <= w40 ? F32Pick::kLdsW4T24 : F32Pick::kLdsW4T40;
}

inline F32Pick pick_f32(int64_t N, int64_t P, int64_t cus_override = 0) {
    const int64_t nq = P >> 2, cus = cus_override > 0 ? cus_override : cu_count();
    // up to 32K params (32,768 included: 1.23x faster than the CU-fill pick at
    // 1024 clients, profiles/r02_lds/range_32k_80k_after/)
    // (round 3: the terms formed by the loaders; six chunks in flight up to
    // 16K params, four above: 1024 x 32K 22.6 against 24.4 us with six,
    // profiles/r03_premul/check_sweep.log)
    if (nq <= (1 << 13)) return nq <= (1 << 12) ? F32Pick::kLdsW2T16 : F32Pick::kLdsW2T16D4;
    // 80K-256K params: two-wave blocks over 32-quad tiles, 16-row chunks: best
    // or within 5 % at 100-1024 clients x 82K-246K, where the 4-wave CU-fill
    // pick lost up to 24 % (131,136 params; profiles/r02_lds/range_32k_256k/)
    if (nq >= 20480 && nq < (1 << 16)) return F32Pick::kLdsW2T32;
    if (nq < (1 << 16)) return pick_lds_tile(P, cus);
    const int64_t tiles4 = (((P + 3) >> 2) + 4 * kBlock - 1) / (4 * kBlock);
    // fewer 16 KiB column tiles than ~0.7 (0.9) x CUs: the grid-stride fold
    // would leave CUs idle; the picks below spread the columns over more blocks
    const bool under = 10 * tiles4 < 7 * cus, mid = 10 * tiles4 < 9 * cus;
    if (N >= 256 && under) return F32Pick::kLdsW8;
    // 48+ clients at 0.7-1 tiles per CU: one block per 16 KiB tile, 8 rows x 4
    // quads ahead, plain stores (round-3 sweep of 15 forms over 42 shapes,
    // profiles/r03_even/: best or within 2 % at 740K-1M params for 64-1024
    // clients, where the 4 KiB tile and 8 KiB balanced picks were 5-20 %
    // behind; the even split over all CUs, k_fold_f32_even, was 10-60 % behind)
    if (N >= 48 && !under && tiles4 < cus) return F32Pick::kTileC4Plain;
    // Between 0.7 and 0.9 tiles per CU every form swings by up to 25 % with the
    // model size (1024 x 700K-1M in 10-40K steps, profiles/r02_small_n/pitch_scan*;
    // extra row padding changes nothing, pitch_pad/);
    // the picks there minimise the mean and worst ratio to the best form over
    // 32 measured shapes (grid_v4, grid_v5, pitch_scan2).
    // One lane per column (4x the waves of the tile form): 48-111 clients below
    // 3/5 of a tile per CU (4-9 % faster at 50-100 x 300K-582K), 48-79 clients
    // up to 0.9 tiles per CU (64 x 300K-860K: best or tied at every size).
    if (N >= 48 && N < 112 && (5 * tiles4 < 3 * cus || (N < 80 && mid))) return F32Pick::kColumn;
    // One block per 4 KiB tile: each block's rows are short with few clients,
    // so ~one grid-stride block per CU keeps too few bytes in flight (8-30 %
    // faster at 10-128 x 582K and 10-32 x 1M, profiles/r02_small_n/).
    if (under || (N < 112 && mid) || (N < 64 && tiles4 < cus)) return F32Pick::kTileC1;
    // 112+ clients at 0.7-0.9 tiles per CU: balanced passes over 8 KiB tiles
    // (within 8 % of the best form at every measured size)
    if (mid) return F32Pick::kGsBalC2;
    // under 24 clients above one tile per CU: one block per 16 KiB tile (7-10 %
    // at 10 x 4M-10M)
    if (N < 24 && tiles4 >= cus) return F32Pick::kTileC4;
    if (tiles4 > cus && tiles4 < 2 * cus) return F32Pick::kGsBalC2;
    return F32Pick::kGsBalC4;
}

// bf16 "auto": octets per lane from the client count.  Sweeps on MI355X
//  put the optimum near 8 MB per block (rows x C x 4 KiB):
// 256 rows -> C=8 (u2c8), 512 -> C=4, 1024 -> C=2 (u8c2); C shrinks further
// while the launch would have fewer than ~1000 blocks.
inline int pick_octets(int64_t N, int64_t P) {
    int c = N <= 384 ? 8 : (N <= 768 ? 4 : 2);
    while (c > 1 && (P >> 3) / ((int64_t)c * kBlock) < 1000) c >>= 1;
    return c;
}

// Grid-stride fold: grid = min(tiles, per_cu x CUs); per_cu < 0 = balanced passes.
template <int U, int C, bool NT, bool SC, bool ACC, bool FIN, bool NTS, int B>
void launch_gs(hipStream_t st, int per_cu, const float* X, int64_t N, int64_t P, int64_t ldx, const float* a,
               const float* s, const float* acc_in, float d, float* out) {
    const int64_t per_block = (int64_t)B * C, units = (P >> 2) + ((P & 3) ? 1 : 0);
    const int64_t tiles = (units + per_block - 1) / per_block;  // incl. the column-tail lane
    // per_cu >= 1000: a fixed block count (per_cu - 1000), balanced passes (sweeps only)
    int64_t grid = per_cu >= 1000 ? per_cu - 1000 : (int64_t)(per_cu > 0 ? per_cu : -per_cu) * cu_count();
    if (grid > tiles) grid = tiles;
    if (per_cu < 0 || per_cu >= 1000) {
        // balanced passes: the fewest blocks that still finish in the same
        // number of passes, so the last pass is (nearly) full instead of
        // leaving up to a whole pass of CUs idle
        const int64_t passes = (tiles + grid - 1) / grid;
        grid = (tiles + passes - 1) / passes;
    }
    hipLaunchKernelGGL((k_fold_f32_gs<U, C, NT, SC, ACC, FIN, NTS, B>), dim3((unsigned)grid), dim3(B), 0, st, X,
                       N, P, ldx, a, s, acc_in, d, out, tiles);
}

// One block per C*kBlock-quad tile (the column-tail lane's tile included),
// every (scored, accumulate, finalize) combination.
template <int U, int C, bool NTS>
int launch_tile_flags(hipStream_t st, bool sc, bool acc, bool fin, const float* X, int64_t N, int64_t P,
                      int64_t ldx, const float* a, const float* s, const float* acc_in, float d, float* out) {
    const int64_t per_block = (int64_t)kBlock * C, units = (P >> 2) + ((P & 3) ? 1 : 0);
    const int64_t tiles = (units + per_block - 1) / per_block;
    if (tiles > 0x7FFFFFFF) return fail(FA_ERR_ARG, "P=%lld too large for a tile launch", (long long)P);
    const dim3 grid((unsigned)tiles), block(kBlock);
#define FA_T(SC, ACC, FIN) \
    hipLaunchKernelGGL((k_fold_f32_tile<U, C, true, SC, ACC, FIN, NTS>), grid, block, 0, st, X, N, P, ldx, a, s, acc_in, d, out)
    if (sc) {
        if (acc) { if (fin) FA_T(true, true, true); else FA_T(true, true, false); }
        else     { if (fin) FA_T(true, false, true); else FA_T(true, false, false); }
    } else {
        if (acc) { if (fin) FA_T(false, true, true); else FA_T(false, true, false); }
        else     { if (fin) FA_T(false, false, true); else FA_T(false, false, false); }
    }
#undef FA_T
    return FA_OK;
}

// ALLF: instantiate every (scored, accumulate, finalize) combination -- only the
// auto variant needs them (fa_fold_f32); tuning variants are always a plain
// fold with the divide (acc == false, fin == true), so they instantiate two.
template <int U, int C, bool NTS, int B = kBlock, bool ALLF = false>
void launch_gs_flags(hipStream_t st, int per_cu, bool sc, bool acc, bool fin, const float* X, int64_t N, int64_t P,
                     int64_t ldx, const float* a, const float* s, const float* acc_in, float d, float* out) {
#define FA_G(SC, ACC, FIN) launch_gs<U, C, true, SC, ACC, FIN, NTS, B>(st, per_cu, X, N, P, ldx, a, s, acc_in, d, out)
    if constexpr (!ALLF) {
        if (sc) FA_G(true, false, true); else FA_G(false, false, true);
    } else if (sc) {
        if (acc) { if (fin) FA_G(true, true, true); else FA_G(true, true, false); }
        else     { if (fin) FA_G(true, false, true); else FA_G(true, false, false); }
    } else {
        if (acc) { if (fin) FA_G(false, true, true); else FA_G(false, true, false); }
        else     { if (fin) FA_G(false, false, true); else FA_G(false, false, false); }
    }
#undef FA_G
}

// Column bands: the fold as several back-to-back balanced grid-stride
// launches over contiguous column bands of about `passes` x CUs tiles each.
// Columns are independent, so this is the same arithmetic; the kernel
// boundaries re-align the blocks, which otherwise drift apart over many
// passes (C3: 4 bands of 611 tiles, 5.80 ms, against 5.91 ms as one launch,
// DESIGN.md 5).
template <int U, int C, bool NTS, bool ALLF = false>
void launch_gs_bands(hipStream_t st, int passes, bool sc, bool acc, bool fin, const float* X, int64_t N,
                     int64_t P, int64_t ldx, const float* a, const float* s, const float* acc_in, float d,
                     float* out) {
    const int64_t tq = (int64_t)kBlock * C;  // quads per tile
    const int64_t units = (P >> 2) + ((P & 3) ? 1 : 0);
    const int64_t tiles = (units + tq - 1) / tq;
    const int64_t per_band = (int64_t)passes * cu_count();
    const int64_t nb = (tiles + per_band - 1) / per_band;
    const int64_t band_tiles = (tiles + nb - 1) / nb;
    for (int64_t b = 0; b < nb; ++b) {
        const int64_t c0 = b * band_tiles * tq * 4;  // first column of the band (a multiple of 4 KiB x C)
        if (c0 >= P) break;
        const int64_t pb = (P - c0) < band_tiles * tq * 4 ? (P - c0) : band_tiles * tq * 4;
        launch_gs_flags<U, C, NTS, kBlock, ALLF>(st, -1, sc, acc, fin, N == 0 ? X : X + c0, N, pb, ldx, a, s,
                                   acc_in ? acc_in + c0 : nullptr, d, out + c0);
    }
}

template <bool SC, bool ACC, bool FIN>
void launch_scalar(hipStream_t st, const float* X, int64_t N, int64_t P, int64_t ldx, const float* a,
                   const float* s, const float* acc_in, float d, float* out) {
    hipLaunchKernelGGL((k_fold_f32_scalar<SC, ACC, FIN>), grid_for(P), dim3(kBlock), 0, st, X, N, P, ldx,
                       a, s, acc_in, d, out);
}

// Even-split fold (k_fold_f32_even): G blocks, per = ceil(nq / G) quads each.
template <int U, int C, bool ALLF = false>
void launch_even_flags(hipStream_t st, int64_t G, bool sc, bool acc, bool fin, const float* X, int64_t N, int64_t P,
                       int64_t ldx, const float* a, const float* s, const float* acc_in, float d, float* out) {
    const int64_t nq = P >> 2;
    if (G < 1) G = 1;
    int64_t per = (nq + G - 1) / G;
    if (per < 1) per = 1;
    const int64_t grid = nq > 0 ? (nq + per - 1) / per : 1;  // no empty trailing blocks
#define FA_E(SC, ACC, FIN)                                                                                   \
    hipLaunchKernelGGL((k_fold_f32_even<U, C, SC, ACC, FIN>), dim3((unsigned)grid), dim3(kBlock), 0, st, X, N, P, \
                       ldx, a, s, acc_in, d, out, per)
    if constexpr (!ALLF) {
        if (sc) FA_E(true, false, true); else FA_E(false, false, true);
    } else if (sc) {
        if (acc) { if (fin) FA_E(true, true, true); else FA_E(true, true, false); }
        else     { if (fin) FA_E(true, false, true); else FA_E(true, false, false); }
    } else {
        if (acc) { if (fin) FA_E(false, true, true); else FA_E(false, true, false); }
        else     { if (fin) FA_E(false, false, true); else FA_E(false, false, false); }
    }
#undef FA_E
}

// Quads per lane of the even split: the fewest that cover a block's range in
// one chunk (up to 4); rows in flight so that a lane keeps >= 16 quad loads
// (U*C) ahead of its adds whatever C is.
inline int even_quads_per_lane(int64_t P, int64_t G) {
    const int64_t nq = P >> 2;
    const int64_t per = (nq + G - 1) / (G > 0 ? G : 1);
    const int64_t c = (per + kBlock - 1) / kBlock;
    return c < 1 ? 1 : (c > 4 ? 4 : (int)c);
}
template <bool ALLF = false>
void launch_even_auto(hipStream_t st, int64_t G, bool sc, bool acc, bool fin, const float* X, int64_t N, int64_t P,
                      int64_t ldx, const float* a, const float* s, const float* acc_in, float d, float* out) {
    switch (even_quads_per_lane(P, G)) {
        case 1: launch_even_flags<16, 1, ALLF>(st, G, sc, acc, fin, X, N, P, ldx, a, s, acc_in, d, out); break;
        case 2: launch_even_flags<8, 2, ALLF>(st, G, sc, acc, fin, X, N, P, ldx, a, s, acc_in, d, out); break;
        case 3: launch_even_flags<8, 3, ALLF>(st, G, sc, acc, fin, X, N, P, ldx, a, s, acc_in, d, out); break;
        default: launch_even_flags<8, 4, ALLF>(st, G, sc, acc, fin, X, N, P, ldx, a, s, acc_in, d, out); break;
    }
}

// LDS-staged narrow fold: one block per TQ quads (the partial tail quad included).
template <int NW, int R, int TQ, int DEPTH = 1, bool ALLF = false, bool ROWS = false, bool COLF = true,
          int LOPT = 0, bool DW = false>
int launch_lds_flags(hipStream_t st, bool sc, bool acc, bool fin, const float* X, int64_t N, int64_t P,
                     int64_t ldx, const float* a, const float* s, const float* acc_in, float d, float* out) {
    // blocks over the full quads, plus one for the P%4 tail columns
    const int64_t blocks = ((P >> 2) + TQ - 1) / TQ + ((P & 3) ? 1 : 0);
    if (blocks * NW * 64 > (int64_t)0xFFFFFFFF)  // work-items per launch dimension
        return fail(FA_ERR_ARG, "P=%lld too large for an LDS-staged launch", (long long)P);
    const dim3 grid((unsigned)blocks), block(NW * 64);
#define FA_L(SC, ACC, FIN)                                                                                   \
    hipLaunchKernelGGL((k_fold_f32_lds<NW, R, TQ, SC, ACC, FIN, DEPTH, ROWS, COLF, LOPT, DW>), grid, block, 0, st, X, N, P, ldx, a, s, \
                       acc_in, d, out)
    if constexpr (!ALLF) {
        if (sc) FA_L(true, false, true); else FA_L(false, false, true);
    } else if (sc) {
        if (acc) { if (fin) FA_L(true, true, true); else FA_L(true, true, false); }
        else     { if (fin) FA_L(true, false, true); else FA_L(true, false, false); }
    } else {
        if (acc) { if (fin) FA_L(false, true, true); else FA_L(false, true, false); }
        else     { if (fin) FA_L(false, false, true); else FA_L(false, false, false); }
    }
#undef FA_L
    return FA_OK;
}

// bf16 grid-stride launch (per_cu < 0: balanced passes) and its column-band form
template <int U, int C>
void launch_bf16_gs(hipStream_t st, int per_cu, const uint16_t* X, int64_t N, int64_t P, int64_t ldx,
                    const float* a, const float* s, float d, float* out, uint16_t* outb) {
    const int64_t per_block = (int64_t)kBlock * C, units = (P >> 3) + ((P & 7) ? 1 : 0);
    const int64_t tiles = (units + per_block - 1) / per_block;
    int64_t g = (int64_t)(per_cu > 0 ? per_cu : -per_cu) * cu_count();
    if (g > tiles) g = tiles;
    if (per_cu < 0) {
        const int64_t passes = (tiles + g - 1) / g;
        g = (tiles + passes - 1) / passes;
    }
    if (s)
        hipLaunchKernelGGL((k_fedavg_bf16_gs<U, C, true>), dim3((unsigned)g), dim3(kBlock), 0, st, X, N, P, ldx, a,
                           s, d, out, outb, tiles);
    else
        hipLaunchKernelGGL((k_fedavg_bf16_gs<U, C, false>), dim3((unsigned)g), dim3(kBlock), 0, st, X, N, P, ldx,
                           a, s, d, out, outb, tiles);
}

template <int U, int C>
void launch_bf16_bands(hipStream_t st, int passes, const uint16_t* X, int64_t N, int64_t P, int64_t ldx,
                       const float* a, const float* s, float d, float* out, uint16_t* outb) {
    const int64_t to = (int64_t)kBlock * C;  // octets per tile
    const int64_t units = (P >> 3) + ((P & 7) ? 1 : 0);
    const int64_t tiles = (units + to - 1) / to;
    const int64_t per_band = (int64_t)passes * cu_count();
    const int64_t nb = (tiles + per_band - 1) / per_band;
    const int64_t band_tiles = (tiles + nb - 1) / nb;
    for (int64_t b = 0; b < nb; ++b) {
        const int64_t c0 = b * band_tiles * to * 8;
        if (c0 >= P) break;
        const int64_t pb = (P - c0) < band_tiles * to * 8 ? (P - c0) : band_tiles * to * 8;
        launch_bf16_gs<U, C>(st, -1, X + c0, N, pb, ldx, a, s, d, out ? out + c0 : nullptr, outb ? outb + c0 : nullptr);
    }
}

// ---- one launch per exchange step (k_*_step, fa_fedavg_*_rounds) ---------
// A step form: wide tiles (UB rows ahead x CB octets / quads per lane) dealt
// statically, and a dynamic pool of narrow tiles (US x CS) over the step's
// last columns, sized in passes of the grid over wide tiles (pool100 = 100:
// one pass; 0: every tile static).  256-thread blocks, one per CU.
struct StepSpec {
    const char* name;
    bool bf16;
    int ub, cb, us, cs, pool100;
    bool last_only = false;   // the pool never reaches past the last round's columns
    bool round_tail = false;  // each round but the last: whole passes of wide tiles, the rest in narrow static tiles
    bool bal = false;         // balanced rounds: each round's wide tiles over its own balanced block count
};
// The policy's two forms and one comparison form per dtype beside the round-4
// bf16 policy (the bench library and the GPU tests run every one).  Round 4
// measured 41 forms on the whole step with the exchange proxy's copies
// included (DESIGN_HISTORY.md R4; profiles/r04_step/): pool sizes, reduced
// grids, sc1 stores, pass barriers, all-dynamic tiles; round 5 the balanced
// rounds (profiles/r05_step/, r05_exchange/).  What is left:
//   bf16_step_bal_u8c4               the bf16 policy (a C4 rank's slots, round
//     5): each round's 8 x 4-octet wide tiles dealt over its own balanced
//     block count (step_tiles_bal), no dynamic pool; with the write-through
//     tile stores 0.978-0.989 ms alone against 1.011-1.017 for the round-4
//     policy, 1.013-1.018 / 1.046-1.050 beside copy-engine copies, the whole
//     step 1.15-1.18 / 1.20-1.22 beside 32-64 copy blocks (profiles/r05_step/wt/)
//   f32_step_sd_u8c4_p75             the fp32 policy (a C3 rank): 8 x 4-quad
//     static tiles and a 0.75-pass pool of 16 x 1-quad tiles; with the
//     write-through tile stores 5.81 ms alone against 5.80-5.81 per round,
//     the fold 5.90-5.93 beside 16-64 host-copy blocks against 6.06-6.18
//     (profiles/r05_step/wt_f32/); balanced rounds lost (6.05-6.10 against
//     5.91-5.95 alone, before the write-through stores)
//   bf16_step_rt_u8c4n8c2_p100_last  comparison: round 4's bf16 policy, whole
//     passes of wide tiles per round, the rest of each round in narrow static
//     tiles over all blocks, the last round's columns a one-pass dynamic pool
//   bf16_step_static_u8c4            comparison: every tile static (the one
//     launch without its dynamic part or its balancing)
//   f32_step_bal_u8c4                comparison: the fp32 step with balanced
//     rounds
constexpr StepSpec kStepSpecs[] = {
    {"bf16_step_bal_u8c4", true, 8, 4, 8, 2, 0, true, false, true},
    {"f32_step_sd_u8c4_p75", false, 8, 4, 16, 1, 75},
    {"bf16_step_rt_u8c4n8c2_p100_last", true, 8, 4, 8, 2, 100, true, true},
    {"bf16_step_static_u8c4", true, 8, 4, 8, 4, 0},
    {"f32_step_bal_u8c4", false, 8, 4, 16, 1, 0, true, false, true},
};
constexpr int kNumStepForms = (int)(sizeof(kStepSpecs) / sizeof(kStepSpecs[0]));
inline const char* step_form_name(int f) { return (f >= 0 && f < kNumStepForms) ? kStepSpecs[f].name : ""; }
constexpr bool name_eq(const char* a, const char* b) { return *a == *b && (*a == 0 || name_eq(a + 1, b + 1)); }
constexpr int step_form_index(const char* name) {
    for (int i = 0; i < kNumStepForms; ++i)
        if (name_eq(kStepSpecs[i].name, name)) return i;
    return -1;
}
inline int pick_step(bool bf16) {
    constexpr int kBf16 = step_form_index("bf16_step_bal_u8c4");
    constexpr int kF32 = step_form_index("f32_step_sd_u8c4_p75");
    static_assert(kBf16 >= 0 && kF32 >= 0, "policy step forms");
    return bf16 ? kBf16 : kF32;
}

// The per-launch state of fa_fedavg_*_rounds: the signal words in device
// memory, the waiters' timeout record in mapped host memory and the host
// epoch (fa_rounds in fedavg_hip.h).
struct RoundsState {
    int device = 0;
    unsigned int* sig = nullptr;          // kSigWords, zeroed at creation
    unsigned int* status_host = nullptr;  // [kStatusWords] page-locked, mapped: the epoch whose round-k wait timed
                                          // out (fa_rounds_wait's waiter, or a peer exchange's, fa_peers)
    unsigned int* status_dev = nullptr;   // the same words as the device addresses them
    unsigned int epoch = 0;               // of the last launch (0: none yet)
    unsigned int checked = 0;             // epochs up to this one were reported by rounds_check
    int rounds = 0;                       // of the last launch
    bool launched = false;                // the last launch was enqueued
    long long max_ticks = 0;              // a waiter's give-up time in wall-clock ticks
    int sys = 0;                          // publish rounds at system scope (a peer exchange's state): 1 = sc0 sc1
                                          // tile stores, no per-block fence (the product); 2 = sc1 tile stores
                                          // and a system release fence per block and round (round 5's form,
                                          // fa_bench_rounds_set_sys A/B only); 0 = agent scope
    hipEvent_t start = nullptr;           // recorded on the launch's stream just before the launch: a waiter's
                                          // stream waits for it, so its give-up clock starts with the fold
    hipStream_t last_stream = nullptr;    // the stream of the last launch
    hipEvent_t done = nullptr;            // recorded just after the launch: the next launch with this state
                                          // waits for it, whatever stream it is on (a stream handle reused
                                          // after its stream was destroyed cannot overlap two launches)
    hipEvent_t gate = nullptr;            // a peer exchange's state (fa_peers): recorded at the end of each
    bool gated = false;                   // exchange, and the next launch waits for it (peer_exchange.hpp)
};

// The segments of one step launch over `rounds` slots at local columns
// [offsets[k], offsets[k+1]): every round's columns in wide tiles, except the
// last pool columns of the step (cut at wide-tile boundaries, walking back
// from the last round) in narrow tiles.  FA status.
inline int build_step_table(const StepSpec& sp, int rounds, const int64_t* offsets, const int64_t* out_offsets,
                            int64_t ldx, int64_t grid, StepTable& T) {
    const int64_t ucols = sp.bf16 ? 8 : 4;  // columns per octet / quad
    const int64_t wide_cols = (int64_t)kBlock * sp.cb * ucols;
    T = StepTable{};
    T.rounds = rounds;
    int64_t pool = (sp.pool100 * grid * wide_cols) / 100;  // columns
    if (sp.last_only && pool > offsets[rounds] - offsets[rounds - 1]) pool = offsets[rounds] - offsets[rounds - 1];
    int64_t split[kMaxRounds];  // round k: columns [0, split) wide-static, [split, width) narrow-dynamic
    for (int k = rounds - 1; k >= 0; --k) {
        const int64_t c0 = offsets[k], w = offsets[k + 1] - offsets[k];
        if (c0 < 0 || w < 1 || c0 % ucols || offsets[k + 1] > ldx)
            return fail(FA_ERR_ARG, "round %d: columns [%lld, %lld) (every round non-empty, %lld-aligned, within ldx)",
                        k, (long long)c0, (long long)offsets[k + 1], (long long)ucols);
        if (out_offsets && (out_offsets[k] < 0 || out_offsets[k] % ucols))
            return fail(FA_ERR_ARG, "round %d: output column %lld (non-negative, %lld-aligned)", k,
                        (long long)out_offsets[k], (long long)ucols);
        if (pool <= 0) { split[k] = w; continue; }
        if (pool >= w) { split[k] = 0; pool -= w; continue; }
        split[k] = ((w - pool) / wide_cols) * wide_cols;  // the static part ends on a wide-tile boundary
        pool = 0;
    }
    auto units = [&](int64_t w) { return sp.bf16 ? (w >> 3) + ((w & 7) ? 1 : 0) : (w >> 2) + ((w & 3) ? 1 : 0); };
    int64_t total = 0;
    // static segments first (all of them precede every dynamic one in column
    // order: only a suffix of the step is dynamic), then the dynamic ones
    auto add_seg = [&](int k, int64_t lo, int64_t hi, bool small, bool is_static) {
        const int64_t c0 = offsets[k];
        const int64_t per = small ? (int64_t)kBlock * sp.cs : (int64_t)kBlock * sp.cb;
        const int g = T.segs++;
        total += (units(hi - lo) + per - 1) / per;
        T.seg_end[g] = total;
        T.col0[g] = c0 + lo;
        T.ocol0[g] = (out_offsets ? out_offsets[k] : c0) + lo;
        T.width[g] = hi - lo;
        T.round[g] = k;
        T.small[g] = small ? 1 : 0;
        T.round_tiles[k] += (units(hi - lo) + per - 1) / per;
        if (is_static) T.static_tiles = total;
        // balanced: the fewest blocks that fold the segment in the same number of passes
        const int64_t n = (units(hi - lo) + per - 1) / per, passes = (n + grid - 1) / grid;
        T.stride[g] = passes > 0 ? (n + passes - 1) / passes : 1;
    };
    for (int pass = 0; pass < 2; ++pass)
        for (int k = 0; k < rounds; ++k) {
            const int64_t w = offsets[k + 1] - offsets[k];
            const int64_t lo = pass == 0 ? 0 : split[k], hi = pass == 0 ? split[k] : w;
            if (hi <= lo) continue;
            if (pass == 0 && sp.round_tail && !sp.bal && k + 1 < rounds) {
                // whole passes of wide tiles, then the rest of the round's static columns narrow
                const int64_t full = ((hi - lo) / wide_cols / grid) * grid;
                const int64_t mid = lo + full * wide_cols;
                if (mid > lo) add_seg(k, lo, mid, false, true);
                if (hi > mid) add_seg(k, mid, hi, true, true);
                continue;
            }
            add_seg(k, lo, hi, pass == 1, pass == 0);
        }
    if (total > 0x7FFFFFFF) return fail(FA_ERR_ARG, "rounds fold: too many tiles");
    return FA_OK;
}

// A waiter's give-up time: 30 s after the fold reached the head of its
// stream, or FEDAVG_ROUND_WAIT_US microseconds (tests force the timeout path
// with a limit far below one fold).
inline long long round_wait_ticks(int khz) {
    long long us = 30LL * 1000 * 1000;
    const char* e = getenv("FEDAVG_ROUND_WAIT_US");
    if (e && e[0]) {
        char* end = nullptr;
        const long long v = strtoll(e, &end, 10);
        if (end && *end == 0 && v >= 0) us = v;
    }
    return (long long)khz * us / 1000;
}

// Create / destroy a launch state on `device`; enqueue a waiter for round k.
inline int rounds_state_init(RoundsState& o, int device) {
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess) {
        (void)hipGetLastError();
        return fail(FA_ERR_ARG, "rounds state: no device %d", device);
    }
    o.device = device;
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess || khz <= 0) khz = 100000;
    o.max_ticks = round_wait_ticks(khz);
    hipError_t e = hipMalloc((void**)&o.sig, kSigWords * sizeof(unsigned int));
    if (e == hipSuccess) e = hipMemset(o.sig, 0, kSigWords * sizeof(unsigned int));
    if (e == hipSuccess)
        e = hipHostMalloc((void**)&o.status_host, kStatusWords * sizeof(unsigned int),
                          hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess) {
        memset(o.status_host, 0, kStatusWords * sizeof(unsigned int));
        e = hipHostGetDevicePointer((void**)&o.status_dev, o.status_host, 0);
    }
    if (e == hipSuccess) e = hipEventCreateWithFlags(&o.start, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&o.done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    (void)hipSetDevice(prev);
    if (e != hipSuccess) {
        if (o.sig) (void)hipFree(o.sig);
        if (o.status_host) (void)hipHostFree(o.status_host);
        if (o.start) (void)hipEventDestroy(o.start);
        if (o.done) (void)hipEventDestroy(o.done);
        o.sig = nullptr;
        o.status_host = o.status_dev = nullptr;
        o.start = o.done = nullptr;
        return fail(FA_ERR_HIP, "rounds state: %s", hipGetErrorString(e));
    }
    return FA_OK;
}
inline void rounds_state_free(RoundsState& o) {
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(o.device);
    (void)hipDeviceSynchronize();  // no launch or waiter may still use the words
    if (o.sig) (void)hipFree(o.sig);
    if (o.status_host) (void)hipHostFree(o.status_host);
    if (o.start) (void)hipEventDestroy(o.start);
    if (o.done) (void)hipEventDestroy(o.done);
    if (o.gate) (void)hipEventDestroy(o.gate);
    o.sig = nullptr;
    o.status_host = o.status_dev = nullptr;
    o.start = o.done = o.gate = nullptr;
    o.gated = false;
    (void)hipSetDevice(prev);
}
inline int rounds_wait(RoundsState& o, int round, hipStream_t st) {
    if (!o.launched) return fail(FA_ERR_ARG, "rounds wait: the last rounds fold was not launched");
    if (round < 0 || round >= o.rounds) return fail(FA_ERR_ARG, "rounds wait: round %d of %d", round, o.rounds);
    if (o.start && hipStreamWaitEvent(st, o.start, 0) != hipSuccess) return check_launch("rounds wait: event");
    hipLaunchKernelGGL(k_wait_round, dim3(1), dim3(64), 0, st, o.sig + kSigFlag + round, o.epoch,
                       o.sig + kSigTimeout, o.status_dev ? o.status_dev + round : nullptr, o.max_ticks);
    return check_launch("k_wait_round");
}
// Rounds whose wait timed out in the launches since the last check (host
// memory only, no HIP call): valid for the waits that have already run.
inline int rounds_check(RoundsState& o) {
    if (!o.status_host) return 0;
    int n = 0;
    for (int k = 0; k < kStatusWords; ++k) {
        const unsigned int v = __atomic_load_n(&o.status_host[k], __ATOMIC_ACQUIRE);
        if (v != 0 && (int)(v - o.checked) > 0 && (int)(v - o.epoch) <= 0) ++n;
    }
    o.checked = o.epoch;
    return n;
}

// Enqueue one step launch of form f over `rounds` slots at local columns
// [offsets[k], offsets[k+1]).
inline int launch_step(RoundsState& R, int f, hipStream_t st, const void* X, int64_t N, int64_t ldx,
                       const float* a, const float* s, float divisor, float* out, uint16_t* outb, int rounds,
                       const int64_t* offsets, const int64_t* out_offsets = nullptr) {
    R.launched = false;
    if (f < 0 || f >= kNumStepForms) return fail(FA_ERR_ARG, "unknown step form %d", f);
    if (rounds < 1 || rounds > kMaxRounds || !offsets) return fail(FA_ERR_ARG, "rounds must be 1..%d", kMaxRounds);
    const StepSpec& sp = kStepSpecs[f];
    const int64_t col_align = sp.bf16 ? 8 : 4;
    // fp32 rows write out; bf16 rows out and/or outb (ABI 5: out may be null)
    if (!X || !a || N < 1 || (sp.bf16 ? (!out && !outb) : !out))
        return fail(FA_ERR_ARG, sp.bf16 ? "null X/a, no output (out_f32 and out_bf16 both null) or N < 1"
                                        : "null X/a/out or N < 1");
    if (ldx % col_align || !aligned16(X) || !aligned16(out) || (outb && !aligned16(outb)))
        return fail(FA_ERR_ARG, "rounds fold needs 16-B aligned X/out and ldx %% %lld == 0", (long long)col_align);
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
        (void)hipGetLastError();
        return fail(FA_ERR_ARG, "rounds fold cannot be captured (its epochs would replay)");
    }
    int64_t grid = cu_count();
    StepTable T;
    int rc = build_step_table(sp, rounds, offsets, out_offsets, ldx, grid, T);
    if (rc) return rc;
    T.sys = R.sys ? 1 : 0;
    T.sysfence = R.sys == 2 ? 1 : 0;
    const int wtm = R.sys == 1 ? kWtSystem : kWtAgent;  // the tiles' store flavour (a template argument)
    T.wt = 1;  // both step kernels store their tiles write-through (bf16_tile / fold_tile <..., WT>)
    const int64_t total = T.seg_end[T.segs - 1];
    if (grid > total) grid = total;
    const unsigned int epoch = R.epoch + 1 == 0 ? 1 : R.epoch + 1;
    // after the previous launch with this state: stream order when it ran on
    // this stream, else a wait for its done event
    if (R.epoch != 0 && R.done && st != R.last_stream && hipStreamWaitEvent(st, R.done, 0) != hipSuccess)
        return check_launch("rounds fold: previous launch");
    // a peer exchange's state: after the exchange of the previous launch
    if (R.gated && R.gate && hipStreamWaitEvent(st, R.gate, 0) != hipSuccess)
        return check_launch("rounds fold: previous exchange");
    if (R.start && hipEventRecord(R.start, st) != hipSuccess) return check_launch("rounds fold: start event");
    const uint16_t* Xb = static_cast<const uint16_t*>(X);
    const float* Xf = static_cast<const float*>(X);
    // the kernel instantiation is found from the form's tile shapes (never by
    // its index): a form whose shapes no instantiation below has is refused
    bool launched = false;
#define FA_STB(UB, CB, US, CS, BAL, WTM)                                                                         \
    if (!launched && sp.bf16 && sp.ub == UB && sp.cb == CB && sp.us == US && sp.cs == CS && sp.bal == BAL &&     \
        wtm == WTM) {                                                                                            \
        launched = true;                                                                                         \
        if (s)                                                                                                   \
            hipLaunchKernelGGL((k_fedavg_bf16_step<UB, CB, US, CS, true, kBlock, BAL, WTM>), dim3((unsigned)grid), \
                               dim3(kBlock), 0, st, Xb, N, ldx, a, s, divisor, out, outb, T, R.sig, epoch);     \
        else                                                                                                     \
            hipLaunchKernelGGL((k_fedavg_bf16_step<UB, CB, US, CS, false, kBlock, BAL, WTM>),                    \
                               dim3((unsigned)grid), dim3(kBlock), 0, st, Xb, N, ldx, a, s, divisor, out, outb, T, \
                               R.sig, epoch);                                                                    \
    }
#define FA_STF(UB, CB, US, CS, BAL, WTM)                                                                         \
    if (!launched && !sp.bf16 && sp.ub == UB && sp.cb == CB && sp.us == US && sp.cs == CS && sp.bal == BAL &&    \
        wtm == WTM) {                                                                                            \
        launched = true;                                                                                         \
        if (s)                                                                                                   \
            hipLaunchKernelGGL((k_fold_f32_step<UB, CB, US, CS, true, kBlock, BAL, WTM>), dim3((unsigned)grid),  \
                               dim3(kBlock), 0, st, Xf, N, ldx, a, s, divisor, out, T, R.sig, epoch);           \
        else                                                                                                     \
            hipLaunchKernelGGL((k_fold_f32_step<UB, CB, US, CS, false, kBlock, BAL, WTM>), dim3((unsigned)grid), \
                               dim3(kBlock), 0, st, Xf, N, ldx, a, s, divisor, out, T, R.sig, epoch);           \
    }
    FA_STB(8, 4, 8, 2, false, kWtAgent)
    FA_STB(8, 4, 8, 4, false, kWtAgent)
    FA_STB(8, 4, 8, 2, true, kWtAgent)
    FA_STF(8, 4, 16, 1, false, kWtAgent)
    FA_STF(8, 4, 16, 1, true, kWtAgent)
    // system-coherent stores: the two policy forms only (a peer exchange's launches)
    FA_STB(8, 4, 8, 2, true, kWtSystem)
    FA_STF(8, 4, 16, 1, false, kWtSystem)
#undef FA_STB
#undef FA_STF
    if (!launched)
        return fail(FA_ERR_ARG, "step form %s: no kernel for its tile shapes%s", sp.name,
                    wtm == kWtSystem ? " with system-coherent stores (the policy forms only)" : "");
    rc = check_launch("rounds fold");
    if (rc) return rc;
    if (R.done && hipEventRecord(R.done, st) != hipSuccess)
        return check_launch("rounds fold: done event");
    R.last_stream = st;
    R.epoch = epoch;
    R.rounds = rounds;
    R.launched = true;
    return FA_OK;
}

// ---- the pointer-table fold's forms (fa_fedavg_f32_ptrs_aligned) ----------
// Row bases come from a device table; the LDS-staged forms mirror the stacked
// fold's narrow picks, the grid-stride form its large-model default.
enum class PtrsForm { kLdsW2T16Ring, kLdsW2T16D2, kLdsW2T32, kLdsW4T24, kLdsW4T40, kLdsW8, kLdsW4T32, kRowsGs };
constexpr int kNumPtrsForms = (int)PtrsForm::kRowsGs + 1;
inline const char* ptrs_form_name(PtrsForm f) {
    switch (f) {
        case PtrsForm::kLdsW2T16Ring: return "ptrs_lds_w2_t16_ring";
        case PtrsForm::kLdsW2T16D2: return "ptrs_lds_w2_t16_d2";
        case PtrsForm::kLdsW2T32: return "ptrs_lds_w2_t32";
        case PtrsForm::kLdsW4T24: return "ptrs_lds_w4_t24";
        case PtrsForm::kLdsW4T40: return "ptrs_lds_w4_t40";
        case PtrsForm::kLdsW8: return "ptrs_lds_w8_t32";
        case PtrsForm::kLdsW4T32: return "ptrs_lds_w4_t32";
        case PtrsForm::kRowsGs: return "ptrs_rows_gs_16k";
    }
    return "";
}

// The policy: the stacked fold's LDS picks for narrow models, the 32-quad
// LDS fold up to ~3M params (it beat the tile kernel on table rows: 100 x
// 582K 42.3 against 76.6 us, 1024 x 2.5M 1.62 against 1.70 ms, but not at 4M
// with 1024 clients, 2.60 against 2.49 ms; profiles/r02_lds/dw_ptrs.log,
// ptrs_large.log, ptrs_mid.log), then ~one block per CU over 16 KiB tiles.
inline PtrsForm pick_ptrs(int64_t N, int64_t P) {
    switch (pick_f32(N, P)) {
        case F32Pick::kLdsW2T16:  // with the pointer ring (LOPT 4)
        case F32Pick::kLdsW2T16D4: return PtrsForm::kLdsW2T16Ring;
        case F32Pick::kLdsW2T16D2: return PtrsForm::kLdsW2T16D2;  // 1.2-1.6x over the 4-wave 32-quad table fold
                                                                  // at 32K-65K (profiles/r02_lds/ptrs_two_wave/)
        case F32Pick::kLdsW2T32: return PtrsForm::kLdsW2T32;
        case F32Pick::kLdsW4T24: return PtrsForm::kLdsW4T24;
        case F32Pick::kLdsW4T40: return PtrsForm::kLdsW4T40;
        case F32Pick::kLdsW8: return PtrsForm::kLdsW8;
        default: break;
    }
    return (P >> 2) < ((int64_t)3 << 18) ? PtrsForm::kLdsW4T32 : PtrsForm::kRowsGs;
}

inline void ptrs_candidates(int64_t N, int64_t P, int policy, std::vector<int>& v) {
    (void)N;
    v.push_back(policy);
    auto add = [&](PtrsForm f) {
        for (int x : v)
            if (x == (int)f) return;
        v.push_back((int)f);
    };
    if ((P >> 2) < (1 << 16))
        for (PtrsForm f : {PtrsForm::kLdsW2T16Ring, PtrsForm::kLdsW2T16D2, PtrsForm::kLdsW2T32, PtrsForm::kLdsW4T24,
                           PtrsForm::kLdsW4T40, PtrsForm::kLdsW8, PtrsForm::kLdsW4T32})
            add(f);
    else
        for (PtrsForm f : {PtrsForm::kLdsW4T32, PtrsForm::kLdsW8, PtrsForm::kLdsW4T40, PtrsForm::kRowsGs})
            add(f);
}

inline int launch_ptrs_form(PtrsForm f, hipStream_t st, const float* const* xi, int64_t N, int64_t P, const float* a,
                            const float* s, float divisor, float* out) {
    const bool sc = s != nullptr;
    const float* X = (const float*)xi;
    switch (f) {
        case PtrsForm::kLdsW2T16Ring:  // + terms by the loaders, exact stash waits (LOPT 4|8|2; round 3:
            // 1024 x 16K-30K stall-aware 11-14 % faster, plain 1-7 %, profiles/r03_premul/ptrs_exact.log)
            return launch_lds_flags<2, 32, 16, 4, false, true, true, 14>(st, sc, false, true, X, N, P, P, a, s, nullptr,
                                                                         divisor, out);
        case PtrsForm::kLdsW2T16D2:
            return launch_lds_flags<2, 32, 16, 2, false, true>(st, sc, false, true, X, N, P, P, a, s, nullptr, divisor,
                                                               out);
        case PtrsForm::kLdsW2T32:
            return launch_lds_flags<2, 16, 32, 2, false, true>(st, sc, false, true, X, N, P, P, a, s, nullptr, divisor,
                                                               out);
        case PtrsForm::kLdsW4T24:
            return launch_lds_flags<4, 32, 24, 2, false, true>(st, sc, false, true, X, N, P, P, a, s, nullptr, divisor,
                                                               out);
        case PtrsForm::kLdsW4T40:
            return launch_lds_flags<4, 32, 40, 2, false, true>(st, sc, false, true, X, N, P, P, a, s, nullptr, divisor,
                                                               out);
        case PtrsForm::kLdsW8:
            return launch_lds_flags<8, 64, 32, 1, false, true>(st, sc, false, true, X, N, P, P, a, s, nullptr, divisor,
                                                               out);
        case PtrsForm::kLdsW4T32:
            return launch_lds_flags<4, 16, 32, 2, false, true>(st, sc, false, true, X, N, P, P, a, s, nullptr, divisor,
                                                               out);
        case PtrsForm::kRowsGs: {
            const int64_t units = (P >> 2) + ((P & 3) ? 1 : 0);
            const int64_t tiles = (units + (int64_t)kBlock * 4 - 1) / ((int64_t)kBlock * 4);
            const int64_t cap = cu_count();
            const int64_t g = tiles > cap ? cap : tiles;
            if (sc)
                hipLaunchKernelGGL((k_fold_f32_rows_gs<8, 4, true>), dim3((unsigned)g), dim3(kBlock), 0, st, xi, N,
                                   P, a, s, divisor, out, tiles);
            else
                hipLaunchKernelGGL((k_fold_f32_rows_gs<8, 4, false>), dim3((unsigned)g), dim3(kBlock), 0, st, xi, N,
                                   P, a, s, divisor, out, tiles);
            return FA_OK;
        }
    }
    return fail(FA_ERR_ARG, "unknown pointer-table form");
}

// The tuner (tuner.hpp): a measured form per shape.
constexpr int kTuneF32 = 1, kTuneBf16 = 2, kTunePtrs = 3;
inline const char* tune_form_name(int kind, int form) {
    if (kind == kTunePtrs) return ptrs_form_name((PtrsForm)form);
    return kind == kTuneF32 ? f32_pick_name((F32Pick)form) : bf16_form_name((Bf16Form)form);
}
// a form's index from its name (the tuner's cache file and fa_tune_import)
inline int tune_form_from_name(int kind, const char* name) {
    const int n = kind == kTuneF32 ? kNumF32Picks : kind == kTuneBf16 ? kNumBf16Forms : kind == kTunePtrs ? kNumPtrsForms : 0;
    for (int f = 0; f < n; ++f)
        if (strcmp(tune_form_name(kind, f), name) == 0) return f;
    return -1;
}
// the cache file's device identity: gfx arch and CU count ("" = unknown: not persisted)
inline std::string tune_device_ident(int dev) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) {
        (void)hipGetLastError();
        return std::string();
    }
    char buf[128];
    snprintf(buf, sizeof(buf), "%s:%d", prop.gcnArchName, prop.multiProcessorCount);
    return buf;
}
fa_tune::Tuner g_tuner(tune_form_name, tune_form_from_name, tune_device_ident, FA_ABI_VERSION);

// fp32 candidates: the policy pick first, then the forms that won somewhere
// near this shape in the sweeps (profiles/r02_small_n/, r03_even/, r03_slot_sweep/).
inline void f32_candidates(int64_t N, int64_t P, int policy, std::vector<int>& v) {
    auto add = [&](F32Pick p) {
        for (int x : v)
            if (x == (int)p) return;
        v.push_back((int)p);
    };
    v.push_back(policy);
    const int64_t nq = P >> 2, cus = cu_count();
    const int64_t tiles4 = (((P + 3) >> 2) + 4 * kBlock - 1) / (4 * kBlock);
    if (nq < (1 << 16)) {  // narrow models: the LDS-staged forms, the 4 KiB tile
        for (F32Pick p : {F32Pick::kLdsW2T16, F32Pick::kLdsW2T16D4, F32Pick::kLdsW2T16D2, F32Pick::kLdsW2T32,
                          F32Pick::kLdsW4T24, F32Pick::kLdsW4T40, F32Pick::kLdsW8, F32Pick::kLdsQfW4T32, F32Pick::kTileC1})
            add(p);
    } else if (tiles4 < 2 * cus) {  // under two 16 KiB tiles per CU: where the forms swing most
        for (F32Pick p : {F32Pick::kGsBalC4, F32Pick::kGsBalC2, F32Pick::kTileC4Plain, F32Pick::kTileC4,
                          F32Pick::kTileU8C2, F32Pick::kTileC1, F32Pick::kEvenU4C4, F32Pick::kLdsQfW4T32,
                          F32Pick::kLdsW8, F32Pick::kGs1C4, F32Pick::kGsBands6})
            add(p);
        add(F32Pick::kColumn);
    } else if (policy == (int)F32Pick::kGsBalC4 && tiles4 >= 3 * cus) {
        // 3+ tiles per CU with the band form: every sweep and tuner decision at
        // 2.5M-25M params (C3, C5, their multi-GPU slots) kept the policy
        // (profiles/r03_tuner/, r03_c5_c3_sweep/: within 0.5 % of the best of 106
        // forms), so measuring there only costs the first call (C3: 132 ms)
    } else {  // large models: the grid-stride forms, the 16 KiB tile, the even split
        for (F32Pick p : {F32Pick::kGsBalC4, F32Pick::kGsBands6, F32Pick::kGsBalC2, F32Pick::kGs1C4,
                          F32Pick::kTileC4Plain, F32Pick::kEvenU4C4, F32Pick::kLdsQfW4T32})
            add(p);
    }
}

// Launch one fp32 form (the 16-B aligned vector path), every (scored,
// accumulate, finalize) combination for the policy's forms; the tuning-only
// forms instantiate the plain one-shot fold alone.
inline int launch_f32_pick(F32Pick pick, hipStream_t st, bool sc, bool acc, bool fin, const float* X, int64_t N,
                           int64_t P, int64_t ldx, const float* a, const float* s, const float* acc_in,
                           float divisor, float* out) {
    if (f32_tuning_only(pick) && (acc || !fin))
        return fail(FA_ERR_ARG, "fold form %s runs one-shot folds only", f32_pick_name(pick));
    int rc = FA_OK;
    switch (pick) {  // every (scored, accumulate, finalize) combination
        case F32Pick::kLdsW2T16:
            // the narrowest models (one block per CU): two-wave blocks (1024 x
            // 16K: 18.9 us against 22.0 for four waves, 256 x 16K: 6.6 against
            // 7.8; profiles/r02_lds/sweep_small.log); round 3: the loaders form
            // the terms (LOPT bit 3) and six chunks are in flight (1024 x 16K
            // 18.5 -> 16.6 us, 4096 x 16K 65.7 -> 56.3, stall-aware 1024 x 16K
            // 21.8 -> 18.7; profiles/r03_premul/), with a scheduling barrier
            // after each stage's loads (LOPT bit 1): without it the compiler
            // sinks the stall-aware form's factor loads and its stash waits
            // drain the pipeline to 6 of 72 loads (exact waits: 4096 x 16K
            // stall-aware 64.8 -> 59.7 us, plain within 1 %)
            rc = launch_lds_flags<2, 32, 16, 6, true, false, true, 10>(st, sc, acc, fin, X, N, P, ldx, a, s, acc_in,
                                                                       divisor, out);
            break;
        case F32Pick::kLdsW2T16D4:  // the same with four chunks in flight (16K-32K params)
            rc = launch_lds_flags<2, 32, 16, 4, true, false, true, 10>(st, sc, acc, fin, X, N, P, ldx, a, s, acc_in,
                                                                       divisor, out);
            break;
        case F32Pick::kLdsW2T16D2:
            rc = launch_lds_flags<2, 32, 16, 2, true>(st, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out);
            break;
        case F32Pick::kLdsW2T32:
            rc = launch_lds_flags<2, 16, 32, 2, true>(st, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out);
            break;
        case F32Pick::kLdsW4T24:
            rc = launch_lds_flags<4, 32, 24, 2, true>(st, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out);
            break;
        case F32Pick::kLdsW4T40:
            rc = launch_lds_flags<4, 32, 40, 2, true>(st, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out);
            break;
        case F32Pick::kLdsW8:
            rc = launch_lds_flags<8, 64, 32, 1, true>(st, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out);
            break;
        case F32Pick::kColumn:
#define FA_SC(SC, ACC, FIN) launch_scalar<SC, ACC, FIN>(st, X, N, P, ldx, a, s, acc_in, divisor, out)
            if (sc) {
                if (acc) { if (fin) FA_SC(true, true, true); else FA_SC(true, true, false); }
                else     { if (fin) FA_SC(true, false, true); else FA_SC(true, false, false); }
            } else {
                if (acc) { if (fin) FA_SC(false, true, true); else FA_SC(false, true, false); }
                else     { if (fin) FA_SC(false, false, true); else FA_SC(false, false, false); }
            }
#undef FA_SC
            break;
        case F32Pick::kTileC1:  // plain stores (non-temporal ones cost 3-10 % here)
            rc = launch_tile_flags<4, 1, false>(st, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out);
            break;
        case F32Pick::kTileC4:
            rc = launch_tile_flags<8, 4, true>(st, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out);
            break;
        case F32Pick::kTileC4Plain:
            rc = launch_tile_flags<8, 4, false>(st, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out);
            break;
        case F32Pick::kGsBalC2:
            launch_gs_flags<8, 2, true, kBlock, true>(st, -1, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out);
            break;
        case F32Pick::kGsBalC4:  // one band below 3 x CUs tiles; 3-pass bands were 0.3-1 % faster than
                                 // 4-pass ones at 512-1024 clients (profiles/r02_bands/)
            launch_gs_bands<8, 4, true, true>(st, 3, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out);
            break;
        // tuning-only forms (the sweeps' winners between the policy's measured shapes)
        case F32Pick::kGsBands6:
            launch_gs_bands<8, 4, true>(st, 6, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out);
            break;
        case F32Pick::kGs1C4:
            launch_gs_flags<8, 4, true>(st, 1, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out);
            break;
        case F32Pick::kTileU8C2:
            rc = launch_tile_flags<8, 2, false>(st, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out);
            break;
        case F32Pick::kEvenU4C4:
            launch_even_flags<4, 4>(st, cu_count(), sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out);
            break;
        case F32Pick::kLdsQfW4T32:  // LDS-staged, 4 waves, 16-row chunks of 32-quad tiles, quad fold
            rc = launch_lds_flags<4, 16, 32, 2, false, false, false>(st, sc, acc, fin, X, N, P, ldx, a, s, acc_in,
                                                                      divisor, out);
            break;
    }
    return rc;
}

// The product fp32 fold: checks, then the scalar fallback for unaligned input
// or the shape-picked vector fold (pick_f32).  acc_in continues a fold
// (fa_fold_f32); with acc_in and N == 0 it only finalises.
inline int fold_f32_auto(const float* X, int64_t N, int64_t P, int64_t ldx, const float* a, const float* s,
                         const float* acc_in, float divisor, int finalize, float* out, void* stream) {
    if (!(acc_in && N == 0)) {
        int rc = check_common(N, P, ldx, X, a, out);
        if (rc) return rc;
    } else if (P > 0 && !out) {
        return fail(FA_ERR_ARG, "null out pointer");
    }
    if (P == 0) { g_err[0] = 0; return FA_OK; }
    hipStream_t st = (hipStream_t)stream;
    StreamDevice on_stream_device(stream);
    const bool sc = s != nullptr, acc = acc_in != nullptr, fin = finalize != 0;
    const bool vec = (N == 0 || aligned16(X)) && (ldx % 4 == 0) && aligned16(out) &&
                     (!acc || aligned16(acc_in));
    if (!vec && N > 0 && (P >> 2) > 0 && ((P >> 2) < (1 << 13) || (N >= 256 && (P >> 2) < (1 << 16)))) {
        // rows not 16-B aligned (an odd pitch: a torch.stack of an odd-sized
        // model), narrow models: the LDS-staged fold with 4-byte loads.  The
        // per-column scalar fold below re-reads each row's segment once per
        // lane-column and ran 1.7x slower at 1024 x 16K-67K; from ~256K params
        // (or below 256 clients) it is as fast (profiles/r02_lds/dw_sweep.log)
        int rc;
        if ((P >> 2) < (1 << 13))
            rc = launch_lds_flags<2, 32, 16, 4, true, false, true, 0, true>(st, sc, acc, fin, X, N, P, ldx, a, s,
                                                                            acc_in, divisor, out);
        else
            rc = launch_lds_flags<4, 32, 40, 2, true, false, true, 0, true>(st, sc, acc, fin, X, N, P, ldx, a, s,
                                                                            acc_in, divisor, out);
        if (rc) return rc;
        return check_launch("fold_f32 (4-byte loads)");
    }
    if (!vec) {
#define FA_SC(SC, ACC, FIN) launch_scalar<SC, ACC, FIN>(st, X, N, P, ldx, a, s, acc_in, divisor, out)
        if (sc) {
            if (acc) { if (fin) FA_SC(true, true, true); else FA_SC(true, true, false); }
            else     { if (fin) FA_SC(true, false, true); else FA_SC(true, false, false); }
        } else {
            if (acc) { if (fin) FA_SC(false, true, true); else FA_SC(false, true, false); }
            else     { if (fin) FA_SC(false, false, true); else FA_SC(false, false, false); }
        }
#undef FA_SC
        return check_launch("k_fold_f32_scalar");
    }
    const F32Pick policy = pick_f32(N, P);
    // a plain one-shot fold (no accumulator in, with the divide) takes the
    // form the tuner measured fastest on this device.  Not when `out` overlaps
    // the rows: the measuring call runs several launches, and a later one
    // would read what an earlier one wrote (one launch alone reads every row
    // of a column before it writes that column)
    if (!acc && fin && N > 0 && !overlaps(out, (size_t)P * 4, X, ((size_t)(N - 1) * ldx + P) * 4)) {
        const int rc = g_tuner.run(kTuneF32, N, P, ldx, sc, (int)policy, (double)N * (double)P * 4.0, st,
                                   [&](std::vector<int>& c) { f32_candidates(N, P, (int)policy, c); },
                                   [&](int form) {
                                       return launch_f32_pick((F32Pick)form, st, sc, acc, fin, X, N, P, ldx, a, s,
                                                              acc_in, divisor, out);
                                   });
        if (rc) return rc;
        return check_launch("fold_f32");
    }
    int rc = launch_f32_pick(policy, st, sc, acc, fin, X, N, P, ldx, a, s, acc_in, divisor, out);
    if (rc) return rc;
    return check_launch("fold_f32");
}

// The policy's bf16 form by shape.
inline Bf16Form pick_bf16(int64_t N, int64_t P) {
    // 2.9M-5.6M params, 128+ clients (the 3.125M-param round slot of an 8-GPU C4 bucket):
    // four octets per lane (8 rows x 4 x 16 B in flight per lane), column bands of 4
    // passes: 0.238 against 0.260 ms at 256 x 3.125M (profiles/r03_c4_budget/), 5-11 %
    // faster at 3.1M-5M and 128-256 clients, but 2-8 % slower at 2.5M-3M and 6.25M-8M
    // (profiles/r02_slots/bf16_octets_scan/), hence the narrow range
    if (N >= 128 && (P >> 3) >= 368000 && (P >> 3) < 700000) return Bf16Form::kBandsU8C4;
    // per-GPU C4 buckets (256 x 12.5M) and their multi-GPU round slots
    // (256 x 3.125M): grid-stride, 8 rows x 2 octets, balanced passes in
    // column bands of 4 passes: +7 % over the row-streaming pick (DESIGN.md
    // 5), +1-1.4 % over one block per CU (profiles/r02_slots/)
    if (N >= 128 && (P >> 3) >= ((int64_t)1 << 17) && (P >> 3) < ((int64_t)1 << 22)) return Bf16Form::kBandsU8C2;
    // whole large models (C4's 100M on one GPU): balanced grid-stride
    // launches over 32 KiB tiles (fewer tile switches per block), in
    // column bands of 2 passes: +4 % over one launch
    if ((P >> 3) >= ((int64_t)1 << 22)) return Bf16Form::kBandsU2C8;
    // smaller models: one block per tile, octets per lane from the client count
    switch (pick_octets(N, P)) {
        case 8: return Bf16Form::kV8U2C8;
        case 4: return Bf16Form::kV8U4C4;
        case 2: return Bf16Form::kV8U8C2;
        default: return Bf16Form::kV8U8C1;
    }
}

inline void bf16_candidates(int64_t N, int64_t P, int policy, std::vector<int>& v) {
    auto add = [&](Bf16Form f) {
        for (int x : v)
            if (x == (int)f) return;
        v.push_back((int)f);
    };
    v.push_back(policy);
    // 1M+ octets (8.4M+ params: C4's per-GPU bucket, the whole model): the
    // band forms kept the policy at every measured shape (profiles/r03_tuner/)
    if ((P >> 3) >= ((int64_t)1 << 20) && (policy == (int)Bf16Form::kBandsU8C2 || policy == (int)Bf16Form::kBandsU2C8))
        return;
    if ((P >> 3) >= ((int64_t)1 << 17))
        for (Bf16Form f : {Bf16Form::kBandsU8C2, Bf16Form::kBandsU8C4, Bf16Form::kBandsU4C4, Bf16Form::kGsBalU8C2,
                           Bf16Form::kGs1U8C4, Bf16Form::kBandsU2C8, Bf16Form::kBandsU16C2, Bf16Form::kV8U8C1})
            add(f);
    else
        for (Bf16Form f : {Bf16Form::kV8U8C1, Bf16Form::kV8U8C2, Bf16Form::kV8U4C4, Bf16Form::kV8U2C8,
                           Bf16Form::kGs1U8C4, Bf16Form::kGsBalU8C2, Bf16Form::kBandsU8C4})
            add(f);
}

inline void launch_bf16_form(Bf16Form f, hipStream_t st, const uint16_t* X, int64_t N, int64_t P, int64_t ldx,
                             const float* a, const float* s, float divisor, float* out_f32, uint16_t* out_bf16) {
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
    switch (f) {
        case Bf16Form::kV8U2C8: FA_BF(2, 8); break;
        case Bf16Form::kV8U4C4: FA_BF(4, 4); break;
        case Bf16Form::kV8U8C2: FA_BF(8, 2); break;
        case Bf16Form::kV8U8C1: FA_BF(8, 1); break;
        case Bf16Form::kBandsU8C4: launch_bf16_bands<8, 4>(st, 4, X, N, P, ldx, a, s, divisor, out_f32, out_bf16); break;
        case Bf16Form::kBandsU8C2: launch_bf16_bands<8, 2>(st, 4, X, N, P, ldx, a, s, divisor, out_f32, out_bf16); break;
        case Bf16Form::kBandsU2C8: launch_bf16_bands<2, 8>(st, 2, X, N, P, ldx, a, s, divisor, out_f32, out_bf16); break;
        case Bf16Form::kBandsU4C4: launch_bf16_bands<4, 4>(st, 4, X, N, P, ldx, a, s, divisor, out_f32, out_bf16); break;
        case Bf16Form::kBandsU16C2:
            launch_bf16_bands<16, 2>(st, 4, X, N, P, ldx, a, s, divisor, out_f32, out_bf16);
            break;
        case Bf16Form::kGsBalU8C2: launch_bf16_gs<8, 2>(st, -1, X, N, P, ldx, a, s, divisor, out_f32, out_bf16); break;
        case Bf16Form::kGs1U8C4: launch_bf16_gs<8, 4>(st, 1, X, N, P, ldx, a, s, divisor, out_f32, out_bf16); break;
    }
#undef FA_BF
}

// The product bf16 fold (exact upcast, fp32 fold in order, optional RNE bf16 copy).
inline int bf16_auto(const uint16_t* X, int64_t N, int64_t P, int64_t ldx, const float* a, const float* s,
                     float divisor, float* out_f32, uint16_t* out_bf16, void* stream) {
    int rc = check_common(N, P, ldx, X, a, bf16_any_out(out_f32, out_bf16));
    if (rc) return rc;
    if (P == 0) { g_err[0] = 0; return FA_OK; }
    hipStream_t st = (hipStream_t)stream;
    StreamDevice on_stream_device(stream);
    const bool vec = aligned16(X) && (ldx % 8 == 0) && aligned16(out_f32) && aligned16(out_bf16);
    if (!vec) {
        if (s)
            hipLaunchKernelGGL(k_fedavg_bf16_scalar<true>, grid_for(P), dim3(kBlock), 0, st, X, N, P, ldx, a, s,
                               divisor, out_f32, out_bf16);
        else
            hipLaunchKernelGGL(k_fedavg_bf16_scalar<false>, grid_for(P), dim3(kBlock), 0, st, X, N, P, ldx, a, s,
                               divisor, out_f32, out_bf16);
        return check_launch("k_fedavg_bf16_scalar");
    }
    const Bf16Form policy = pick_bf16(N, P);
    const size_t xbytes = ((size_t)(N - 1) * ldx + P) * 2;
    if ((out_f32 && overlaps(out_f32, (size_t)P * 4, X, xbytes)) ||
        (out_bf16 && overlaps(out_bf16, (size_t)P * 2, X, xbytes))) {
        launch_bf16_form(policy, st, X, N, P, ldx, a, s, divisor, out_f32, out_bf16);  // in place: one launch
        return check_launch("fedavg_bf16");
    }
    g_tuner.run(kTuneBf16, N, P, ldx, s != nullptr, (int)policy, (double)N * (double)P * 2.0, st,
                [&](std::vector<int>& c) { bf16_candidates(N, P, (int)policy, c); },
                [&](int form) {
                    launch_bf16_form((Bf16Form)form, st, X, N, P, ldx, a, s, divisor, out_f32, out_bf16);
                    return FA_OK;
                });
    return check_launch("fedavg_bf16");
}

}  // namespace
