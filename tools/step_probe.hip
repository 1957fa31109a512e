// step_probe.hip -- the one-launch bf16 step kernel (k_fedavg_bf16_step,
// csrc/fold_kernels.hpp) timed alone at a C4 rank's slots, beside variants of
// its tile-dealing loop compiled in the same translation unit, so that a
// question about the step's code costs one short compile and one GPU call
// instead of a library build.  Every variant folds the same columns with the
// same tile body, so every output bit must equal the first variant's.
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -I include \
//         -I fedlesscan_amd/csrc tools/step_probe.hip -o tools/step_probe.bin
//   tools/step_probe.bin [reps]
// Variants:
//   lib_rt    the library kernel, round 4's policy table (rt_u8c4n8c2_p100_last)
//   lib_bal   the library kernel, balanced rounds (the round-5 policy)
//   r04_rt    round 4's tile-dealing loop (pass-barrier bookkeeping compiled in,
//             disabled at run time; relaxed flag exchange), the same tile body
//   lean_rt   the current loop with the tile lambda reduced to one call site
//   bal_nopub the balanced loop with its per-round publication compiled out
//             (no drain, barrier, write-back or count: timing only)
//   static    every tile static, block b folding b, b + G, ... across the
//             rounds (bf16_step_static_u8c4's table)
//   perround  the rounds as 4 separate balanced grid-stride launches
//             (launch_bf16_gs, per_cu -1: what per-round launches run)
//   whole     the step's columns as ONE balanced grid-stride launch
//   bal_nofence  the balanced loop publishing without the per-block release
//             fence (plain stores: NOT a valid hand-off, timing only)
//   bal_sc1   the balanced loop with write-through (sc1) 16-B output stores and
//             no per-block release fence: every storing wave's vmcnt(0), a
//             barrier, the count; the completing block acquires and raises
//             the flag with a release store (MI355X_MICROARCH.md, valid forms)
//   bal_libtile  the same loop over the library's write-through tile body
//   lib_bal_wide the library's step_tiles_bal with one tile body for both
//             tile kinds
// (The list run is the vs[] table in main; the library's tables get wt = 1,
// as launch_step sets it.)
#include "fold_kernels.hpp"

#include <algorithm>
#include <vector>

namespace {

#define PCHECK(x)                                                                           \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

// round 4's loop (git bd08368), pass barriers never taken (sync_passes 0)
template <class Tile>
__device__ __forceinline__ void r04_step_tiles(const StepTable& T, unsigned int* sig, unsigned int epoch,
                                               int sync_passes, Tile tile) {
    __shared__ unsigned int nxt[2];
    const int64_t ntiles = T.seg_end[T.segs - 1];
    const int64_t Ts = T.static_tiles;
    const int64_t G = gridDim.x;
    int p = 0;
    int64_t t = blockIdx.x;
    const int S = sync_passes;
    if (t >= Ts) {
        for (int i = 0; S && i < 32; ++i) __syncthreads();
        if (threadIdx.x == 0) nxt[p] = atomicAdd(&sig[0], 1u);
        __syncthreads();
        t = Ts + nxt[p];
        p ^= 1;
    }
    int g = 0;
    while (g + 1 < T.segs && t >= T.seg_end[g]) ++g;
    int k = T.round[g];
    unsigned int cnt = 0;
    while (t < ntiles) {
        const bool dyn_next = t + G >= Ts;
        unsigned int nx = 0;
        if (dyn_next && threadIdx.x == 0) nx = atomicAdd(&sig[0], 1u);
        tile(g, t - (g ? T.seg_end[g - 1] : 0));
        ++cnt;
        int64_t tn = t + G;
        if (dyn_next) {
            if (threadIdx.x == 0) nxt[p] = nx;
            __syncthreads();
            tn = Ts + nxt[p];
            p ^= 1;
        }
        if (S && t < Ts) {  // never at run time: the bookkeeping round 4 compiled in
            const int64_t jt = t / G;
            if (tn < Ts) {
                const int64_t jn = tn / G;
                if (jn % S == 0) __syncthreads();
            } else {
                for (int64_t i = jt / S + 1; i <= 32; ++i) __syncthreads();
            }
        }
        int gn = g;
        while (gn < T.segs && tn >= T.seg_end[gn]) ++gn;
        const int kn = gn < T.segs ? T.round[gn] : kMaxRounds;
        if (kn != k) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (threadIdx.x == 0) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const unsigned int nk = (unsigned int)T.round_tiles[k];
                if (atomicAdd(&sig[kSigDone + k], cnt) + cnt == nk) {
                    atomicExch(&sig[kSigDone + k], 0u);
                    atomicExch(&sig[kSigFlag + k], epoch);
                }
            }
            cnt = 0;
            k = kn;
        }
        t = tn;
        g = gn < T.segs ? gn : g;
    }
    if (threadIdx.x == 0) {
        if (atomicAdd(&sig[1], 1u) == gridDim.x - 1) {
            atomicExch(&sig[0], 0u);
            atomicExch(&sig[1], 0u);
        }
    }
}

template <int UB, int CB, int US, int CS>
__global__ __launch_bounds__(kBlock) void k_r04_step(const uint16_t* __restrict__ X, int64_t N, int64_t ldx,
                                                     const float* __restrict__ a, float divisor,
                                                     float* __restrict__ out, uint16_t* __restrict__ outb, StepTable T,
                                                     unsigned int* sig, unsigned int epoch, int sync_passes) {
    r04_step_tiles(T, sig, epoch, sync_passes, [&](int g, int64_t bid) {
        const int64_t c0 = T.col0[g];
        uint16_t* ob = outb ? outb + c0 : nullptr;
        if (T.small[g])
            bf16_tile<US, CS, false, kBlock>(bid, X + c0, N, T.width[g], ldx, a, nullptr, divisor, out + c0, ob);
        else
            bf16_tile<UB, CB, false, kBlock>(bid, X + c0, N, T.width[g], ldx, a, nullptr, divisor, out + c0, ob);
    });
}

template <int UB, int CB, int US, int CS>
__global__ __launch_bounds__(kBlock) void k_lean_step(const uint16_t* __restrict__ X, int64_t N, int64_t ldx,
                                                      const float* __restrict__ a, float divisor,
                                                      float* __restrict__ out, uint16_t* __restrict__ outb,
                                                      StepTable T, unsigned int* sig, unsigned int epoch) {
    step_tiles(T, sig, epoch, [&](int g, int64_t bid) {
        const int64_t c0 = T.col0[g];
        uint16_t* ob = outb ? outb + c0 : nullptr;
        if (T.small[g])
            bf16_tile<US, CS, false, kBlock>(bid, X + c0, N, T.width[g], ldx, a, nullptr, divisor, out + c0, ob);
        else
            bf16_tile<UB, CB, false, kBlock>(bid, X + c0, N, T.width[g], ldx, a, nullptr, divisor, out + c0, ob);
    });
}

// a 16-B write-through store (sc1: the line leaves the XCD's L2 for memory):
// a raw buffer store over a wave-uniform base, cache-policy operand 8 = sc1
// (gfx94x/gfx950 encoding of the operand: 1 sc0, 2 nt, 16 sc1)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wt_rsrc(void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(base, (short)0, -1, 0x00020000);
}
__device__ __forceinline__ void st16_sc1(__amdgpu_buffer_rsrc_t r, int64_t byte_off, u32x4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)byte_off, 0, 16);
}

// bf16_tile / fold_octets (csrc/fold_kernels.hpp) with the output stores
// chosen: SC1 write-through, else non-temporal.  Unscored.
template <int U, int C, bool SC1>
__device__ __forceinline__ void fold_octets_st(const u32x4* __restrict__ p, int64_t ldo, int64_t N,
                                               const float* __restrict__ a, float divisor, float* __restrict__ out,
                                               uint16_t* __restrict__ outb, int64_t o0) {
    f32x4 ev[C], od[C];
    {
        const float a0 = a[0];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            f32x4 e, o;
            unpack_bf16x8(__builtin_nontemporal_load(p + c * kBlock), e, o);
            ev[c] = term4<false>(e, a0, 1.0f);
            od[c] = term4<false>(o, a0, 1.0f);
        }
    }
    int64_t i = 1;
    for (; i + U <= N; i += U) {
        u32x4 v[U][C];
        octets_ld<U, C>(v, p, i, ldo);
        octets_add<U, C, false>(ev, od, v, a, nullptr, i);
    }
    for (; i < N; ++i) {
        const float ai = a[i];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            f32x4 e, o;
            unpack_bf16x8(__builtin_nontemporal_load(p + i * ldo + c * kBlock), e, o);
            ev[c] = add4(ev[c], term4<false>(e, ai, 1.0f));
            od[c] = add4(od[c], term4<false>(o, ai, 1.0f));
        }
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const f32x4 e = div4(ev[c], divisor), o = div4(od[c], divisor);
        const int64_t oc = o0 + (int64_t)c * kBlock;
        f32x4* o4 = reinterpret_cast<f32x4*>(out) + 2 * oc;
        const u32x4 lo = __builtin_bit_cast(u32x4, f32x4{e.x, o.x, e.y, o.y});
        const u32x4 hi = __builtin_bit_cast(u32x4, f32x4{e.z, o.z, e.w, o.w});
        u32x4 b;
        b.x = (uint32_t)f2bf_rne(e.x) | ((uint32_t)f2bf_rne(o.x) << 16);
        b.y = (uint32_t)f2bf_rne(e.y) | ((uint32_t)f2bf_rne(o.y) << 16);
        b.z = (uint32_t)f2bf_rne(e.z) | ((uint32_t)f2bf_rne(o.z) << 16);
        b.w = (uint32_t)f2bf_rne(e.w) | ((uint32_t)f2bf_rne(o.w) << 16);
        if constexpr (SC1) {
            const __amdgpu_buffer_rsrc_t ro = wt_rsrc(out), rb = wt_rsrc(outb);
            st16_sc1(ro, 32 * oc, lo);
            st16_sc1(ro, 32 * oc + 16, hi);
            st16_sc1(rb, 16 * oc, b);
        } else {
            st16(o4, lo);
            st16(o4 + 1, hi);
            st16(reinterpret_cast<u32x4*>(outb) + oc, b);
        }
    }
}

template <int U, int C, bool SC1>
__device__ __forceinline__ void bf16_tile_st(int64_t bid, const uint16_t* __restrict__ X, int64_t N, int64_t P,
                                             int64_t ldx, const float* __restrict__ a, float divisor,
                                             float* __restrict__ out, uint16_t* __restrict__ outb) {
    const int64_t no = P >> 3, ldo = ldx >> 3;  // P % 8 == 0 here (64-aligned slots)
    const int64_t o0 = bid * (kBlock * C) + threadIdx.x;
    const u32x4* X8 = reinterpret_cast<const u32x4*>(X);
    if (o0 + (int64_t)(C - 1) * kBlock < no) {
        fold_octets_st<U, C, SC1>(X8 + o0, ldo, N, a, divisor, out, outb, o0);
        return;
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int64_t o = o0 + (int64_t)c * kBlock;
        if (o < no) fold_octets_st<U, 1, SC1>(X8 + o, ldo, N, a, divisor, out, outb, o);
    }
}

// the round's publication without the per-block release fence: every storing
// wave drained, a barrier, one lane counts; the completing block acquires and
// raises the flag with a release store
__device__ __forceinline__ void publish_nofence(const StepTable& T, unsigned int* sig, unsigned int epoch, int k,
                                                unsigned int cnt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned int nk = (unsigned int)T.round_tiles[k];
        if (__hip_atomic_fetch_add(&sig[kSigDone + k], cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + cnt ==
            nk) {
            __hip_atomic_store(&sig[kSigDone + k], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            __hip_atomic_store(&sig[kSigFlag + k], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

template <bool SC1, bool LIBTILE = false>
__global__ __launch_bounds__(kBlock) void k_bal_nofence(const uint16_t* __restrict__ X, int64_t N, int64_t ldx,
                                                        const float* __restrict__ a, float divisor,
                                                        float* __restrict__ out, uint16_t* __restrict__ outb,
                                                        StepTable T, unsigned int* sig, unsigned int epoch) {
    const int64_t b = blockIdx.x;
    int k = -1;
    unsigned int cnt = 0;
    for (int g = 0; g < T.segs; ++g) {
        const int64_t lo = g ? T.seg_end[g - 1] : 0;
        if (lo >= T.static_tiles) break;
        if (T.round[g] != k) {
            if (k >= 0 && cnt) publish_nofence(T, sig, epoch, k, cnt);
            k = T.round[g];
            cnt = 0;
        }
        const int64_t n = T.seg_end[g] - lo, S = T.stride[g];
        const int64_t c0 = T.col0[g];
        for (int64_t i = b; b < S && i < n; i += S) {
            if constexpr (LIBTILE)
                bf16_tile<8, 4, false, kBlock, true>(i, X + c0, N, T.width[g], ldx, a, nullptr, divisor, out + c0,
                                                     outb + c0);
            else
                bf16_tile_st<8, 4, SC1>(i, X + c0, N, T.width[g], ldx, a, divisor, out + c0, outb + c0);
            ++cnt;
        }
    }
    if (k >= 0 && cnt) publish_nofence(T, sig, epoch, k, cnt);
    step_reset(sig);
}

// step_tiles_bal with the per-round publication optional (PUB false: timing only)
template <bool PUB, class Wide>
__device__ __forceinline__ void bal_tiles(const StepTable& T, unsigned int* sig, unsigned int epoch, Wide wide) {
    const int64_t b = blockIdx.x;
    const int64_t Ts = T.static_tiles;
    int k = -1;
    unsigned int cnt = 0;
    for (int g = 0; g < T.segs; ++g) {
        const int64_t lo = g ? T.seg_end[g - 1] : 0;
        if (lo >= Ts) break;
        if (T.round[g] != k) {
            if (PUB && k >= 0 && cnt) step_publish(T, sig, epoch, k, cnt);
            k = T.round[g];
            cnt = 0;
        }
        const int64_t n = T.seg_end[g] - lo, S = T.stride[g];
        for (int64_t i = b; b < S && i < n; i += S) {
            wide(g, i);
            ++cnt;
        }
    }
    if (PUB && k >= 0 && cnt) step_publish(T, sig, epoch, k, cnt);
    if (PUB) step_reset(sig);
}

// the library's step_tiles_bal with one tile body for wide and narrow tiles
__global__ __launch_bounds__(kBlock) void k_lib_bal_wide_only(const uint16_t* __restrict__ X, int64_t N, int64_t ldx,
                                                              const float* __restrict__ a, float divisor,
                                                              float* __restrict__ out, uint16_t* __restrict__ outb,
                                                              StepTable T, unsigned int* sig, unsigned int epoch) {
    auto wide = [&](int g, int64_t bid) {
        const int64_t c0 = T.col0[g];
        bf16_tile<8, 4, false, kBlock, true>(bid, X + c0, N, T.width[g], ldx, a, nullptr, divisor, out + c0,
                                             outb ? outb + c0 : nullptr);
    };
    step_tiles_bal(T, sig, epoch, wide, wide);
}

template <bool PUB>
__global__ __launch_bounds__(kBlock) void k_bal_step(const uint16_t* __restrict__ X, int64_t N, int64_t ldx,
                                                     const float* __restrict__ a, float divisor,
                                                     float* __restrict__ out, uint16_t* __restrict__ outb, StepTable T,
                                                     unsigned int* sig, unsigned int epoch) {
    bal_tiles<PUB>(T, sig, epoch, [&](int g, int64_t bid) {
        const int64_t c0 = T.col0[g];
        bf16_tile<8, 4, false, kBlock>(bid, X + c0, N, T.width[g], ldx, a, nullptr, divisor, out + c0,
                                       outb ? outb + c0 : nullptr);
    });
}

__global__ void k_fill(uint16_t* X, int64_t n, uint64_t seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        X[i] = (uint16_t)(((z >> 8) & 0x8000u) | ((0x70u + ((z >> 20) & 0xFu)) << 7) | (z & 0x7Fu));
    }
}

}  // namespace

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 30;
    const int64_t N = 256, rounds = 4;
    const int64_t offs[5] = {0, 4934912, 4934912 + 3454464, 4934912 + 3454464 + 2418112,
                             4934912 + 3454464 + 2418112 + 1692672};
    const int64_t P = offs[4], ldx = P;
    const int64_t grid = cu_count();
    uint16_t *X, *outb;
    float *a, *out;
    unsigned int* sig;
    PCHECK(hipMalloc(&X, (size_t)N * ldx * 2));
    PCHECK(hipMalloc(&a, N * 4));
    PCHECK(hipMalloc(&out, P * 4));
    PCHECK(hipMalloc(&outb, P * 2));
    PCHECK(hipMalloc(&sig, kSigWords * 4));
    PCHECK(hipMemset(sig, 0, kSigWords * 4));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, X, N * ldx, 777ull);
    std::vector<float> ha(N);
    double tot = 0;
    for (int64_t i = 0; i < N; ++i) tot += (ha[i] = (float)(1 + (i * 7919) % 97));
    PCHECK(hipMemcpy(a, ha.data(), N * 4, hipMemcpyHostToDevice));
    const float div = (float)tot;
    StepTable Trt, Tbal, Tst;
    if (build_step_table(kStepSpecs[step_form_index("bf16_step_rt_u8c4n8c2_p100_last")], (int)rounds, offs, ldx, grid,
                         Trt) ||
        build_step_table(kStepSpecs[step_form_index("bf16_step_bal_u8c4")], (int)rounds, offs, ldx, grid, Tbal) ||
        build_step_table(kStepSpecs[step_form_index("bf16_step_static_u8c4")], (int)rounds, offs, ldx, grid, Tst)) {
        fprintf(stderr, "step table: %s\n", g_err);
        return 1;
    }
    Trt.wt = Tbal.wt = Tst.wt = 1;  // as launch_step sets it for the bf16 step (write-through tiles)
    hipStream_t st;
    PCHECK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    PCHECK(hipEventCreate(&e0));
    PCHECK(hipEventCreate(&e1));
    unsigned int epoch = 0;
    const double bytes = (double)N * P * 2 + (double)P * 6;
    printf("C4 rank step: N %lld, P %lld in %lld rounds, grid %lld, %.3f GB per launch, %d reps\n", (long long)N,
           (long long)P, (long long)rounds, (long long)grid, bytes / 1e9, reps);
    struct V {
        const char* name;
        int which;
    } vs[] = {{"lib_bal", 1}, {"bal_sc1", 9}, {"bal_libtile", 10}, {"lib_bal_wide", 11}, {"perround", 6},
              {"lib_bal", 1}, {"bal_sc1", 9}, {"bal_libtile", 10}, {"lib_bal_wide", 11}, {"perround", 6},
              {"lib_bal", 1}, {"bal_sc1", 9}, {"bal_libtile", 10}, {"lib_bal_wide", 11}};
    std::vector<uint32_t> ref(P), cur(P);
    bool have = false;
    for (const V& v : vs) {
        auto launch = [&]() {
            ++epoch;
            const StepTable& Tv = v.which == 1 || v.which == 4 || v.which >= 8 ? Tbal : v.which == 5 ? Tst : Trt;
            (void)Tv;
            const unsigned int g = (unsigned int)std::min<int64_t>(grid, Tv.seg_end[Tv.segs - 1]);
            switch (v.which) {
                case 0:
                    hipLaunchKernelGGL((k_fedavg_bf16_step<8, 4, 8, 2, false, kBlock, false>), dim3(g), dim3(kBlock),
                                       0, st, X, N, ldx, a, nullptr, div, out, outb, Trt, sig, epoch);
                    break;
                case 1:
                    hipLaunchKernelGGL((k_fedavg_bf16_step<8, 4, 8, 2, false, kBlock, true>), dim3(g), dim3(kBlock),
                                       0, st, X, N, ldx, a, nullptr, div, out, outb, Tbal, sig, epoch);
                    break;
                case 2:
                    hipLaunchKernelGGL((k_r04_step<8, 4, 8, 2>), dim3(g), dim3(kBlock), 0, st, X, N, ldx, a, div, out,
                                       outb, Trt, sig, epoch, 0);
                    break;
                case 3:
                    hipLaunchKernelGGL((k_lean_step<8, 4, 8, 2>), dim3(g), dim3(kBlock), 0, st, X, N, ldx, a, div,
                                       out, outb, Trt, sig, epoch);
                    break;
                case 4:
                    hipLaunchKernelGGL((k_bal_step<false>), dim3(g), dim3(kBlock), 0, st, X, N, ldx, a, div, out,
                                       outb, Tbal, sig, epoch);
                    break;
                case 5:
                    hipLaunchKernelGGL((k_fedavg_bf16_step<8, 4, 8, 4, false, kBlock, false>), dim3(g), dim3(kBlock),
                                       0, st, X, N, ldx, a, nullptr, div, out, outb, Tst, sig, epoch);
                    break;
                case 8:
                    hipLaunchKernelGGL((k_bal_nofence<false>), dim3(g), dim3(kBlock), 0, st, X, N, ldx, a, div, out,
                                       outb, Tbal, sig, epoch);
                    break;
                case 9:
                    hipLaunchKernelGGL((k_bal_nofence<true>), dim3(g), dim3(kBlock), 0, st, X, N, ldx, a, div, out,
                                       outb, Tbal, sig, epoch);
                    break;
                case 10:
                    hipLaunchKernelGGL((k_bal_nofence<true, true>), dim3(g), dim3(kBlock), 0, st, X, N, ldx, a, div,
                                       out, outb, Tbal, sig, epoch);
                    break;
                case 11: {
                    StepTable Tw = Tbal;
                    Tw.wt = 1;
                    hipLaunchKernelGGL(k_lib_bal_wide_only, dim3(g), dim3(kBlock), 0, st, X, N, ldx, a, div, out, outb,
                                       Tw, sig, epoch);
                    break;
                }
                case 6:
                    for (int k = 0; k < rounds; ++k)
                        launch_bf16_gs<8, 4>(st, -1, X + offs[k], N, offs[k + 1] - offs[k], ldx, a, nullptr, div,
                                             out + offs[k], outb + offs[k]);
                    break;
                default:
                    launch_bf16_gs<8, 4>(st, -1, X, N, P, ldx, a, nullptr, div, out, outb);
            }
        };
        PCHECK(hipMemsetAsync(out, 0xFF, P * 4, st));
        launch();
        PCHECK(hipGetLastError());
        PCHECK(hipStreamSynchronize(st));
        PCHECK(hipMemcpy(have ? cur.data() : ref.data(), out, P * 4, hipMemcpyDeviceToHost));
        const bool same = !have || memcmp(ref.data(), cur.data(), P * 4) == 0;
        have = true;
        std::vector<float> ms;
        for (int r = 0; r < reps; ++r) {
            PCHECK(hipEventRecord(e0, st));
            launch();
            PCHECK(hipEventRecord(e1, st));
            PCHECK(hipEventSynchronize(e1));
            float t;
            PCHECK(hipEventElapsedTime(&t, e0, e1));
            ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        printf("%-8s median %.4f ms (min %.4f)  %.1f GB/s  bits %s\n", v.name, ms[ms.size() / 2], ms[0],
               bytes / ms[ms.size() / 2] / 1e6, same ? "same" : "DIFFER");
        fflush(stdout);
    }
    return 0;
}
