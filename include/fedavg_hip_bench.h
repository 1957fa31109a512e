/*
 * fedavg_hip_bench.h — C-ABI of libfedavg_hip_bench.so: bench and tuning
 * support for the engine of fedavg_hip.h.  NOT part of the product ABI and
 * not a reference interface: nothing in the drop-in path (fedlesscan_amd/)
 * loads this library.  bench.py and the GPU tests use it to generate
 * synthetic client matrices straight into HBM, to measure the streaming-read
 * ceiling next to the fold, and to sweep the kernel variants the product's
 * auto policy was chosen from.
 *
 * Same conventions as fedavg_hip.h (device pointers, hipStream_t, FA_* codes);
 * fa_bench_last_error() describes this library's last failure.
 */
#ifndef FEDAVG_HIP_BENCH_H
#define FEDAVG_HIP_BENCH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

const char* fa_bench_last_error(void);

/* Deterministic generator, bit-identical to fedlesscan_amd/synth.py. */
int fa_synth_f32(float* X, int64_t nrows, int64_t ncols, int64_t ldx, uint64_t seed,
                 int64_t row0, int64_t col0, void* stream);
int fa_synth_bf16(uint16_t* X, int64_t nrows, int64_t ncols, int64_t ldx, uint64_t seed,
                  int64_t row0, int64_t col0, void* stream);
/* Contiguous read-only sweep of n floats, one 64 KiB chunk per block (16 B
 * per lane) -> one partial per block in sink[block % sink_len] (values are
 * meaningless): the streaming-read ceiling the fold is compared with. */
int fa_read_sweep_f32(const float* X, int64_t n, float* sink, int64_t sink_len, void* stream);
/* A copy kernel on a fixed number of blocks (dst <- src, n floats, 16-B
 * aligned, n % 4 == 0): stands in for a collective's kernels next to the fold
 * (tools/exchange_interference.py), which occupy a few CUs each. */
int fa_bench_copy_f32(float* dst, const float* src, int64_t n, int blocks, void* stream);
/* A stream on `device` limited to the CUs whose bit is set in mask[0..words)
 * (hipExtStreamCreateWithCUMask), and its release: the exchange proxy's
 * fold stream that leaves some CUs to the collective. */
int fa_bench_stream_cu_mask(int device, const uint32_t* mask, int words, void** stream);
int fa_bench_stream_destroy(void* stream);
/* fa_fedavg_f32 with an explicit kernel variant; variant 0 = the product's
 * auto fold.  Layouts the vector kernels cannot take (X / out not 16-B
 * aligned, ldx % 4 != 0) run the product's scalar fold whatever the variant.
 * Returns FA_ERR_ARG for an unknown variant. */
int fa_fedavg_f32_variant(const float* X, int64_t N, int64_t P, int64_t ldx,
                          const float* a, const float* s, float divisor,
                          float* out, void* stream, int variant);
int fa_num_variants(void);
/* [host] short name of a variant, e.g. "gsband4_u8c4nt_nts"; "" if out of range. */
const char* fa_variant_name(int variant);
/* [host, no GPU needed] the kernel form the product's fp32 auto fold picks for
 * N clients x P params (16-B aligned rows) on a GPU with `cus` compute units
 * (<= 0: the current device's), e.g. "tile_4k", "gs_bands_16k"; "" if N or P < 1. */
const char* fa_f32_pick_name(int64_t N, int64_t P, int64_t cus);
/* One kernel form of the product's fp32 / bf16 fold, by index (the forms the
 * shape policy and the tuner choose between: fa_num_*_forms, fa_*_form_name);
 * a plain one-shot fold.  Lets the tests check every form the tuner may pick. */
int fa_num_f32_forms(void);
const char* fa_f32_form_name(int form);
int fa_fedavg_f32_form(const float* X, int64_t N, int64_t P, int64_t ldx, const float* a, const float* s,
                       float divisor, float* out, void* stream, int form);
int fa_num_ptrs_forms(void);
const char* fa_ptrs_form_name(int form);
int fa_fedavg_f32_ptrs_form(const float* const* xi, int64_t N, int64_t P, const float* a, const float* s,
                            float divisor, float* out, void* stream, int form);
int fa_num_bf16_forms(void);
const char* fa_bf16_form_name(int form);
int fa_fedavg_bf16_form(const uint16_t* X, int64_t N, int64_t P, int64_t ldx, const float* a, const float* s,
                        float divisor, float* out_f32, uint16_t* out_bf16, void* stream, int form);
/* Same for the bf16 fold (variant 0 = fa_fedavg_bf16). */
int fa_fedavg_bf16_variant(const uint16_t* X, int64_t N, int64_t P, int64_t ldx,
                           const float* a, const float* s, float divisor,
                           float* out_f32, uint16_t* out_bf16, void* stream, int variant);
int fa_num_bf16_variants(void);
const char* fa_bf16_variant_name(int variant);
/* The pointer-table fold (xi = device table of N row pointers) with an
 * explicit kernel, tile and loader schedule, variant in
 * [0, fa_num_ptrs_variants()): variants named ptrs_o* need every row and out
 * 16-B aligned (as fa_fedavg_f32_ptrs_aligned); ptrs_dw_*, ptrs_rows_scalar
 * and ptrs_generic take rows at any 4-B offset (as fa_fedavg_f32_ptrs). */
int fa_fedavg_f32_ptrs_variant(const float* const* xi, int64_t N, int64_t P,
                               const float* a, const float* s, float divisor,
                               float* out, void* stream, int variant);
int fa_num_ptrs_variants(void);
const char* fa_ptrs_variant_name(int variant);

/* One launch per exchange step with a chosen step form (fa_step_form_name;
 * the product's fa_fedavg_*_rounds runs the policy's form): a bench-library
 * launch state, the launch and its waiter.  X/out_bf16 are bf16 for the
 * bf16_* forms (out or out_bf16 may be NULL, not both), fp32 otherwise
 * (out_bf16 ignored). */
int fa_num_step_forms(void);
const char* fa_step_form_name(int form);
int fa_bench_rounds_create(void** r, int device);
int fa_bench_rounds_destroy(void* r);
int fa_fedavg_rounds_form(void* r, int form, const void* X, int64_t N, int64_t ldx, const float* a, const float* s,
                          float divisor, float* out, uint16_t* out_bf16, int rounds, const int64_t* offsets,
                          void* stream);
int fa_bench_rounds_wait(void* r, int round, void* stream);
/* How the state's launches publish their rounds: 0 agent scope (the default,
 * sc1 tile stores); 1 system scope as a peer exchange's state (fa_peers_rounds:
 * sc0 sc1 tile stores, the policy forms only); 2 system scope as round 5 did
 * (sc1 tile stores and a system release fence per block and round): the A/B of
 * what the system-scope publication costs the fold (tools/peer_step_decomp.py). */
int fa_bench_rounds_set_sys(void* r, int sys);

#ifdef __cplusplus
}
#endif

#endif /* FEDAVG_HIP_BENCH_H */
