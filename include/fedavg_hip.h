/*
 * fedavg_hip.h — C-ABI of libfedavg_hip.so, the MI355X (gfx950) FedAvg /
 * FedLesScan parameter-aggregation engine.
 *
 * The reference has no native code; its hot path is the numpy fold in
 *   fedless/aggregator/fed_avg_aggregator.py:24-42   FedAvgAggregator._aggregate
 *   fedless/aggregator/stall_aware_aggregation.py:42-67  StallAwareAggregator._aggregate
 * The Python drop-in classes (fedlesscan_amd/aggregator/) bind these entry
 * points with ctypes; INTEGRATION.md shows the binding a maintainer would add
 * to the reference itself.
 *
 * Conventions
 *  - Every data pointer is DEVICE memory (hipMalloc / torch CUDA tensors)
 *    unless marked [host].  The caller owns all buffers; the library never
 *    allocates or frees in a compute call.
 *  - X is row-major [N][ldx]: row i = client i's flattened parameters, in the
 *    order the reference iterates client_results.  ldx >= P (elements).
 *  - a[i] = fl(n_i), the client's cardinality rounded to the compute type the
 *    way numpy rounds a Python scalar; s[i] = fl((r_i+1)/(R+1)) for the
 *    stall-aware variant, NULL for FedAvg; divisor = fl(sum_i n_i) with the
 *    sum taken exactly (Python int).  These are [device] arrays of N.
 *  - stream is a hipStream_t (NULL = legacy default stream).  All work is
 *    enqueued on it; no call synchronises.  Calls are reentrant; the only
 *    state they keep is the measured kernel form per shape (fa_set_autotune),
 *    which changes which kernel runs, never the result.
 *  - Result, bit for bit:  acc = t_0; acc = acc + t_i (i = 1..N-1, in order);
 *    out = acc / divisor, where t_i = (x_i * a_i) [* s_i] with separate
 *    roundings (no FMA) and an IEEE divide.
 *  - Return FA_OK (0) or an FA_ERR_* code; fa_last_error() describes the last
 *    failure on the calling thread.
 */
#ifndef FEDAVG_HIP_H
#define FEDAVG_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FA_ABI_VERSION 6

enum fa_status {
    FA_OK = 0,
    FA_ERR_ARG = 1,        /* bad size/pointer/stride -> ValueError                          */
    FA_ERR_NO_CLIENTS = 2, /* N == 0 -> InsufficientClientResults.  ABI guard only: the strategies never
                              fold zero rows (an empty round aggregates to [] on the host, as the
                              reference's _aggregate does: fed_avg_aggregator.py:31-42) */
    FA_ERR_SHAPE = 3,      /* -> InvalidParameterShapeError (exceptions.py:13)                  */
    FA_ERR_HIP = 4,        /* launch / runtime failure -> AggregationError (exceptions.py:1)    */
};

int fa_abi_version(void);
/* [host] message for the last failing call on this thread ("" if none). */
const char* fa_last_error(void);

/* ---- FedAvg / stall-aware fold over a stacked [N][ldx] matrix --------------
 * replaces FedAvgAggregator._aggregate      (fed_avg_aggregator.py:24-42)  when s == NULL
 * replaces StallAwareAggregator._aggregate  (stall_aware_aggregation.py:42-67) when s != NULL */
int fa_fedavg_f32(const float* X, int64_t N, int64_t P, int64_t ldx,
                  const float* a, const float* s, float divisor,
                  float* out, void* stream);

/* OPT-IN, NOT BIT-EXACT.  The same weighted mean for models too narrow to
 * fill the GPU (a few thousand to ~100K params): each column's clients are
 * cut into 32 contiguous slices folded in order, and the partial sums are
 * combined in a fixed pairwise tree (wavefront shuffles, then LDS).  Results
 * are deterministic run to run but differ from the reference's left fold
 * (fed_avg_aggregator.py:38-41) in the last bits: a different association
 * of the same sum.  Needs 16-B aligned X and out, ldx % 4 == 0. */
int fa_fedavg_f32_splitn(const float* X, int64_t N, int64_t P, int64_t ldx,
                         const float* a, const float* s, float divisor,
                         float* out, void* stream);

/* Same fold over N separately allocated client rows: xi is a [device] array of
 * N [device] pointers, each to P floats (the list-of-arrays form the reference
 * passes: fed_avg_aggregator.py:32-35). */
int fa_fedavg_f32_ptrs(const float* const* xi, int64_t N, int64_t P,
                       const float* a, const float* s, float divisor,
                       float* out, void* stream);
/* The same with every row promised 16-B aligned by the caller (and out 16-B
 * aligned): the tiled, grid-stride schedule of the stacked fold. */
int fa_fedavg_f32_ptrs_aligned(const float* const* xi, int64_t N, int64_t P,
                               const float* a, const float* s, float divisor,
                               float* out, void* stream);

/* Chunked fold, the building block of streaming ingest
 * (StreamFedAvgAggregator.aggregate, fed_avg_aggregator.py:111-153):
 *   acc_in == NULL : acc = t_0 + ... (as fa_fedavg_f32)
 *   acc_in != NULL : acc = acc_in[p] + t_0 + t_1 + ...  (continues a fold in order)
 *   finalize != 0  : out = acc / divisor, else out = acc (partial, unrounded by /)
 * acc_in may alias out.  Folding rows in chunks this way is bit-identical to
 * one fa_fedavg_f32 over all rows. */
int fa_fold_f32(const float* X, int64_t N, int64_t P, int64_t ldx,
                const float* a, const float* s, const float* acc_in,
                float divisor, int finalize, float* out, void* stream);

/* Single-row forms with scalar factors, for ingest that folds
 * each client as it arrives:
 *   fa_accumulate_f32: acc = first ? t : acc + t,  t = fl(fl(x*a) * s)
 *                      (s = 1.0f for FedAvg: multiplying by 1 is exact)
 *   fa_finalize_f32:   out = acc / divisor   (acc may alias out)
 * Accumulating the rows in client order and finalising once is bit-identical
 * to fa_fedavg_f32 over the stacked rows. */
int fa_accumulate_f32(float* acc, const float* x, float a, float s, int first, int64_t P, void* stream);
int fa_finalize_f32(const float* acc, float divisor, float* out, int64_t P, void* stream);

/* bf16 updates (BASELINE config 4; no reference path: defined as exact upcast
 * to f32 + the f32 fold).  out_f32 [P] (the fp32 result) and out_bf16 [P] (its
 * RNE bf16 copy) are each optional, at least one given (ABI 5: a multi-GPU
 * step exchanges only the bf16 copy, so it stores no fp32 result; both NULL ->
 * FA_ERR_ARG).  The bf16 bits are the same whether out_f32 is given or not. */
int fa_fedavg_bf16(const uint16_t* X, int64_t N, int64_t P, int64_t ldx,
                   const float* a, const float* s, float divisor,
                   float* out_f32, uint16_t* out_bf16, void* stream);

/* ---- one launch per exchange step (ABI 3) -----------------------------------
 * At N > 1 a rank folds its columns in `rounds` slots and all-gathers each
 * slot while the next one folds (fedlesscan_amd/sharding.py).  Folding each
 * slot in its own launch leaves a tail per launch, and the launches beside the
 * exchange lose blocks to the collective's kernels.  fa_fedavg_*_rounds folds
 * every slot of a step in ONE launch: column tiles are taken from a device
 * counter (round 0's first, then round 1's, ...), so a round's last tiles
 * overlap the next round's first ones and blocks that share a CU with other
 * kernels fold fewer tiles; when round k's last tile is done the launch
 * raises round k's flag.  fa_rounds_wait(r, k, stream) enqueues on another
 * stream a one-lane kernel that returns once round k of r's last launch is
 * complete (its results visible device-wide): the exchange of round k
 * enqueued behind it on that stream starts mid-launch.  Same bits as
 * fa_fedavg_f32 / fa_fedavg_bf16 on each slot.
 *   fa_rounds_create / _destroy: the launch state (device signal words) for
 *     one device; launches with one object must be ordered (one stream), and
 *     destroy synchronises the device.
 *   offsets [host] rounds + 1 local columns: round k folds columns
 *     [offsets[k], offsets[k+1]) of X (and writes the same columns of out);
 *     every round non-empty, 16-B aligned (offsets % 4, bf16 % 8), ldx too;
 *     1 <= rounds <= 8.  Not under graph capture (FA_ERR_ARG).
 *   fa_rounds_wait: round < the last launch's rounds; the stream first waits
 *     for the launch to reach the head of its own stream (an event recorded
 *     just before it), then a waiter that sees no completion within 30 s
 *     (FEDAVG_ROUND_WAIT_US at fa_rounds_create: another limit, for tests)
 *     returns anyway: whatever is queued behind it would read an unfinished
 *     round.  The waiter records that in page-locked host memory.
 *   fa_rounds_check (ABI 4): [host, no HIP call, no synchronisation] the
 *     number of rounds whose wait timed out in the launches since the last
 *     check (or creation), as far as the waits that have already run show --
 *     call it once the waits are known complete (an event recorded behind
 *     them); nonzero means an exchange behind a wait read an unfinished round
 *     and its result must not be used (fedlesscan_amd/sharding.py raises
 *     AggregationError on every rank).
 *   fa_rounds_timeouts: (synchronous) every timed-out wait since creation.
 *   fa_fedavg_bf16_rounds: out_f32 / out_bf16 as fa_fedavg_bf16 (ABI 5: either
 *     may be NULL, not both).
 *   out_offsets (ABI 5) [host] rounds output columns, or NULL: round k's
 *     results go to columns [out_offsets[k], out_offsets[k] + width k) of the
 *     outputs instead of [offsets[k], offsets[k+1]) (each 4-aligned, bf16
 *     8-aligned) -- a rank writes its slot of round k straight into its own
 *     chunk of the gathered model, and the all-gather runs in place. 
 *   One object per launching stream (engine.py keeps one per stream object). */
typedef struct fa_rounds fa_rounds;
int fa_rounds_create(fa_rounds** r, int device);
int fa_rounds_destroy(fa_rounds* r);
int fa_fedavg_f32_rounds(fa_rounds* r, const float* X, int64_t N, int64_t ldx,
                         const float* a, const float* s, float divisor, float* out,
                         int rounds, const int64_t* offsets, const int64_t* out_offsets, void* stream);
int fa_fedavg_bf16_rounds(fa_rounds* r, const uint16_t* X, int64_t N, int64_t ldx,
                          const float* a, const float* s, float divisor,
                          float* out_f32, uint16_t* out_bf16,
                          int rounds, const int64_t* offsets, const int64_t* out_offsets, void* stream);
int fa_rounds_wait(fa_rounds* r, int round, void* stream);
int fa_rounds_check(fa_rounds* r);
int fa_rounds_timeouts(fa_rounds* r);
/* [host] the kernel form fa_fedavg_bf16_rounds (bf16 != 0) / _f32_rounds runs */
const char* fa_rounds_form(int bf16);

/* ---- kernel-free peer exchange of a step (ABI 4; ABI 5: no fence) ----------
 * The reference saves ONE global model per round (aggregation.py:125-138 ->
 * ParameterDao.save, client_daos.py:351-378); at N > 1 every rank folds its
 * slots and needs every other rank's.  An RCCL all-gather runs copy kernels on
 * a few CUs beside the next round's fold; here each rank PULLS its peers'
 * finished slots with hipMemcpyAsync on two copy streams from their send
 * buffers, opened once through IPC handles.  One object per rank and layout;
 * every call below that names a step is made by every rank of the group, in
 * the same order.
 *   fa_peers_create:  this rank's two send buffers (send_bytes each, a 16-B
 *                     multiple; step e's fold writes buffer e % 2) and its own
 *                     rounds state (device memory)
 *   fa_peers_handle_bytes / fa_peers_handle: [host] this rank's IPC handles
 *   fa_peers_open:    [host] every rank's handles, world x handle_bytes in rank
 *                     order (all-gathered by the caller); opens the peers'
 *   fa_peers_send:    [host] the send buffer of the NEXT fold launch with
 *                     fa_peers_rounds (ask before every step): the fold writes
 *                     this rank's slots there (out_bf16 for bf16 rows, out for fp32)
 *   fa_peers_rounds:  [host] the rounds state (owned by the fa_peers) to pass
 *                     to fa_fedavg_*_rounds: its launches store their tiles
 *                     system-coherent and publish every round at system scope,
 *                     and each waits for the state's previous exchange
 *   fa_peers_exchange: enqueue, after the launch, on another stream: per round
 *                     k, a wait until every rank has completed round k, then
 *                     rank q's bytes [src_offsets[k], src_offsets[k+1]) of its
 *                     send buffer of this step are copied to dst +
 *                     dst_offsets[k * world + q] (this rank's own slot
 *                     included, last).  A wait that gives up is reported by
 *                     fa_rounds_check(fa_peers_rounds).  The next fold launch
 *                     with the state waits for this exchange; with the two
 *                     buffers that is what keeps a buffer from being rewritten
 *                     before every peer has pulled it (no fence, no ack)
 *   fa_peers_destroy: after every rank's last exchange (a barrier) */
typedef struct fa_peers fa_peers;
int fa_peers_create(fa_peers** x, int device, int world, int rank, int64_t send_bytes);
int fa_peers_destroy(fa_peers* x);
int fa_peers_handle_bytes(void);
int fa_peers_handle(fa_peers* x, void* out);
int fa_peers_open(fa_peers* x, const void* all_handles);
void* fa_peers_send(fa_peers* x);
fa_rounds* fa_peers_rounds(fa_peers* x);
int fa_peers_exchange(fa_peers* x, int rounds, const int64_t* src_offsets, void* dst, const int64_t* dst_offsets,
                      void* stream);

/* The same folds with the per-client factors a[0..N), s[0..N) (s may be
 * NULL) in HOST memory, as the reference's caller holds them (Python numbers,
 * fed_avg_aggregator.py:32-41).  The library copies them into a page-locked
 * slot of its own, sends them in one async H2D on a staging stream of its own
 * that `stream` waits for (an event) ahead of the fold, and reuses the slot
 * only after that fold has completed, so a and s may be freed or rewritten as
 * soon as the call returns.  X, xi, out stay device
 * pointers.  _ptrs: rows_aligned != 0 takes fa_fedavg_f32_ptrs_aligned's
 * kernels (every row 16-B aligned, out 16-B aligned), 0 fa_fedavg_f32_ptrs. */
int fa_fedavg_f32_hostf(const float* X, int64_t N, int64_t P, int64_t ldx,
                        const float* a, const float* s, float divisor,
                        float* out, void* stream);
int fa_fedavg_f32_ptrs_hostf(const float* const* xi, int64_t N, int64_t P,
                             const float* a, const float* s, float divisor,
                             int rows_aligned, float* out, void* stream);
int fa_fedavg_bf16_hostf(const uint16_t* X, int64_t N, int64_t P, int64_t ldx,
                         const float* a, const float* s, float divisor,
                         float* out_f32, uint16_t* out_bf16, void* stream);
/* The _hostf entries refuse a capturing stream (FA_ERR_ARG, ABI 6): a graph
 * would have to own the staged copy.  Under capture, write the factors into
 * memory the graph owns (PyTorch: a tensor allocated inside the capture) with
 * fa_factors_fill -- dst[0..N) = a, then dst[N..2N) = s when s != NULL, by
 * kernels whose arguments carry the values, so replays need no host memory --
 * and call the device-factor entry (fa_fedavg_f32, fa_fedavg_bf16, ...). */
int fa_factors_fill(float* dst, const float* a, const float* s, int64_t N, void* stream);
/* The one-launch step with host factors (ABI 5): as fa_fedavg_*_rounds, the
 * factors staged by the library like the folds above (one C call per step). */
int fa_fedavg_f32_rounds_hostf(fa_rounds* r, const float* X, int64_t N, int64_t ldx,
                               const float* a, const float* s, float divisor, float* out,
                               int rounds, const int64_t* offsets, const int64_t* out_offsets, void* stream);
int fa_fedavg_bf16_rounds_hostf(fa_rounds* r, const uint16_t* X, int64_t N, int64_t ldx,
                                const float* a, const float* s, float divisor,
                                float* out_f32, uint16_t* out_bf16,
                                int rounds, const int64_t* offsets, const int64_t* out_offsets, void* stream);

/* Measured form choice.  Every kernel form of the fp32, bf16 and row-table
 * folds computes the same bits; which is fastest depends on how a shape's
 * tiles fall on the CUs.  For plain one-shot folds (fa_fedavg_f32, _bf16,
 * _f32_ptrs_aligned and their _hostf forms) the FIRST call of a new (device,
 * kind, N, P, ldx, scored) shape runs every candidate form on the caller's
 * data and stream (an untimed launch each, then two timed passes of batched
 * launches between events), and once those events have completed -- read
 * back without synchronising on later calls -- the shape runs the fastest
 * (the shape policy's own form unless another is > 3 % faster).  Outputs are
 * bit-identical whatever form runs.  Library-wide switch, on unless
 * FEDAVG_AUTOTUNE=0 at load; FEDAVG_AUTOTUNE_LOG=1 prints each decision.
 *   fa_set_autotune:     1 on, 0 off (the policy form only), -1 query;
 *                        returns the previous setting
 *   fa_autotune_pending: shapes seen whose measurement is not complete
 *   fa_fold_form:        the form a shape runs on the stream's device:
 *                        the measured choice, "" while it is being measured,
 *                        the policy's form for an unseen shape or with the
 *                        tuner off.
 * The measuring call runs several launches into the same output, so a fold
 * whose out overlaps its input rows keeps the policy's single launch; for
 * fa_fedavg_f32_ptrs_aligned (row pointers live in device memory) out must
 * not alias a row -- as the reference, which returns new arrays. */
enum fa_fold_kind {
    FA_FOLD_F32 = 1,      /* fa_fedavg_f32 (_hostf)                     */
    FA_FOLD_BF16 = 2,     /* fa_fedavg_bf16 (_hostf)                    */
    FA_FOLD_F32_ROWS = 3, /* fa_fedavg_f32_ptrs_aligned (_hostf), ldx = P */
};
int fa_set_autotune(int mode);
int fa_autotune_pending(void);
const char* fa_fold_form(int kind, int64_t N, int64_t P, int64_t ldx, int scored, void* stream);
/* Decisions outlive the process (ABI 3).  A shape's key takes the client
 * count as its power-of-two bucket (a round with 1000 results reuses what
 * 1024 measured) plus the policy's form.  Every decision is merged into a
 * text cache file (one line per shape: device arch and CU count, ABI version,
 * kind, client bucket, policy form, P, ldx, scored, chosen form -- forms by
 * name), written under an exclusive lock through a temp file and a rename;
 * the first tuned call of a process reads it, so a cold process (one FaaS
 * invocation: aggregation.py:71-75) runs a known shape's form on its first
 * call.  Unparseable lines, another ABI or an unknown form are ignored.
 * Default path $XDG_CACHE_HOME/fedlesscan_amd/tuner.txt or
 * ~/.cache/fedlesscan_amd/tuner.txt; FEDAVG_TUNE_CACHE=<path> or =0 (off).
 *   fa_tune_cache_path: set the file at run time ("" or NULL: off)
 *   fa_tune_export:     [host] this process's decisions as those lines into
 *                       buf (NUL-terminated, truncated to cap - 1); returns
 *                       the full length
 *   fa_tune_import:     [host] apply such lines (a decision made elsewhere
 *                       replaces this process's own for the same shape);
 *                       returns the number of lines applied.  A multi-GPU job
 *                       broadcasts rank 0's export so that every rank runs the
 *                       same forms. */
int fa_tune_cache_path(const char* path);
int64_t fa_tune_export(char* buf, int64_t cap);
int fa_tune_import(const char* text);
/* Step-form decisions (ABI 4).  A multi-GPU exchange step runs as one
 * fa_fedavg_*_rounds launch or as one fold launch per round; which is faster
 * depends on how much the exchange's kernels slow the fold on the machine,
 * so ShardedAggregator measures it once (an opt-in probe) and keeps the
 * answer in the tuner's cache file as a "fedavg-step" line, exported and
 * imported with the kernel forms.  key = "<device identity> <f32|bf16>
 * <world size> <client-count bucket (a power of two)> <P> <w0,w1,...>" (the
 * layout's 1-8 slot widths).  A cold process then runs the recorded form with
 * no probe (aggregation.py:71-75 builds a fresh strategy per invocation).
 *   fa_step_lookup: 1 one launch per step, 0 per-round launches, -1 no
 *                   decision, -2 malformed key (the file is read once)
 *   fa_step_record: record (and merge into the file) a decision */
int fa_step_lookup(const char* key);
int fa_step_record(const char* key, int one_launch);

/* float64 updates (the reference unit-test fixture is float64,
 * test/test_aggregation.py:23-38). */
int fa_fedavg_f64(const double* X, int64_t N, int64_t P, int64_t ldx,
                  const double* a, const double* s, double divisor,
                  double* out, void* stream);

/* Integer updates: numpy keeps `layer * n` and the np.add fold in the integer
 * dtype (wrapping) and true-divides into float64 (fed_avg_aggregator.py:33,39).
 * a = integer cardinalities [device, int64]; out float64. */
int fa_fedavg_i32(const int32_t* X, int64_t N, int64_t P, int64_t ldx,
                  const int64_t* a, double divisor, double* out, void* stream);
int fa_fedavg_i64(const int64_t* X, int64_t N, int64_t P, int64_t ldx,
                  const int64_t* a, double divisor, double* out, void* stream);

/* ---- host staging: page-locked documents and direct DMA ---------------------
 * A result store that keeps documents in page-locked memory lets the ingest
 * DMA each client's layers straight from the document into the device chunk,
 * with no host-side packing copy (fedlesscan_amd/ingest.py, store.py).
 *   fa_host_is_pinned: 1 if [p, p+n) lies inside ONE page-locked host
 *     allocation known to the HIP runtime (hipHostMalloc, hipHostRegister,
 *     torch pinned memory), else 0.  Never fails.
 *   fa_host_alloc / fa_host_free: hipHostMalloc / hipHostFree.
 *   fa_copy_h2d: hipMemcpyAsync host -> device of n bytes on stream. */
int fa_host_is_pinned(const void* p, int64_t n);
int fa_host_alloc(void** p, int64_t n);
int fa_host_free(void* p);
int fa_copy_h2d(void* dst, const void* src, int64_t n, void* stream);

/* ---- single-process multi-GPU ------------------------------------------------
 * The reference calls the strategy in-process, once per round
 * (aggregation.py:71-97).  The multi-GPU drop-in (fedlesscan_amd/multigpu.py)
 * folds one column bucket per GPU in that same process and reassembles the
 * model on one of them:
 *   fa_copy_peer: n bytes from src (on src_device) to dst (on dst_device),
 *     hipMemcpyPeerAsync over xGMI, enqueued on `stream` (normally the source
 *     GPU's stream that produced src, so it runs after that fold).  Peer
 *     access is enabled both ways the first time a pair is used.
 * Every compute entry above runs on the GPU that owns its stream, whatever
 * device the calling thread has current. */
int fa_copy_peer(void* dst, int dst_device, const void* src, int src_device, int64_t n, void* stream);

/* ---- native streaming ingest: host rows -> pinned slots -> DMA -> chunked fold --
 * The strategies' aggregate() (fed_avg_aggregator.py:57-92,
 * stall_aware_aggregation.py:82-117) decodes every client and then folds; here
 * each decoded row is handed over as it is decoded.  A process-wide pool of
 * copy workers packs rows into `slots` page-locked chunks of about chunk_bytes
 * (whole rows, pitch P rounded up to 64 floats); one issuer thread per pipe
 * sends each full chunk with one DMA on the pipe's copy stream and folds it on
 * the round's compute stream with fa_fold_f32, chunks in row order, the
 * accumulator carried across them: bit-identical to fa_fedavg_f32 over all
 * rows.  A chunk slot is refilled only after its fold has completed.
 *   fa_ingest_create:  allocate a pipe for models of P floats on `device`
 *   fa_ingest_begin:   start a round folding into acc [device, P] on `stream`;
 *                      expected_rows = the round's row count if known (0: not):
 *                      the first chunks hold 1, 2, 4, ... rows and, with the
 *                      count known, the last ones at most half of what is left,
 *                      so neither the start nor the tail waits for a full chunk
 *   fa_ingest_add:     one client row [host]: n pieces (srcs[i], sizes[i] bytes)
 *                      that concatenate to P floats, its factors a = fl32(n_i)
 *                      and s = fl32(score) when has_s (every row or none).  The
 *                      pieces must stay valid until fa_ingest_finish returns.
 *   fa_ingest_finish:  fold the last chunk and divide by `divisor`; returns when
 *                      every copy is done and every DMA and fold is enqueued
 *                      (the caller waits on `stream` for the result); after an
 *                      error it returns once no copy reads the pieces any more
 *   fa_ingest_destroy: wait for outstanding copies, free everything.
 * The pipe is reusable round after round (begin ... finish).  A begin after a
 * round that was abandoned (an add failed, or finish never came) drains that
 * round first (its queued chunks are not folded) and drops its partly filled
 * chunk, so none of its rows join the new round. */
typedef struct fa_ingest fa_ingest;
int fa_ingest_create(fa_ingest** pipe, int64_t P, int64_t chunk_bytes, int slots, int device);
int fa_ingest_rows_per_chunk(const fa_ingest* pipe);
int fa_ingest_begin(fa_ingest* pipe, float* acc, void* stream, int64_t expected_rows);
int fa_ingest_add(fa_ingest* pipe, const void* const* srcs, const int64_t* sizes, int64_t n, float a, float s,
                  int has_s);
int fa_ingest_finish(fa_ingest* pipe, float divisor);
int fa_ingest_destroy(fa_ingest* pipe);

/* ---- host-side ingest (no GPU): NPZ wire format -> pinned staging ----------
 * Client blobs are uncompressed NPZ archives (NpzWeightsSerializer,
 * serialization.py:280-306, written by the client, client.py:186-199). */
enum fa_dtype { FA_DT_F32 = 1, FA_DT_F64 = 2, FA_DT_I32 = 3, FA_DT_I64 = 4, FA_DT_F16 = 5,
                FA_DT_U8 = 6, FA_DT_I8 = 7, FA_DT_BOOL = 8 };
/* [host] Index the .npy members of an NPZ blob in archive order (= the order
 * of list(np.load(f).values()), serialization.py:304-306): payload byte offset,
 * element count, fa_dtype, ndim and shape (8 slots per layer).  Returns the
 * number of layers, or -1 when the blob must go through np.load instead
 * (compressed member, Fortran order, big-endian/object dtype, malformed, or
 * more than max_layers members).  All arrays are [host] with max_layers slots. */
int fa_npz_index(const uint8_t* blob, int64_t len, int64_t* offsets, int64_t* counts, int32_t* dtypes,
                 int32_t* ndims, int64_t* shapes, int max_layers);
/* [host] Copy n byte ranges: srcs[i] (sizes[i] bytes) -> dst + dst_offsets[i],
 * split by bytes over up to nthreads threads (0 = hardware concurrency).  The
 * pinned-staging packer of the ingest pipeline (fedlesscan_amd/ingest.py). */
int fa_pack(void* dst, const int64_t* dst_offsets, const void* const* srcs, const int64_t* sizes, int64_t n,
            int nthreads);
/* [host] zlib-compatible CRC-32 of data[0..n) continuing crc_in (0 to
 * start), split over up to nthreads threads (0 = hardware concurrency);
 * *crc_out = zlib.crc32(data, crc_in).  The member checksum of the NPZ writer
 * (fedlesscan_amd/npz.py write_npz: the saved round+1 model, aggregation.py
 * :139-147 -> NpzWeightsSerializer.serialize, serialization.py:290-296). */
int fa_crc32(const void* data, int64_t n, uint32_t crc_in, int nthreads, uint32_t* crc_out);

/* ---- host-side ingest (no GPU): the persisted BSON document -----------------
 * The reference stores each ClientResult as bson.encode(result.dict()) in
 * GridFS (client_daos.py:73) and reads it back with
 * ClientResult.parse_obj(bson.decode(file.read())) (client_daos.py:142), a
 * decode that copies the NPZ blob.  fa_bson_elements replaces the walk inside
 * bson.decode for one document level: for the document starting at
 * buf[doc_off] it reports, per element in order, the type byte, the name
 * (offset, length without NUL) and the value (offset, length):
 *   string/code/symbol -> the UTF-8 bytes without NUL; binary -> the payload
 *   (subtype in subtypes[], old subtype 2 unwrapped); document/array -> the
 *   embedded document itself (walk it with doc_off = its offset); fixed-size
 *   scalars -> their 1/4/8/12/16 bytes; null/undefined/min/max key -> length 0.
 * Offsets are relative to buf.  Returns the element count (only the first
 * max_elems are written; any output array may be NULL), or a negative
 * FA_BSON_* code.  Every length is bounds-checked against the enclosing
 * document. */
enum fa_bson_status { FA_BSON_MALFORMED = -1, FA_BSON_UNSUPPORTED = -2 };
int64_t fa_bson_elements(const uint8_t* buf, int64_t buf_len, int64_t doc_off, uint8_t* types,
                         int64_t* name_offs, int32_t* name_lens, int64_t* val_offs, int64_t* val_lens,
                         uint8_t* subtypes, int64_t max_elems);
/* [host] The whole tree of the document at buf[doc_off] in one call, in
 * pre-order: every element, then (for a document or array) its subtree.
 * parents[k] is the index of element k's enclosing document/array element, or
 * -1 at the top level; the other arrays as fa_bson_elements.  Nesting deeper
 * than 100 levels is FA_BSON_MALFORMED.  Returns the total element count. */
int64_t fa_bson_walk(const uint8_t* buf, int64_t buf_len, int64_t doc_off, uint8_t* types, int32_t* parents,
                     int64_t* name_offs, int32_t* name_lens, int64_t* val_offs, int64_t* val_lens,
                     uint8_t* subtypes, int64_t max_elems);

#ifdef __cplusplus
}
#endif
#endif /* FEDAVG_HIP_H */
