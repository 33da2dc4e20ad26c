/*
 * matcha_gossip.h -- C ABI of the MI355X (gfx950) gossip hot path.
 *
 * Plain pointers and sizes only.  "dev" pointers are HIP device pointers; "host" pointers are
 * ordinary host memory.  `stream` is a hipStream_t passed as void* (0 = legacy default).
 * Every entry point returns MX_OK (0) or a negative MX_ERR_* code; mx_last_error() returns
 * a thread-local message describing the last failure.
 *
 * The reference is pure Python over mpi4py.  Each entry point names the
 * reference function(s) it replaces; the binding a maintainer would add on the reference side
 * (a ctypes stub) is in INTEGRATION.md.
 */
#ifndef MATCHA_GOSSIP_H
#define MATCHA_GOSSIP_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MX_OK 0
#define MX_ERR_INVALID (-1)   /* bad argument (shape, alignment, range)               */
#define MX_ERR_HIP (-2)       /* HIP runtime error                                     */
#define MX_ERR_RCCL (-3)      /* RCCL error                                            */
#define MX_ERR_RNG (-4)       /* MT19937 word stream exhausted by resample events      */
#define MX_ERR_UNSUPPORTED (-5)

/* ---------------------------------------------------------------- library */
const char* mx_version(void);
const char* mx_last_error(void);

/* ---------------------------------------------------------------- schedule (L2)
 * Per-iteration activation flags on the GPU, bit-exact with numpy's legacy global RNG.
 *
 * mx_flags_binomial replaces MatchaProcessor.set_flags (graph_manager.py:298-309):
 *   for m in 0..M-1: flags[:, m] = np.random.binomial(1, p[m], T)   (matching-major draws)
 * and, with M == 1 and the output ignored, the discarded draw of FixedProcessor.set_flags
 * (graph_manager.py:213).
 *   key_in/pos_in   numpy MT19937 state (np.random.get_state()[1:3]) before the draws (host)
 *   p               activation probabilities (host, float64[M]); NaN / negative -> 0 as
 *                   graph_manager.py:305-306 does; values > 1 are rejected
 *   flags_dev       uint8 [T][M] output, row t = active_flags[t]
 *   key_out/pos_out MT19937 state after the draws (host) -- hand back to np.random.set_state
 * Blocking (synchronises `stream`).
 */
int mx_flags_binomial(const uint32_t* key_in, int pos_in, const double* p, int M, int64_t T,
                      uint8_t* flags_dev, uint32_t* key_out, int* pos_out, void* stream);

/* Same, but forces the sequential (resample-aware) walk; used by tests to pin the fix-up path. */
int mx_flags_binomial_sequential(const uint32_t* key_in, int pos_in, const double* p, int M,
                                 int64_t T, uint8_t* flags_dev, uint32_t* key_out, int* pos_out,
                                 void* stream);

/* ---------------------------------------------------------------- round plans
 * Precomputes, for every iteration t of a device-resident flag table, the per-row neighbour
 * walk of decenCommunicator.averaging (communicator.py:99-117): for each local row r
 * (global worker row_base + r) the source slots of its active partners in ascending matching
 * order, its degree and selfweight f32(1 - degree * alpha).  Partners held by another rank
 * get receive-slab slots numbered in (matching asc, sender id asc) order -- the same order
 * mx_exchange_round posts its RCCL receives in.
 *   partner_dev  int32 [M][n_global]   (GraphProcessor.neighbors_info, graph_manager.py:157-180)
 *   owner_dev    int32 [n_global]      rank owning each worker; NULL = all local
 *   plan_dev     int32 [T][mx_plan_words(n_local, M)]
 * Plan record layout (int32 words): [0] any flag set, [1] n_remote, [2] mode
 *   bits (0 after mx_plan_build): bit 0 idle-row mode (mx_plan_set_idle), bit 1 receive slots in
 *   peer GPUs' memory (mx_plan_set_peer_reads), [3] 1 if the round has more than 156 distinct
 *   remote partners (not representable: mx_plan_build then returns MX_ERR_INVALID after one
 *   4-byte read-back and a stream synchronize at build time),
 *   [4, 4+n_local) degree, [4+n_local, 4+2n_local) selfweight (f32 bits),
 *   [4+2n_local + r*M + e] source slot of row r's e-th partner (slot < n_local: local row,
 *   slot >= n_local: receive slab row slot - n_local).
 */
int64_t mx_plan_words(int n_local, int M);
int mx_plan_build(const uint8_t* flags_dev, int64_t T, int M, const int32_t* partner_dev,
                  int n_global, const int32_t* owner_dev, int my_rank, int row_base,
                  int n_local, double alpha, int32_t* plan_dev, void* stream);

/* Idle rows of an active round (degree 0 while some matching is active).  The reference still
 * runs them through averaging: recv = zeros; recv.add_(x, alpha=1 - 0*alpha) (communicator.py:
 * 113-117), i.e. x = 0 + 1.0 * x, which is x itself except that -0.0 becomes +0.0 (and a
 * signalling NaN is quieted).  mode 0 (mx_plan_build's default): such rows are not touched -- no
 * HBM traffic for them, equal to the reference under IEEE ==.  mode 1: they are streamed and
 * rewritten as fma(1.0f, x, 0.0f), bit-identical to the reference.  Sets word [2] of every
 * record of a plan table built by mx_plan_build. */
int mx_plan_set_idle(int32_t* plan_dev, int64_t T, int n_local, int M, int mode, void* stream);

/* ---------------------------------------------------------------- the hot path
 * One decentralized averaging round, in place, for every local worker:
 *   y_r = fma(f32(1-d_r*alpha), x_r, fma(f32(alpha), x_{j_d}, ... fma(f32(alpha), x_{j_1}, 0)))
 * with the partners j_1..j_d in ascending matching order -- decenCommunicator.averaging +
 * prepare_comm_buffer + reset_model (communicator.py:87-131), with flatten_tensors /
 * unflatten_tensors (comm_helpers.py:12-56) fused away: the kernel reads and writes the
 * workers' tensors where they live.
 *   seg_ptrs_dev  float* [nseg][n_slots] device table: worker slot k's copy of tensor s.
 *                 Slots [0, n_local) are the local workers (read + written in place);
 *                 slots [n_local, n_slots) are receive-slab rows (read only).
 *   seg_len_dev   int64 [nseg] floats per tensor;  tile_off_dev int64 [nseg+1] prefix of
 *                 ceil(len / mx_mix_tile(n_slots)) per tensor (see mx_mix_layout);
 *                 total_tiles = tile_off[nseg] (host copy, sizes the grid)
 *   seg_vec_dev   uint8 [nseg]: 1 if every slot pointer of that tensor is 16-byte aligned
 *   plan_dev      plan table from mx_plan_build; iter selects the record
 * Rows with degree 0 are neither read nor written (unless mx_plan_set_idle asked for the
 * reference's 0 + 1.0 * x).  No-op when the record's flags are all 0.  1-156 slots (> 64, or
 * M > 32 matchings: the untuned mix_kernel_wide); mx_mix_tile returns 0 above that.
 */
int mx_mix_tile(int n_slots);
/* Tuning knobs of the mixing kernel (process-wide), by name:
 *   blocks_per_cu  persistent workgroups per CU (grid = CUs x this, capped by the tile count)
 *   unroll         16-byte accesses per lane per slot per iteration, n_slots <= 8: 1, 2 or 4
 *                  (register-indexed kernel), 1 or 2 (LDS kernel)
 *   nontemporal    streaming (non-temporal) load/store hints: 1 on, 0 off, 2 = auto (default: the row
 *                  kernel drops them for rows of 32-320 MB, about the Infinity Cache)
 *   prefetch       issue the next iteration's loads before mixing/storing the current one
 *   regidx         register-indexed kernel (no LDS) instead of the LDS-column one, n_slots <= 8
 *   chunked        single-segment layouts: equal contiguous chunk per workgroup (1) or tile stride (0)
 *   grid           > 0: exact persistent grid size (overrides blocks_per_cu); 0 = CUs x blocks_per_cu
 *   readlane_min   LDS kernel: slot-count classes >= this (16 / 32 / 64) fetch one step's slots with
 *                  one LDS read + v_readlane and keep short chains by select (default 32)
 *   rows           row-per-wave kernel (tile staged in LDS, each wave walks whole rows' own
 *                  partner lists): 2 = every slot count (default; <= 8 slots needs unroll 1 or 2),
 *                  1 = 9-64 slots only, 0 = never
 *   split          row kernel: sub-tiles of 256+ columns per layout tile, so short rows still
 *                  give every persistent workgroup work, and 2 for 8-16 slots on flat grids:
 *                  0 = auto (default), 1 / 2 / 4 = forced
 *                  (capped at 4 for 8/16 slots, 2 for 32, 1 for 64); layouts are unaffected
 *   flat_small     row kernel, 8-16 slots: rounds of at most flat_small x (CUs x blocks_per_cu) work items
 *                  launch one workgroup per item instead of the persistent grid (default 256;
 *                  0 = always persistent; ignored when grid > 0)
 *   mid_bpc        row kernel, 8 slots, rows of at most mid_tiles x CUs layout tiles (0.4-2M params): a
 *   mid_tiles      persistent grid of mid_bpc workgroups per CU instead of the flat one (defaults 4 / 8;
 *                  mid_bpc 0 = off)
 *   spec           row kernel, 8 local slots (no receive slots), flat grid, streaming hints, rounds
 *                  moving > 64 MB (with the auto hints: > 320 MB, e.g. 8 rows of > 10.5M params): a
 *                  round whose active local
 *                  rows the caller passed (mx_gossip_mix_packed's need_host) issues their first tile's
 *                  loads before it reads the plan record (1 on, default; 0 off)
 *   spec_wgpc      ... and runs at this many workgroups per CU, capped with dynamic LDS (default 5;
 *                  0 = as many as fit): fewer tiles in flight, each issued at once -- the headline
 *                  round 0.2700 -> 0.2637 ms on one box (tools/occ_sweep.py)
 *   spec_glds      ... staging those tiles by LDS-DMA (global_load_lds_dwordx4) instead of registers,
 *                  512-column sub-tiles (default 1; headline 0.2627 -> 0.2591 ms)
 *   mean_wgpc      mx_mean_rows_to's tile kernel on rounds moving > 64 MB: workgroups per CU (default
 *                  3; 0 = as many as fit) -- 8 x 25.6M in place 0.2796 -> 0.2590 ms (tools/occ_sweep.py)
 *   spec_launches  (mx_mix_get only) SPEC launches so far in this process, modulo 2^31
 *   ns48           33-48 slots: 1 = a 48-slot row-kernel class instead of the 64-slot one (default 0)
 *   rows_pf2       row kernel, persistent grids of 32-64 slots: two tiles' loads in flight instead of
 *                  one -- 1 on, 0 off, 2 auto (default): when at most 5/8 of the class's slots are
 *                  staged (a GPU's share of a big topology: few local rows, many received ones)
 *   rows_tpb       row kernel, 32-64-slot classes on unsplit tiles: workgroup size 256 (default) / 512 /
 *                  1024 -- the tile's items dealt to 4 / 8 / 16 waves (measured neutral, r3)
 *   wide_tpb       wide kernel: workgroup size 256 / 512 / 1024 (default 1024: 16 waves walk the rows of
 *                  one staged piece)
 *   wide_pf2       wide kernel, 1024-thread workgroups: two pieces' loads in flight (default 1)
 *   wide_lds_kb    wide kernel: LDS budget per staged piece, 8-158 KB (default 158: 64 x 4 columns of
 *                  every slot up to 156 slots); smaller -> narrower pieces, more workgroups per CU
 *   wide_per_cu    wide kernel: workgroups per CU cap, 0 = auto (LDS- and wave-limited, <= 4)
 *   wide_plan_lds  wide kernel: copy the round's plan record to LDS when that costs no occupancy
 *                  (default 1)
 * "unroll" changes the tile size: rebuild layouts (mx_mix_layout) after setting it.
 * mx_mix_get returns the current value (negative on an unknown key).
 * mx_mix_kernel_name: the kernel mx_gossip_mix launches for n_slots under the current knobs
 * ("mix_kernel_rows", "mix_kernel_reg", "mix_kernel" for <= 64 slots and <= 32 matchings;
 * "mix_kernel_wide" for 65-156 slots -- also used for any slot count when M > 32; "" when
 * n_slots > 156). */
int mx_mix_set(const char* key, int value);
int mx_mix_get(const char* key);
const char* mx_mix_kernel_name(int n_slots);
int mx_mix_layout(const int64_t* seg_len_host, int nseg, int n_slots, int64_t* tile_off_host);
int mx_gossip_mix(float* const* seg_ptrs_dev, const int64_t* seg_len_dev,
                  const int64_t* tile_off_dev, const uint8_t* seg_vec_dev, int nseg,
                  int64_t total_tiles, int n_slots, const int32_t* plan_dev, int64_t iter,
                  int n_local, int M, float alpha, void* stream);
/* The same call with its per-group arguments packed once (a round of a launch-bound row pays the
 * host cost of converting 13 arguments per call, ~1 us of a ~4 us launch from Python): `call` is
 * an mx_mix_call the caller built and keeps alive; the same bits as mx_gossip_mix.
 *   need_host  optional (NULL = none): host uint64 [n_iters], bit r set when local row r is read
 *              and written in round t (degree > 0, or any row of an active round in idle mode 1)
 *              -- the plan record's own row set, known on the host from its copy of the flags.
 *              With it, 8-slot rounds of large rows load those rows' first tile before the plan
 *              record arrives (mx_mix_set "spec" / "spec_wgpc"); a bit missing or extra costs time,
 *              never bits (the record still decides what is mixed).  iter must be < n_iters. */
typedef struct mx_mix_call {
    float* const* seg_ptrs_dev;
    const int64_t* seg_len_dev;
    const int64_t* tile_off_dev;
    const uint8_t* seg_vec_dev;
    const int32_t* plan_dev;
    int64_t total_tiles;
    int32_t nseg, n_slots, n_local, M;
    float alpha;
    int32_t pad_;
    const uint64_t* need_host;
    int64_t n_iters;
} mx_mix_call;
int mx_gossip_mix_packed(const mx_mix_call* call, int64_t iter, void* stream);
/* Graph-replayable form: the round is read on the device from *iter_dev (int64) when the kernel
 * runs, so one captured launch (hipStreamBeginCapture / torch.cuda.graph) serves every
 * iteration; a counter outside [0, n_iters) makes the launch a no-op.  mx_iter_advance adds `by`
 * to the counter on the stream (capture it after the mix). */
int mx_gossip_mix_at(float* const* seg_ptrs_dev, const int64_t* seg_len_dev,
                     const int64_t* tile_off_dev, const uint8_t* seg_vec_dev, int nseg,
                     int64_t total_tiles, int n_slots, const int32_t* plan_dev, const int64_t* iter_dev,
                     int64_t n_iters, int n_local, int M, float alpha, void* stream);
int mx_iter_advance(int64_t* iter_dev, int64_t by, void* stream);
/* K rounds per replay with one bookkeeping launch: ctrs[j] = *iter_dev + j (j < n), then
 * *iter_dev += n, all on the device; the n mx_gossip_mix_at launches captured after it read
 * &ctrs[0] .. &ctrs[n-1].  Same rounds as n (mix_at + advance-by-1) pairs, half the launches. */
int mx_iter_expand(int64_t* iter_dev, int64_t* ctrs, int n, void* stream);

/* ---------------------------------------------------------------- flatten / unflatten
 * mx_gather replaces flatten_tensors (comm_helpers.py:12-30): flat[off[s] + i] = src[s][i].
 * mx_scatter is the copy_ loop of reset_model over unflatten_tensors views
 * (communicator.py:124-131, comm_helpers.py:33-56): dst[s][i] = flat[off[s] + i].
 *   ptrs_dev  float* [nseg] device;  off_dev int64 [nseg+1] device (off[nseg] = total)
 */
int mx_gather(const float* const* ptrs_dev, const int64_t* off_dev, int nseg, int64_t total,
              float* flat, void* stream);
int mx_scatter(float* const* ptrs_dev, const int64_t* off_dev, int nseg, int64_t total,
               const float* flat, void* stream);

/* ---------------------------------------------------------------- ChocoSGD (compressors.py)
 * mx_topk_abs_diff: q = topk(|x - x_hat|, k) of compressors.get_top_k (compressors.py:3-19)
 * applied to the send buffer of ChocoCommunicator.prepare_comm_buffer (communicator.py:188-190).
 * Writes vals[k] = (x - x_hat)[idx] and idx[k] (int64) sorted by index.  Among equal
 * magnitudes at the k-th threshold the lowest indices are taken (torch.topk(sorted=False)
 * leaves that unspecified).  x_hat may be NULL (treated as zeros: get_top_k on x itself).
 * `work` is a 256-byte aligned device scratch of mx_topk_work_bytes(P) bytes, ZERO-FILLED before
 * its first use (hipMemset); every call leaves its histograms and counters zero again, so no
 * zeroing launch runs per call.  One scratch may serve calls of any P.
 * One full pass over x / x_hat: a sampled top-digit histogram picks a candidate floor, one
 * streaming pass keeps the keys above it, and the exact radix select runs on those only (a
 * too-high floor is detected on the device and the pass re-run keeping every key: the result
 * is exact in every case).
 */
size_t mx_topk_work_bytes(int64_t P);
/* Top-k knobs: "sample_stride" = sample every S-th 1024-element chunk for the candidate floor
 * (0 = auto, about 2^18 sampled elements per row; 1 = exact full histogram, no sampling);
 * "compact_blocks" = persistent workgroups of the full pass, over all rows (0 = auto: 640 for
 * one row, 2560 for several);
 * "sample_pieces" = sampled 1024-element pieces per wave of the sampling pass (default 1);
 * "cand_chunks" = candidate regions per wave of the candidate-histogram / mark passes (0 = auto:
 * 4 for one row, 8 for several);
 * "compact_store" = 1 (default): candidate stores looped over each lane's kept elements, 0: one
 * masked store pair per element;
 * "apply_nt" = mx_choco_apply's access hints: -1 (default) non-temporal with several rows only,
 * 0 / 1 forced;
 * "apply_pf" = 1 (default): mx_choco_apply prefetches every message's tile bounds and first entries
 * under the tile stream, 0: the plain kernel (bounds and entries loaded per message);
 * "apply_persist" = -1 (default): the slot-table apply (mx_choco_apply_slots) of ONE row runs
 * persistent workgroups that acquire and load the message addresses once each, every other apply
 * a workgroup per tile; 0 / 1: one form for all;
 * "select" = 0 (default): the selection after the compaction as four passes (candidate histograms
 * of the 10 and 9 low digits, threshold mark, placement), 1: as ONE launch (select_kernel: B
 * workgroups of 1024 threads per row meeting at two row barriers; measured slower);
 * "fine_floor" = 1 (default): the sampled floor refined to 1/64 of a top digit (key bits 13..18)
 * when it falls in a 4-digit window around the previous call's floor digit on the same scratch (the
 * sampling pass histograms that window's sub-bins too): ~1.35 k candidates instead of 1.5-4 k;
 * 0: the floor is a whole top digit;
 * "floor_hint" = -1 (default): the compaction's candidate floor from a sampled histogram (one
 * sampling launch per call); m >= 0: from the PREVIOUS call's exact k-th key on the same scratch,
 * lowered by an adaptive per-row margin starting at m 12-bit bins (1 bin = 1/16 octave), and no
 * sampling launch -- the first call on a scratch keeps every key; a floor too high re-runs the
 * compaction keeping every key (the fallback), so results never change;
 * "select_blocks" = select_kernel workgroups per row (0 = auto: the fewest whose LDS caches every
 * candidate region, at most 32); "select_trace" = 1: select_kernel stores stage clocks in the
 * scratch (diagnostic, tools/select_trace.py).
 * Knobs tune speed only, never results -- except the test knob "spin_ticks": the bounded row-barrier
 * waits' deadline in 100 MHz ticks (default 2^28, ~2.7 s); 0 makes every wait that has to wait
 * expire, so tests can drive the error path below on purpose.  "spin_ticks" and "compact_trace"
 * live on the device: they apply to the CURRENT device only (set them per device in a process
 * driving several), and mx_topk_get reports the current device's value; every other knob is host-side.
 * mx_topk_get also reads "hist_grid" (the last call's first-candidate-pass grid per row) and
 * "hist_capacity" (the co-resident block cap that grid was held to with sampling on, 0 without). */
int mx_topk_set(const char* key, int64_t value);
int64_t mx_topk_get(const char* key);
/* The rows' sticky error words: a row barrier (the sampled-floor fallback of the first candidate
 * pass, or select_kernel) whose BOUNDED wait expired -- its blocks were not all resident -- leaves
 * that call's output undefined instead of hanging the GPU.  Synchronises `stream`, reads and clears
 * the words; MX_ERR_HIP if any was set.  (work, work_ld_bytes, nrows, P) as in the call checked. */
int mx_topk_check(void* work, int64_t work_ld_bytes, int nrows, int64_t P, void* stream);
/* The same scan, stream-ordered and NON-blocking: the words are read and cleared on `stream` behind
 * the call they belong to, and an expired one sets *flag_dev = first row + 1 with a system-scope
 * release (flag_dev: mx_host_words -- the host polls it without synchronising).  compressors.get_top_k
 * on GPU tensors enqueues it after every call and raises at the next call, or at check_top_k(). */
int mx_topk_err_forward(void* work, int64_t work_ld_bytes, int nrows, int64_t P, int32_t* flag_dev, void* stream);
/* Diagnostics of the candidate floor, per row r: out[5r] = calls made on this scratch, out[5r+1] =
 * how many of them ran the fallback compaction (floor above the k-th key), out[5r+2] = the row's
 * current floor_hint margin (bins), out[5r+3] = the last call's threshold key (bits of |k-th value|),
 * out[5r+4] = its candidate count.  Synchronises `stream`. */
int mx_topk_stats(const void* work, int64_t work_ld_bytes, int nrows, int64_t P, int64_t* out, void* stream);
/* Diagnostic: with mx_topk_set("compact_trace", 1), every workgroup of row 0's candidate compaction
 * stamps the 100 MHz constant clock at its start, once its floor is resolved, and at its end;
 * out[3b .. 3b+2] = workgroup b's stamps of the last launch (nblocks <= 8192).  Synchronises the
 * device.  tools/compact_trace.py reads it (ramp vs tail of the one-row compaction). */
int mx_topk_trace(uint64_t* out, int64_t nblocks);
int mx_topk_abs_diff(const float* x, const float* x_hat, int64_t P, int64_t k, float* vals,
                     int64_t* idx, void* work, void* stream);
/* Batched form (one set of launches for every local worker): row r reads x + r*ld (and
 * x_hat + r*ld), writes its values at out + r*out_ld_bytes and its int64 indices at
 * out + r*out_ld_bytes + idx_off_bytes, and uses work + r*work_ld_bytes
 * (work_ld_bytes >= mx_topk_work_bytes(P)).  bnd_off_bytes >= 0: also writes the message's
 * int32 tile bounds there (bnd[t] = first output entry with index >= 4096 t, t = 0..ceil(P/4096);
 * the layout mx_choco_apply reads); < 0: not written. */
int mx_topk_abs_diff_rows(const float* x, const float* x_hat, int64_t ld, int nrows, int64_t P,
                          int64_t k, void* out, int64_t out_ld_bytes, int64_t idx_off_bytes,
                          int64_t bnd_off_bytes, void* work, int64_t work_ld_bytes, void* stream);

/* ChocoCommunicator.averaging (communicator.py:200-230) for one round of n_local workers,
 * in place on the state rows (a round whose flags are all zero must not be applied):
 *   for each partner j of row r (ascending matching): s_r[idx_j] = s_r[idx_j] + f32(alpha)*v_j
 *   s_r[idx_r] += f32(1-d*alpha) * v_r ; x_hat_r[idx_r] += v_r
 *   x_r = fma(gamma, s_r, x_r) ; x_r = fma(-gamma, x_hat_r, x_r)
 *   x/xhat/s  float [n_local][P] rows with stride ld (floats)
 *   msgs      compressed messages, one per plan slot, msg_ld_bytes apart: a slot holds
 *             vals float[k] at +0, idx int64[k] at +4*round_up(k, 2) and the tile bounds int32
 *             [ceil(P/4096) + 1] right after the indices (mx_choco_msg_bytes(P, k) bytes, written
 *             by mx_topk_abs_diff_rows with bnd_off_bytes = 4*round_up(k, 2) + 8*k); slots
 *             [0, n_local) are the local rows' own messages, the rest received ones
 *   work      unused (the tile bounds travel in the messages); may be NULL
 * One fused pass: per 4096-element tile of a row, s and x_hat are staged in LDS, every message
 * entry in the tile is applied there in the order above, x is updated, and only the touched
 * 64-byte granules of s / x_hat are written back.
 */
int64_t mx_choco_msg_bytes(int64_t P, int64_t k);
/* Scratch of mx_choco_apply: 0 bytes (kept for ABI stability). */
size_t mx_choco_apply_work_bytes(int64_t P, int n_slots);
int mx_choco_apply(float* x, float* xhat, float* s, int64_t ld, int64_t P, int64_t k,
                   const void* msgs, int64_t msg_ld_bytes, int n_slots, const int32_t* plan_dev,
                   int64_t iter, int n_local, int M, float alpha, float gamma, void* work,
                   void* stream);
/* Graph-replayable form (as mx_gossip_mix_at): the round is *iter_dev, read on the device; a
 * round outside [0, n_iters) or with no active matching leaves x, x_hat and s untouched. */
int mx_choco_apply_at(float* x, float* x_hat, float* s, int64_t ld, int64_t P, int64_t k, const void* msgs,
                      int64_t msg_ld_bytes, int n_slots, const int32_t* plan_dev, const int64_t* iter_dev,
                      int64_t n_iters, int n_local, int M, float alpha, float gamma, void* work, void* stream);
/* The pull transport's form (ChocoWorkerGroup under PullTransport; replaces the sendrecv of the
 * compressed messages, communicator.py:214, with loads from the owners' HBM): message `slot` is
 * read at the device address slot_ptrs_dev[slot] (int64 [n_slots]) -- the local rows' messages in
 * this GPU's buffer, the partners' in their owners' IPC-mapped snapshot buffers (mx_snapshot_publish
 * of the message slots, then mx_pull_gate with ld_bytes = the message stride points the remote
 * slots there).  A plan record with the peer-reads bit (mx_plan_set_peer_reads) makes every
 * workgroup acquire at system scope before its first message load.  Same bits as mx_choco_apply. */
int mx_choco_apply_slots(float* x, float* xhat, float* s, int64_t ld, int64_t P, int64_t k,
                         const int64_t* slot_ptrs_dev, int n_slots, const int32_t* plan_dev, int64_t iter,
                         int n_local, int M, float alpha, float gamma, void* stream);

/* ---------------------------------------------------------------- cross-GPU exchange (RCCL)
 * One process per GPU; workers partitioned by owner[].  mx_exchange_round posts, inside one
 * ncclGroupStart/End, an ncclSend of every local row whose active partner lives on another
 * rank (once per destination rank) and an ncclRecv of every distinct remote partner row into
 * the receive slab -- the pairwise comm.sendrecv of decenCommunicator.averaging
 * (communicator.py:110) over xGMI, with each row crossing a link at most once per round.
 * Order: first appearance over (matching ascending, sender worker id ascending); slab slot k
 * is the k-th distinct remote worker in that order (matches mx_plan_build).
 *   flags_row  uint8 [M] host;  partner int32 [M][n_global] host;  owner int32 [n_global] host
 *   rows       device float* [n_local] (host array of device pointers), P floats each
 *   slab       device base; slot k at slab + k * slab_ld
 *   elem_bytes 4 for fp32 rows; also used with 12-byte Choco messages (values + int64 idx)
 */
int mx_rccl_unique_id(void* id_out /* 128 bytes */);
int mx_rccl_init(const void* id /* 128 bytes */, int nranks, int rank, void** comm_out);
/* The communicator is NON-blocking (ncclConfig_t.blocking = 0) and every RCCL call the library
 * makes on it waits for its enqueue against a deadline: a peer rank that never joins (dead, or
 * skipped the call) turns into MX_ERR_RCCL "timed out" instead of a hang.  mx_rccl_init uses
 * $MX_RCCL_TIMEOUT_S (default 300 s); mx_rccl_init_timeout takes it explicitly (the deadline then
 * applies to the init and to every later operation of the process).  An init that times out is
 * aborted before returning; *nonblocking_out (optional) = 1.  Replaces the mpi4py COMM_WORLD set
 * up at train_mpi.py:237-239. */
int mx_rccl_init_timeout(const void* id, int nranks, int rank, int64_t timeout_ms, void** comm_out,
                         int* nonblocking_out);
/* ncclCommAbort: release a communicator whose peers are gone (after a timed-out operation). */
int mx_rccl_abort(void* comm);
/* ncclCommFinalize (waited for with the deadline; aborted on expiry) + ncclCommDestroy. */
int mx_rccl_destroy(void* comm);
/* ncclCommCount: the ranks the communicator holds (the bench line's rccl_ranks). */
int mx_rccl_count(void* comm, int* nranks_out);
/* The deadlines above bound getting an operation enqueued (init, a group's connection setup).
 * A peer that dies or skips an exchange after the connections exist leaves the RCCL kernel
 * waiting on the GPU; mx_rccl_wait is the stream synchronisation with a deadline: an event behind
 * everything enqueued on `stream`, polled until it completes or timeout_ms (<= 0: the init's
 * deadline) passes -- then the communicator is ABORTED (its kernels exit, the stream drains; do not
 * use it again) and MX_ERR_RCCL "timed out" is returned.  Replaces the blocking barriers that
 * bracket averaging (communicator.py:94,119). */
int mx_rccl_wait(void* comm, void* stream, int64_t timeout_ms);
/* The ordered operations mx_exchange_round posts for this rank, host only (no GPU, no RCCL):
 * ops[4i..4i+3] = {kind (0 send / 1 recv), peer rank, local row (send) or slab slot (recv),
 * global id of the worker whose row travels}.  ops == NULL: count only. */
int mx_exchange_plan(const uint8_t* flags_row, int M, const int32_t* partner, int n_global,
                     const int32_t* owner, int my_rank, int row_base, int n_local, int32_t* ops,
                     int cap, int* n_ops);
/* Posts an explicit operation list (mx_exchange_plan's layout) inside one ncclGroupStart/End:
 * kind 0 = ncclSend of rows[op[2]] to op[1], kind 1 = ncclRecv from op[1] into slab slot op[2];
 * row_bytes per operation.  Sends to / receives from one peer pair up in list order.  Every op is
 * validated before anything is posted.  mx_exchange_round = mx_exchange_plan + this. */
int mx_exchange_post(void* comm, const int32_t* ops, int n_ops, void* const* rows, int n_rows, void* slab,
                     int64_t slab_ld_bytes, int64_t row_bytes, void* stream);
int mx_exchange_round(void* comm, const uint8_t* flags_row, int M, const int32_t* partner,
                      int n_global, const int32_t* owner, int my_rank, int row_base, int n_local,
                      void* const* rows, void* slab, int64_t slab_ld_bytes, int64_t row_bytes,
                      int* n_remote_out, void* stream);
/* Pull transport (one process per GPU of a node): device buffers shared through IPC handles
 * (64 bytes, mx_ipc_handle_bytes).  A rank publishes snapshots of its rows in an mx_ipc_alloc
 * buffer and sends the handle to its peers (any host channel); a peer mx_ipc_open's it and the
 * mixing kernel reads the partner rows straight from the owner's HBM over xGMI, in place of
 * comm.sendrecv (communicator.py:110).  mx_ipc_close unmaps a peer buffer, mx_ipc_free releases
 * one's own. */
/* Snapshot of this GPU's rows for its peers: dst[i] = src[i] (n floats, n % 4 == 0, 16-byte
 * aligned), and every workgroup ends with a system-scope release (its stores written back past
 * this GPU's L2 to HBM), so a peer's load over xGMI after the round's barrier sees them. */
int mx_snapshot_publish(const float* src, float* dst, int64_t n, void* stream);
/* The same copy for only the rows a peer reads this round: local row r
 * (0 <= r < n_local, worker row_base + r) is copied -- src + r * src_ld -> dst + r * dst_ld, n floats
 * (multiple of 4, all 16-byte aligned), then the system-scope release -- iff some matching g with
 * flags_row_dev[g] != 0 pairs it with a worker outside [row_base, row_base + n_local) (partner_dev
 * int32 [M][n_global]: the set mx_pull_gate's peers point their slots at); other rows are not
 * touched.  One launch, n_local rows of workgroups; the row test runs on the device. */
int mx_snapshot_publish_rows(const float* src, int64_t src_ld, float* dst, int64_t dst_ld, int64_t n, int n_local,
                             const uint8_t* flags_row_dev, int M, const int32_t* partner_dev, int n_global,
                             int row_base, void* stream);
/* Plan word [2] bit 1: the receive slots of these records point at peer GPUs' IPC-mapped memory;
 * the mixing kernels then start with a system-scope acquire per workgroup (buffer_inv sc0 sc1: no
 * line of a peer's buffer cached on this GPU from an earlier round is served).  on = 1 / 0. */
int mx_plan_set_peer_reads(int32_t* plan_dev, int64_t T, int n_local, int M, int on, void* stream);
/* A rank's snapshot buffer (mx_ipc_alloc, zero-filled): MX_PULL_HEADER_BYTES of header -- its
 * uint64 epoch at offset 0 -- then snapshot 0 and snapshot 1, each n_local rows of ld_bytes. */
#define MX_PULL_HEADER_BYTES 256
typedef struct mx_pull_rank {
    int64_t base;      /* the rank's snapshot buffer as mapped in THIS process (own: the allocation) */
    int32_t row_base;  /* its block of workers [row_base, row_base + n_local) */
    int32_t n_local;
} mx_pull_rank;
/* The pull round's handshake, one single-wave kernel on `stream` between mx_snapshot_publish (into
 * snapshot `parity`) and the mixing launch -- replaces the host synchronize + barrier + pointer-table
 * copy per round (and the reference's sendrecv pairing, communicator.py:99-112):
 *   1. epoch[my_rank] = epoch (system-scope release; the snapshot is complete by stream order);
 *   2. bounded wait for epoch[r] >= epoch of every rank r owning an active remote partner of a
 *      local worker under flags_row_dev (this round) or prev_row_dev (the previous pull round);
 *   3. slot_ptrs_dev[n_local + j] = the j-th distinct remote partner's row in its owner's snapshot
 *      `parity` (plan_kernel's slot numbering); prev_row_dev = flags_row_dev afterwards.
 * ranks_dev: mx_pull_rank[nranks] (device).  On expiry after timeout_s: err_dev[0] = 1, [1] = the
 * rank that did not publish, [2] = the epoch awaited, [3] = the last one seen (err_dev: mx_host_words,
 * read by the host once the stream has passed the gate); err_dev[0] = 2: more remote partners than
 * slots.  1 <= n_global <= 4096, nranks <= 64, epochs start at 1 and rise by one per pull round. */
int mx_pull_gate(const uint8_t* flags_row_dev, uint8_t* prev_row_dev, int M, const int32_t* partner_dev,
                 int n_global, const int32_t* owner_dev, const mx_pull_rank* ranks_dev, int nranks, int my_rank,
                 int row_base, int n_local, int64_t ld_bytes, int parity, uint64_t epoch, int64_t* slot_ptrs_dev,
                 int n_slots, double timeout_s, int32_t* err_dev, void* stream);
/* The pull round's fetch of small payloads (ChocoWorkerGroup: the partners' compressed messages,
 * in place of the sendrecv of communicator.py:214), on `stream` after mx_pull_gate: for every remote
 * slot j below the round's remote count (word [1] of plan_rec_dev, the round's plan record), the
 * first nbytes (rounded up to 16) at slot_ptrs_dev[n_local + j] -- a peer's snapshot row -- are
 * copied to dst + j * dst_ld (dst_ld >= that, 16-byte aligned).  Every workgroup acquires at system
 * scope first.  Grid: up to 64 workgroups per slot times max_remote slots. */
int mx_pull_fetch(const int64_t* slot_ptrs_dev, int n_local, int max_remote, const int32_t* plan_rec_dev, void* dst,
                  int64_t dst_ld, int64_t nbytes, void* stream);
/* n zeroed int32 words of coherent mapped host memory: *host_out for the host, *dev_out for kernels. */
int mx_host_words(int n, int32_t** host_out, int32_t** dev_out);
int mx_host_words_free(int32_t* host);
int mx_ipc_handle_bytes(void);
/* A zero-filled device buffer of at least `bytes` whose IPC handle is exported: the size is rounded up
 * to the export granule (default 2 MiB).  hipIpcGetMemHandle refuses ("invalid argument") a block
 * that lands on the address range of an IPC import this process has just closed
 * (tools/ipc_reuse_probe.py); such a block is kept while a second one -- necessarily elsewhere -- is
 * allocated and exported, then freed (knob "hold", default 1; counted as "recovered").  A block that
 * still cannot be exported is logged to stderr, counted (mx_ipc_stats) and returned as MX_ERR_HIP. */
int mx_ipc_alloc(int64_t bytes, void** ptr_out, void* handle_out);
/* Export accounting, process-wide since load: hipIpcGetMemHandle calls, and mx_ipc_alloc calls that
 * returned no exported block (engine.PullTransport reads them: the bench line's ipc_refused, the
 * multi-process tests' zero checks). */
int mx_ipc_stats(int* exports, int* refused);
/* mx_ipc_alloc's knobs: "granule" (bytes, 1 = unrounded .. 1 GiB), "hold" (1 / 0: recover a refused
 * block with a second one); mx_ipc_get returns them, and "recovered" (refused first blocks whose
 * second block exported); -1 for an unknown key.  Test hooks of tests/test_gpu_round6.py and the
 * refusal probe. */
int mx_ipc_set(const char* key, int64_t value);
int64_t mx_ipc_get(const char* key);
int mx_ipc_open(const void* handle, void** ptr_out);
int mx_ipc_close(void* ptr);
int mx_ipc_free(void* ptr);

/* centralizedCommunicator.averaging (communicator.py:56-67): buf = allreduce_sum(buf) / size.
 * mx_allreduce_mean: RCCL's all-reduce (ring / tree order of RCCL's choosing), then the division;
 *   equal to the reference within fp32 reassociation (1e-6 relative for well-conditioned sums).
 * mx_allreduce_mean_ordered: bit-identical to the reference -- every rank's buffer is
 *   all-gathered into `gather` (float[nranks][count], device) and each rank sums the rows in the
 *   reference's order (mx_mean_rows) and divides by nranks.  order 0: the binomial tree of
 *   mpi4py's object all-reduce (rc.fast_reduce, its default); 1: rank order (fast_reduce off). */
int mx_allreduce_mean(void* comm, float* buf, int64_t count, int nranks, void* stream);
int mx_allreduce_mean_ordered(void* comm, float* buf, int64_t count, float* gather, int order, void* stream);
/* ncclAllGather of `count` floats per rank into gather[nranks][count] (rank order). */
int mx_allgather(void* comm, const float* send, int64_t count, float* gather, void* stream);
/* out[i] = (rows[0][i] + ... + rows[nrows-1][i] in the given order) / nrows for i < count; rows
 * are nrows x ld floats (device), 1 <= nrows <= 2^24 (the tree order for any count: a binary counter
 * of partial sums); out may be rows[0].  The division step of
 * the centralized communicator (communicator.py:61-62) and of sync_allreduce (train_mpi.py:46-55),
 * callable after any transport's gather.  = mx_mean_rows_to with ndst = 1. */
int mx_mean_rows(const float* rows, int nrows, int64_t ld, int64_t count, int order, float* out, void* stream);
/* The same mean (same order, same rounding) written to ndst rows dst + d * dst_ld (d < ndst) in one
 * pass: centralizedCommunicator's all-reduce (communicator.py:56-67) / sync_allreduce (train_mpi.py:
 * 34-56) for workers held as rows of one arena -- dst == rows (dst_ld == ld) rewrites every worker's
 * row with the mean in place (each column of every row is read before that column is written);
 * after an mx_allgather, dst = this rank's own rows.  16-byte accesses when everything is 16-byte
 * aligned and the order is the <= 8-row tree or rank order; up to 8 rows in 512-column tiles
 * staged in LDS.  A dst that overlaps the rows other than at whole-row offsets (offset and dst_ld
 * multiples of ld) is refused (MX_ERR_INVALID). */
int mx_mean_rows_to(const float* rows, int nrows, int64_t ld, int64_t count, int order, float* dst, int ndst,
                    int64_t dst_ld, void* stream);
/* The kernel that carries the bulk of mx_mean_rows_to with the same arguments (static string, e.g.
 * "mean_tile_kernel<1>"; the same dispatch, alignment included; nothing launched), for reports. */
const char* mx_mean_kernel_name(const float* rows, int nrows, int64_t ld, int64_t count, int order, const float* dst,
                                int ndst, int64_t dst_ld);

/* ---------------------------------------------------------------- host: matching decomposition
 * nx.max_weight_matching (graph_manager.py:64, inside GraphProcessor.getSubGraphs 57-83) without
 * networkx: the blossom algorithm networkx 3.4.2 runs, in its visiting orders, so the same maximum
 * matching comes back.  Host memory, no GPU.  Nodes are 0..n-1 in the graph's node order; node v's
 * neighbours are adj[adj_off[v] .. adj_off[v+1]) in its adjacency order (each edge in both lists),
 * adj_w their integer weights (NULL: all 1).  mate_out[v] = partner or -1; order_out[0..*n_order)
 * = nodes in the order they first entered networkx's `mate` dict (its result set is built by
 * iterating that dict). */
int mx_max_weight_matching(int n, const int64_t* adj_off, const int32_t* adj, const int64_t* adj_w,
                           int maxcardinality, int32_t* mate_out, int32_t* order_out, int* n_order);

/* ---------------------------------------------------------------- utilities
 * splitmix64 -> fp32 uniform[-1,1) synthetic inputs, x[i] for counter i+1. */
int mx_synth_fill(float* dst, int64_t n, uint64_t seed, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MATCHA_GOSSIP_H */
