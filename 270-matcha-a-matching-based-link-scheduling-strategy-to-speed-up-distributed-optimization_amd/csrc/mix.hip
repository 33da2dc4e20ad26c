// mix.hip -- the hot path: one in-place decentralized averaging round over every local worker.
//
// Replaces, per round, decenCommunicator.prepare_comm_buffer / averaging / reset_model
// (communicator.py:87-131) together with flatten_tensors / unflatten_tensors
// (comm_helpers.py:12-56): the reference concatenates each worker's tensors, receives every
// active partner's full vector, accumulates recv = fma(alpha, x_j, recv) in ascending matching
// order, adds fma(1 - d*alpha, x_i, recv) and copies back.  Here the workers' tensors stay
// where they are (a [nseg][n_slots] pointer table; one segment per tensor, or one segment per
// flat arena row) and each 256-lane workgroup owns a column tile of EVERY slot:
//
//   1. stream the tile of each needed slot (local rows with degree > 0, received slab rows)
//      from HBM into registers with 16-byte loads -- every byte read once;
//   2. park them in a per-lane LDS column (LDS gives the data-dependent, wave-uniform row
//      indexing of the partner walk; each lane reads only its own column: no barrier);
//   3. per output row, run the reference FMA chain in matching order from LDS and store the
//      tile back in place with 16-byte stores -- every byte written once.
//
// Traffic per round = 2 * n_active * P * 4 bytes (+ n_remote * P * 4 read of the slab): the
// HBM roofline of the north star.  No MFMA: ~0.25 flop/byte.
//
// Scheduling: by default tiles (never straddling a tensor) are strided over a persistent grid,
// so at any moment the whole chip streams one narrow window of every row (DRAM row locality);
// optionally (knob "chunked") a single-segment layout is split into equal contiguous ranges.
// Three kernels share this contract (knob "rows" picks): the default row-per-wave kernel
// (mix_kernel_rows: the tile is staged in LDS by the whole workgroup, then each wave walks whole
// rows' own partner lists -- the fastest at every slot count), the register-indexed kernel for
// <= 8 slots (mix_kernel_reg: one register vector per lane indexed through s_set_gpr_idx, no
// LDS) and the LDS-column kernel (mix_kernel: per-lane columns, every row to the max degree).
#include "mx_common.h"

#include <atomic>
#include <cstdlib>
#include <type_traits>

namespace {
constexpr int kTPB = 256;
constexpr int kMaxM = 32;

// VEC-wide float vectors as clang ext vectors (16-byte global_load/store_dwordx4 for VEC = 4;
// the non-temporal builtins accept them)
template <int VEC>
struct VT;
template <>
struct VT<4> { typedef float type __attribute__((ext_vector_type(4))); };
template <>
struct VT<2> { typedef float type __attribute__((ext_vector_type(2))); };
template <>
struct VT<1> { typedef float type __attribute__((ext_vector_type(1))); };

// Row pointers arrive as generic pointers; accessing them through the global address space makes
// the compiler emit global_load/store (counted on vmcnt only) instead of flat_* (counted on vmcnt
// AND lgkmcnt, so every LDS or scalar-load wait in the loop would also drain the HBM stream).
template <typename F>
using GPtr = __attribute__((address_space(1))) F*;

template <bool NT, typename F>
__device__ __forceinline__ F ld(const float* p) {
    const GPtr<const F> g = (GPtr<const F>)(p);
    if constexpr (NT) return __builtin_nontemporal_load(g);
    else return *g;
}

template <bool NT, typename F>
__device__ __forceinline__ void st(float* p, const F& v) {
    const GPtr<F> g = (GPtr<F>)(p);
    if constexpr (NT) __builtin_nontemporal_store(v, g);
    else *g = v;
}

__device__ __forceinline__ float ld1(const float* p) { return *(GPtr<const float>)(p); }
// 16-byte accesses are legal at row + 4i when the row pointer itself is 16-byte aligned: a scalar
// test of the (wave-uniform) pointer, where the per-segment seg_vec byte would be a vector-memory
// load -- a full round trip at the head of every workgroup before its first tile load
__device__ __forceinline__ bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }
__device__ __forceinline__ void st1(float* p, float v) { *(GPtr<float>)(p) = v; }


// Plan record of this iteration, decoded into LDS (see mx_plan_build); returns the bit mask of
// slots that must be loaded, or 0 when every flag of the round is 0.  Rows of degree 0 are left
// untouched unless the record's idle word (mx_plan_set_idle) asks for the reference's
// `0 + 1.0 * x` (then they are streamed like any other row, with selfweight 1).
template <int NS>
struct PlanLds {
    int32_t w[mx::kPlanHeader + 2 * NS + NS * kMaxM];
};

// The round to mix: `iter`, or with iter_dev (graph-replayable launches) the device counter
// *iter_dev, `iter` then being the schedule length; outside [0, length) the launch is a no-op.
__device__ __forceinline__ int64_t round_of(int64_t iter, const int64_t* iter_dev) {
    if (!iter_dev) return iter;
    const int64_t v = *iter_dev;
    return (v >= 0 && v < iter) ? v : -1;
}

// Remote-slot load path (PullTransport, plan word [2] bit 1 -- mx_plan_set_peer_reads): the receive
// slots point at a peer GPU's IPC-mapped snapshot buffer, which this GPU's L2 holds as non-local
// (MTYPE NC) lines.  The same two snapshot buffers are re-read every other round, so a line cached
// here in round r - 2 could be served stale in round r: nothing on this GPU invalidates it when the
// peer rewrites its HBM (LLVM AMDGPUUsage, memory model GFX942 -- gfx950 shares it: only a
// system-scope acquire, buffer_inv sc0 sc1, "ensures that following loads will not see stale
// MTYPE NC global data").  So before the first load of any slot, one lane of every workgroup issues
// that acquire (invalidating its CU's L1 and the non-local lines of its XCD's L2) and waits for it,
// and the workgroup meets at a barrier (MI355X_MICROARCH.md, "Consumer, always").  Every later load
// of the launch is then fresh: the peer's snapshot was written back to its HBM by a system-scope
// release (mx_snapshot_publish) before the round's host barrier.  Cost: one invalidate per
// workgroup per round (~2 us), nothing per byte; rounds without peer slots skip it.
__device__ __forceinline__ void peer_acquire(int32_t mode_word) {
    if (mode_word & 2) {                         // block-uniform
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");       // system scope: buffer_inv sc0 sc1
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
    }
}

template <int NS>
__device__ __forceinline__ uint64_t load_plan(PlanLds<NS>& sp, const int32_t* plan, int64_t iter,
                                              int n_local, int M) {
    if (iter < 0) return 0;                      // block-uniform: no barrier is skipped unevenly
    const int64_t W = mx::plan_words(n_local, M);
    const int32_t* rec = plan + iter * W;
    for (int i = threadIdx.x; i < W; i += blockDim.x) sp.w[i] = rec[i];
    __syncthreads();
    if (sp.w[0] == 0) return 0;
    peer_acquire(sp.w[2]);
    const int n_remote = sp.w[1];
    const bool idle = (sp.w[2] & 1) != 0;
    const int32_t* deg = sp.w + mx::kPlanHeader;
    uint64_t need = 0;
    for (int r = 0; r < n_local; ++r)
        if (deg[r] > 0 || idle) need |= 1ull << r;
    for (int k = 0; k < n_remote; ++k) need |= 1ull << (n_local + k);
    return need;
}

// Where this lane works in the workgroup's i-th iteration.  A lane's u-th access covers columns
// [(g + u*256) * VEC, +VEC) of segment `seg`; columns >= lim are outside its range.
struct Sched {
    bool chunked;
    int nseg;
    const int64_t* seg_len;
    const int64_t* tile_off;
    int64_t total_tiles, gb, ge, niter;

    template <int VEC, int U>
    __device__ __forceinline__ void init(bool chunked_, int nseg_, const int64_t* seg_len_,
                                         const int64_t* tile_off_, int64_t total_tiles_) {
        chunked = chunked_;
        nseg = nseg_;
        seg_len = seg_len_;
        tile_off = tile_off_;
        total_tiles = total_tiles_;
        if (chunked) {   // equal contiguous group ranges per workgroup
            const int64_t G = (seg_len[0] + VEC - 1) / VEC;
            gb = (int64_t)blockIdx.x * G / gridDim.x;
            ge = ((int64_t)blockIdx.x + 1) * G / gridDim.x;
            niter = (ge - gb + U * kTPB - 1) / (U * kTPB);
        } else {         // tiles strided over the grid
            niter = total_tiles > blockIdx.x ? (total_tiles - blockIdx.x + gridDim.x - 1) / gridDim.x : 0;
        }
    }

    template <int VEC, int U>
    __device__ __forceinline__ void at(int64_t i, int& seg, int64_t& g, int64_t& lim) const {
        if (chunked) {
            seg = 0;
            g = gb + i * (U * kTPB) + threadIdx.x;
            const int64_t e = ge * VEC;
            lim = seg_len[0] < e ? seg_len[0] : e;
        } else {
            const int64_t tile = blockIdx.x + i * gridDim.x;
            int lo = 0, hi = nseg;
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (tile_off[mid] <= tile) lo = mid; else hi = mid;
            }
            seg = lo;
            g = (tile - tile_off[seg]) * (U * kTPB) + threadIdx.x;
            lim = seg_len[seg];
        }
    }
};

// one lane's U accesses of one slot: 16-byte vector loads when the whole span is in range and
// aligned, element loads (zero-filled beyond lim) otherwise
template <int VEC, int U, bool NT, typename F>
__device__ __forceinline__ void load_slot(F (&v)[U], const float* row, int64_t g, int64_t lim, bool vec_ok) {
    const bool full = vec_ok && (g + (U - 1) * kTPB) * VEC + VEC <= lim;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t c = (g + (int64_t)u * kTPB) * VEC;
        if (full) {
            v[u] = ld<NT, F>(row + c);
        } else {
#pragma unroll
            for (int j = 0; j < VEC; ++j) v[u][j] = (c + j < lim) ? ld1(row + c + j) : 0.0f;
        }
    }
}

template <int VEC, bool NT, typename F>
__device__ __forceinline__ void store_one(float* row, int64_t c, int64_t lim, bool full, const F& a) {
    if (full) {
        st<NT, F>(row + c, a);
    } else {
#pragma unroll
        for (int j = 0; j < VEC; ++j)
            if (c + j < lim) st1(row + c + j, a[j]);
    }
}

// LDS-column kernel.  VEC floats per access (16 B for VEC = 4), NS slots, U accesses per lane
// per slot per iteration, NT non-temporal loads/stores, PF prefetch of the next iteration.
template <int VEC, int NS, int U, bool NT, bool PF>
__global__ __launch_bounds__(kTPB) void mix_kernel(float* const* __restrict__ seg_ptrs,
                                                   const int64_t* __restrict__ seg_len,
                                                   const int64_t* __restrict__ tile_off,
                                                   const uint8_t* __restrict__ seg_vec, int nseg,
                                                   int64_t total_tiles, int n_slots,
                                                   const int32_t* __restrict__ plan, int64_t iter, const int64_t* __restrict__ iter_dev,
                                                   int n_local, int M, float alpha, int chunked) {
    using F = typename VT<VEC>::type;
    __shared__ F lds[NS][U][kTPB];
    __shared__ PlanLds<NS> sp;
    const int tid = threadIdx.x;
    const uint64_t need = load_plan<NS>(sp, plan, round_of(iter, iter_dev), n_local, M);
    if (need == 0) return;                    // all flags zero: the reference does no I/O
    const int32_t* deg = sp.w + mx::kPlanHeader;
    const float* sw = reinterpret_cast<const float*>(deg + n_local);
    const int32_t* src = deg + 2 * n_local;
    int dg[NS];                               // wave-uniform degrees (0 beyond n_local)
    const int dgv = (threadIdx.x & 63) < n_local ? deg[threadIdx.x & 63] : 0;   // lane r: row r's degree
    int maxd = 0;
#pragma unroll
    for (int r = 0; r < NS; ++r) {
        dg[r] = r < n_local ? __builtin_amdgcn_readfirstlane(deg[r]) : 0;
        maxd = dg[r] > maxd ? dg[r] : maxd;
    }

    Sched sc;
    sc.init<VEC, U>((chunked & 1) != 0, nseg, seg_len, tile_off, total_tiles);
    if (sc.niter == 0) return;
    F v[NS][U];
    auto load_all = [&](int seg, int64_t g, int64_t lim) {
        float* const* ptrs = seg_ptrs + (int64_t)seg * n_slots;
        const bool vec_ok = seg_vec[seg] != 0;
#pragma unroll
        for (int k = 0; k < NS; ++k)
            if ((need >> k) & 1ull) load_slot<VEC, U, NT>(v[k], ptrs[k], g, lim, vec_ok);
    };
    int seg;
    int64_t g, lim;
    sc.at<VEC, U>(0, seg, g, lim);
    load_all(seg, g, lim);
    for (int64_t i = 0; i < sc.niter; ++i) {
#pragma unroll
        for (int k = 0; k < NS; ++k)
            if ((need >> k) & 1ull) {
#pragma unroll
                for (int u = 0; u < U; ++u) lds[k][u][tid] = v[k][u];
            }
        // registers are free again: with PF the next iteration's loads are issued now, ahead of
        // (older than) this iteration's stores in vmcnt order
        int nseg_i = 0;
        int64_t ng = 0, nlim = 0;
        if (PF && i + 1 < sc.niter) {
            sc.at<VEC, U>(i + 1, nseg_i, ng, nlim);
            load_all(nseg_i, ng, nlim);
        }
        float* const* ptrs = seg_ptrs + (int64_t)seg * n_slots;
        const bool full = seg_vec[seg] && (g + (U - 1) * kTPB) * VEC + VEC <= lim;
        // Edge-major FMA chains: step e adds every row's e-th partner (rows unrolled, so the NS
        // slot lookups and LDS reads of one step are independent and overlap); per row the
        // partners still come in ascending matching order and the self term last, exactly the
        // reference's rounding sequence.
        F acc[NS][U];
#pragma unroll
        for (int r = 0; r < NS; ++r)
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int j = 0; j < VEC; ++j) acc[r][u][j] = 0.0f;
        if (NS >= 16 && (chunked & 2)) {
            // One LDS read per step fetches every row's e-th slot at once (lane r holds row r's,
            // -1 past its degree); v_readlane hands each row its slot as a scalar with no memory
            // round trip, and rows past their degree keep their accumulator through a select.
            const int lr = tid & 63;
            for (int e = 0; e < maxd; ++e) {
                const int myv = (lr < n_local && e < dgv) ? src[lr * M + e] : -1;
#pragma unroll
                for (int r = 0; r < NS; ++r) {
                    const int sl = __builtin_amdgcn_readlane(myv, r);
                    const bool on = sl >= 0;
                    const int sa = on ? sl : 0;
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const F x = lds[sa][u][tid];
#pragma unroll
                        for (int j = 0; j < VEC; ++j) {
                            const float f = __builtin_fmaf(alpha, x[j], acc[r][u][j]);
                            acc[r][u][j] = on ? f : acc[r][u][j];
                        }
                    }
                }
            }
        } else {
            for (int e = 0; e < maxd; ++e) {
#pragma unroll
                for (int r = 0; r < NS; ++r) {
                    if (e < dg[r]) {
                        const int sl = __builtin_amdgcn_readfirstlane(src[r * M + e]);
#pragma unroll
                        for (int u = 0; u < U; ++u) {
                            const F x = lds[sl][u][tid];
#pragma unroll
                            for (int j = 0; j < VEC; ++j) acc[r][u][j] = __builtin_fmaf(alpha, x[j], acc[r][u][j]);
                        }
                    }
                }
            }
        }
#pragma unroll
        for (int r = 0; r < NS; ++r) {
            if (r >= n_local || ((need >> r) & 1ull) == 0) continue;   // degree 0 unless idle rows are kept
            const float s = sw[r];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const F xs = lds[r][u][tid];
#pragma unroll
                for (int j = 0; j < VEC; ++j) acc[r][u][j] = __builtin_fmaf(s, xs[j], acc[r][u][j]);
                store_one<VEC, NT>(ptrs[r], (g + (int64_t)u * kTPB) * VEC, lim, full, acc[r][u]);
            }
        }
        if (i + 1 < sc.niter) {
            if (PF) {
                seg = nseg_i;
                g = ng;
                lim = nlim;
            } else {
                sc.at<VEC, U>(i + 1, seg, g, lim);
                load_all(seg, g, lim);
            }
        }
    }
}

// Register-indexed kernel (VEC = 4, NS <= 8): every slot's column lives in ONE register vector
// of NS*4 floats; the wave-uniform partner slot indexes it through s_set_gpr_idx (VGPR
// indexing), so no LDS is used and occupancy is bounded by VGPRs only.
template <int NS>
using RegVec = float __attribute__((ext_vector_type(NS * 4)));

template <int NS, int U, bool NT, bool PF>
__global__ __launch_bounds__(kTPB) void mix_kernel_reg(float* const* __restrict__ seg_ptrs,
                                                       const int64_t* __restrict__ seg_len,
                                                       const int64_t* __restrict__ tile_off,
                                                       const uint8_t* __restrict__ seg_vec, int nseg,
                                                       int64_t total_tiles, int n_slots,
                                                       const int32_t* __restrict__ plan, int64_t iter, const int64_t* __restrict__ iter_dev,
                                                       int n_local, int M, float alpha, int chunked) {
    using F = typename VT<4>::type;
    __shared__ PlanLds<NS> sp;
    const uint64_t need = load_plan<NS>(sp, plan, round_of(iter, iter_dev), n_local, M);
    if (need == 0) return;
    const int32_t* deg = sp.w + mx::kPlanHeader;
    const float* sw = reinterpret_cast<const float*>(deg + n_local);
    const int32_t* src = deg + 2 * n_local;

    Sched sc;
    sc.init<4, U>(chunked != 0, nseg, seg_len, tile_off, total_tiles);
    if (sc.niter == 0) return;
    // U accesses per lane per slot: columns (g + u * 256) * 4 .. +3, u < U
    auto load_all = [&](RegVec<NS> (&a)[U], int seg, int64_t g, int64_t lim) {
        float* const* ptrs = seg_ptrs + (int64_t)seg * n_slots;
        const bool vec_ok = seg_vec[seg] != 0;
#pragma unroll
        for (int k = 0; k < NS; ++k) {
            if ((need >> k) & 1ull) {
                F q[U];
                load_slot<4, U, NT>(q, ptrs[k], g, lim, vec_ok);
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    a[u][4 * k + 0] = q[u][0];
                    a[u][4 * k + 1] = q[u][1];
                    a[u][4 * k + 2] = q[u][2];
                    a[u][4 * k + 3] = q[u][3];
                }
            }
        }
    };
    int seg;
    int64_t g, lim;
    sc.at<4, U>(0, seg, g, lim);
    RegVec<NS> cur[U], nxt[PF ? U : 1];
    load_all(cur, seg, g, lim);
    for (int64_t i = 0; i < sc.niter; ++i) {
        int nseg_i = 0;
        int64_t ng = 0, nlim = 0;
        if constexpr (PF) {
            if (i + 1 < sc.niter) {
                sc.at<4, U>(i + 1, nseg_i, ng, nlim);
                load_all(nxt, nseg_i, ng, nlim);
            }
        }
        float* const* ptrs = seg_ptrs + (int64_t)seg * n_slots;
        const bool full = seg_vec[seg] && (g + (U - 1) * kTPB) * 4 + 4 <= lim;
        for (int r = 0; r < n_local; ++r) {
            const int d = deg[r];
            if (((need >> r) & 1ull) == 0) continue;
            F acc[U];
#pragma unroll
            for (int u = 0; u < U; ++u) acc[u] = F{0.0f, 0.0f, 0.0f, 0.0f};
            for (int e = 0; e < d; ++e) {
                const int s4 = 4 * __builtin_amdgcn_readfirstlane(src[r * M + e]);
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    acc[u][0] = __builtin_fmaf(alpha, cur[u][s4 + 0], acc[u][0]);
                    acc[u][1] = __builtin_fmaf(alpha, cur[u][s4 + 1], acc[u][1]);
                    acc[u][2] = __builtin_fmaf(alpha, cur[u][s4 + 2], acc[u][2]);
                    acc[u][3] = __builtin_fmaf(alpha, cur[u][s4 + 3], acc[u][3]);
                }
            }
            const int r4 = 4 * __builtin_amdgcn_readfirstlane(r);
            const float s = sw[r];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                acc[u][0] = __builtin_fmaf(s, cur[u][r4 + 0], acc[u][0]);
                acc[u][1] = __builtin_fmaf(s, cur[u][r4 + 1], acc[u][1]);
                acc[u][2] = __builtin_fmaf(s, cur[u][r4 + 2], acc[u][2]);
                acc[u][3] = __builtin_fmaf(s, cur[u][r4 + 3], acc[u][3]);
                store_one<4, NT>(ptrs[r], (g + (int64_t)u * kTPB) * 4, lim, full, acc[u]);
            }
        }
        if (i + 1 < sc.niter) {
            if constexpr (PF) {
                seg = nseg_i;
                g = ng;
                lim = nlim;
#pragma unroll
                for (int u = 0; u < U; ++u) cur[u] = nxt[u];
            } else {
                sc.at<4, U>(i + 1, seg, g, lim);
                load_all(cur, seg, g, lim);
            }
        }
    }
}

// Row-per-wave kernel (9-64 slots).  A tile is 16384 floats of slot data (NS slots x TW columns,
// TW = 1024 / 512 / 256 for NS = 16 / 32 / 64 -- the LDS kernel's tiles, so layouts are shared):
// the whole workgroup stages it in LDS with 16-byte loads (next tile's loads in flight in
// registers while this one is mixed), then each wave takes whole (row, 256-column pass) items and
// walks only that row's own partners: one wave-uniform slot per step, one ds_read_b128 and 4 FMAs
// per lane.  The LDS-column kernel instead runs every row for max-degree steps in every lane,
// with per-row lookups and selects -- VALU-bound at 32-64 slots.  Items are dealt to the 4 waves
// by weight (degree + 1, ranked in wave 0, snake order), two items interleaved per wave for ILP.
//
// SPLIT > 1 (small rows, fewer layout tiles than the persistent grid): each layout tile of
// TW * SPLIT columns is worked as SPLIT sub-tiles of TW columns, so a 181k-parameter round
// spreads over every CU instead of a few dozen (layouts and tile_off stay in layout-tile units).
//
// PF2: two tiles' loads in flight instead of one (two register sets, the loop unrolled by two) --
// a persistent workgroup whose tile stages few of its NS slots (a GPU's share of a big topology:
// few local rows, many received ones) otherwise keeps too little in flight per CU.
template <int NS, int TW, bool NT, int SPLIT = 1, bool PF2 = false, int TPB = kTPB, bool SPEC = false, bool GL = false>
__global__ __launch_bounds__(TPB) void mix_kernel_rows(float* const* __restrict__ seg_ptrs,
                                                        const int64_t* __restrict__ seg_len,
                                                        const int64_t* __restrict__ tile_off,
                                                        const uint8_t* __restrict__ seg_vec, int nseg,
                                                        int64_t total_tiles, int n_slots,
                                                        const int32_t* __restrict__ plan, int64_t iter, const int64_t* __restrict__ iter_dev,
                                                        int n_local, int M, float alpha, uint64_t hint) {
    using F = typename VT<4>::type;
    constexpr int C4 = TW / 4;            // float4 per slot per tile
    constexpr int NQ = TW / 256;          // 256-column passes per row
    constexpr int NI = NS * NQ;           // items per tile (<= 64: one per lane of wave 0)
    constexpr int WV = TPB / 64;          // waves sharing the staged tile
    constexpr int E4 = NS * C4 / TPB;     // float4 staged per lane per tile
    static_assert(NI <= 64 && NI % WV == 0 && E4 >= 1 && E4 * TPB == NS * C4 && C4 % 64 == 0, "row kernel geometry");
    __shared__ F lds[NS * C4];
    __shared__ PlanLds<NS> sp;
    __shared__ int32_t wl[WV][NI / WV];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t total_work = total_tiles * SPLIT;
    const int64_t niter = total_work > blockIdx.x ? (total_work - blockIdx.x + gridDim.x - 1) / gridDim.x : 0;
    if (niter == 0) return;                  // block-uniform, before any barrier

    // tile geometry (segment, first column, limit) and staging; 16-byte accesses wherever the slot's
    // row pointer is 16-byte aligned (al16) -- seg_vec is not read here
    struct Geo {
        float* const* ptrs;
        int64_t col0, lim;
    };
    auto geo = [&](int64_t work) {
        const int64_t tile = work / SPLIT;
        int lo = 0, hi = nseg;
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (tile_off[mid] <= tile) lo = mid; else hi = mid;
        }
        Geo gq;
        gq.ptrs = seg_ptrs + (int64_t)lo * n_slots;
        gq.col0 = (tile - tile_off[lo]) * (TW * SPLIT) + (work % SPLIT) * TW;
        gq.lim = seg_len[lo];
        return gq;
    };
    F R[E4];
    auto stage_mask = [&](F (&RR)[E4], const Geo& gq, uint64_t mask) {
#pragma unroll
        for (int j = 0; j < E4; ++j) {
            const int k = (wave * 64 + TPB * j) / C4;            // wave-uniform slot
            if ((mask >> k) & 1ull) {
                const int64_t c = gq.col0 + (int64_t)((wave * 64 + TPB * j) % C4 + lane) * 4;
                const float* row = gq.ptrs[k];
                if (al16(row) && c + 4 <= gq.lim) {
                    RR[j] = ld<NT, F>(row + c);
                } else {
#pragma unroll
                    for (int t = 0; t < 4; ++t) RR[j][t] = (c + t < gq.lim) ? ld1(row + c + t) : 0.0f;
                }
            }
        }
    };
    const uint64_t local_mask = n_local >= 64 ? ~0ull : (1ull << n_local) - 1;
    Geo cur;
    uint32_t gl_j = 0;                       // GL: loads j of this wave that went straight to LDS
    if constexpr (SPEC) {
        cur = geo(blockIdx.x);
        if constexpr (GL) {
            // LDS-DMA (global_load_lds_dwordx4): a wave's 64 lanes land 1 KB contiguously at a
            // wave-uniform LDS base -- the tile layout's own order; a wave whose columns run past
            // the row end stages through registers instead
            const uint64_t m = hint & local_mask;
#pragma unroll
            for (int j = 0; j < E4; ++j) {
                const int k = (wave * 64 + TPB * j) / C4;
                if ((m >> k) & 1ull) {
                    const int o = (wave * 64 + TPB * j) % C4;
                    const float* row = cur.ptrs[k];
                    if (al16(row) && cur.col0 + (int64_t)(o + 63) * 4 + 4 <= cur.lim) {
                        const int64_t c = cur.col0 + (int64_t)(o + lane) * 4;
                        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(row + c),
                                                         (__attribute__((address_space(3))) void*)&lds[k * C4 + o],
                                                         16, 0, NT ? 2 : 0);
                        gl_j |= 1u << j;
                    } else {
                        const int64_t c = cur.col0 + (int64_t)(o + lane) * 4;
#pragma unroll
                        for (int t = 0; t < 4; ++t) R[j][t] = (c + t < cur.lim) ? ld1(row + c + t) : 0.0f;
                    }
                }
            }
        } else {
            stage_mask(R, cur, hint & local_mask);   // in flight while the plan record is fetched
        }
    }
    const uint64_t need = load_plan<NS>(sp, plan, round_of(iter, iter_dev), n_local, M);
    if (need == 0) return;
    const int32_t* deg = sp.w + mx::kPlanHeader;
    const float* sw = reinterpret_cast<const float*>(deg + n_local);
    const int32_t* src = deg + 2 * n_local;
    auto stage_to = [&](F (&RR)[E4], const Geo& gq) { stage_mask(RR, gq, need); };
    auto stage = [&](const Geo& gq) { stage_to(R, gq); };

    // deal the items (row r, pass q) = r * NQ + q to the waves: wave 0 ranks them by weight
    if (wave == 0) {
        const int r = lane / NQ;
        const int w = (lane < NI && r < n_local && ((need >> r) & 1ull)) ? deg[r] + 1 : 0;
        int rank = 0;
        for (int j = 0; j < NI; ++j) {
            const int wj = __builtin_amdgcn_readlane(w, j);
            rank += (wj > w) || (wj == w && j < lane);
        }
        const int round = rank / WV, within = rank % WV;
        if (lane < NI) wl[(round & 1) ? WV - 1 - within : within][round] = w > 0 ? lane : -1;
    }
    if constexpr (SPEC) {
        // received slots, and any local row the hint left out (a wrong hint costs time, never bits)
        const uint64_t rest = need & ~(hint & local_mask);
        if (rest) stage_mask(R, cur, rest);
    } else {
        cur = geo(blockIdx.x);
        stage(cur);
    }
    F R2[PF2 ? E4 : 1];
    Geo cur2 = cur;
    if constexpr (PF2) {
        if (niter > 1) {
            cur2 = geo(blockIdx.x + gridDim.x);
            stage_to(R2, cur2);
        }
    }
    __syncthreads();
    // ranks grow along a wave's list, so its unused (-1) entries form a suffix
    int nmy = 0;
    while (nmy < NI / WV && wl[wave][nmy] >= 0) ++nmy;
    nmy = __builtin_amdgcn_readfirstlane(nmy);

    // mix the tile staged in LDS (columns of `cur`) and store the local rows
    auto mix_tile = [&](const Geo& cur) {
        auto finish = [&](int it, F acc) {
            const int r = it / NQ;
            const int col = (it % NQ) * 64 + lane;
            const F xs = lds[r * C4 + col];
            const float s = sw[r];
#pragma unroll
            for (int t = 0; t < 4; ++t) acc[t] = __builtin_fmaf(s, xs[t], acc[t]);
            const int64_t c = cur.col0 + (int64_t)col * 4;
            store_one<4, NT>(cur.ptrs[r], c, cur.lim, al16(cur.ptrs[r]) && c + 4 <= cur.lim, acc);
        };
        int p = 0;
        for (; p + 1 < nmy; p += 2) {            // two items interleaved
            const int ia = __builtin_amdgcn_readfirstlane(wl[wave][p]);
            const int ib = __builtin_amdgcn_readfirstlane(wl[wave][p + 1]);
            const int ra = ia / NQ, rb = ib / NQ;
            const int ca = (ia % NQ) * 64 + lane, cb = (ib % NQ) * 64 + lane;
            const int da = deg[ra], db = deg[rb];
            const int dmin = da < db ? da : db;
            F a = F{0.0f, 0.0f, 0.0f, 0.0f}, b = F{0.0f, 0.0f, 0.0f, 0.0f};
            int e = 0;
            for (; e < dmin; ++e) {
                const int sa = __builtin_amdgcn_readfirstlane(src[ra * M + e]);
                const int sb = __builtin_amdgcn_readfirstlane(src[rb * M + e]);
                const F xa = lds[sa * C4 + ca];
                const F xb = lds[sb * C4 + cb];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    a[t] = __builtin_fmaf(alpha, xa[t], a[t]);
                    b[t] = __builtin_fmaf(alpha, xb[t], b[t]);
                }
            }
            for (int ea = e; ea < da; ++ea) {
                const F xa = lds[__builtin_amdgcn_readfirstlane(src[ra * M + ea]) * C4 + ca];
#pragma unroll
                for (int t = 0; t < 4; ++t) a[t] = __builtin_fmaf(alpha, xa[t], a[t]);
            }
            for (int eb = e; eb < db; ++eb) {
                const F xb = lds[__builtin_amdgcn_readfirstlane(src[rb * M + eb]) * C4 + cb];
#pragma unroll
                for (int t = 0; t < 4; ++t) b[t] = __builtin_fmaf(alpha, xb[t], b[t]);
            }
            finish(ia, a);
            finish(ib, b);
        }
        if (p < nmy) {
            const int ia = __builtin_amdgcn_readfirstlane(wl[wave][p]);
            const int ra = ia / NQ, ca = (ia % NQ) * 64 + lane;
            F a = F{0.0f, 0.0f, 0.0f, 0.0f};
            for (int e = 0; e < deg[ra]; ++e) {
                const F xa = lds[__builtin_amdgcn_readfirstlane(src[ra * M + e]) * C4 + ca];
#pragma unroll
                for (int t = 0; t < 4; ++t) a[t] = __builtin_fmaf(alpha, xa[t], a[t]);
            }
            finish(ia, a);
        }
    };
    if constexpr (!PF2) {
        for (int64_t i = 0; i < niter; ++i) {
            if (i) __syncthreads();              // every wave is done reading the previous tile
#pragma unroll
            for (int j = 0; j < E4; ++j) {
                const int k = (wave * 64 + TPB * j) / C4;
                if (((need >> k) & 1ull) && !(i == 0 && ((gl_j >> j) & 1u)))
                    lds[k * C4 + (wave * 64 + TPB * j) % C4 + lane] = R[j];
            }
            if constexpr (GL) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // LDS-DMA landed
            __syncthreads();
            Geo nxt = cur;
            if (i + 1 < niter) {                 // next tile's loads fly while this one is mixed
                nxt = geo(blockIdx.x + (i + 1) * gridDim.x);
                stage(nxt);
            }
            mix_tile(cur);
            cur = nxt;
        }
    } else {
        // tile i in register set (i % 2); after it is parked in LDS, the set takes tile i + 2
        auto step = [&](int64_t i, F (&RR)[E4], Geo& gi) {
            if (i) __syncthreads();
#pragma unroll
            for (int j = 0; j < E4; ++j) {
                const int k = (wave * 64 + TPB * j) / C4;
                if ((need >> k) & 1ull) lds[k * C4 + (wave * 64 + TPB * j) % C4 + lane] = RR[j];
            }
            __syncthreads();
            const Geo here = gi;
            if (i + 2 < niter) {
                gi = geo(blockIdx.x + (i + 2) * gridDim.x);
                stage_to(RR, gi);
            }
            mix_tile(here);
        };
        for (int64_t i = 0; i < niter; i += 2) {
            step(i, R, cur);
            if (i + 1 < niter) step(i + 1, R2, cur2);
        }
    }
}

// Wide kernel: any matching count and up to kWideMaxSlots slots (more workers per GPU, or more
// remote partners, than the NS <= 64 kernels and their 32-matching plan records in LDS take).
// A layout tile (256 columns) is worked in pieces of 64 * VEC columns, VEC = 4 / 2 / 1 chosen so
// that a piece of every slot fits the LDS budget (default 158 KB: VEC = 4 up to 156 slots, one
// 1024-thread workgroup per CU, two when the piece is <= 79 KB): the whole workgroup stages a piece
// of every needed slot (16 / 8 / 4-byte loads, slot wave-uniform), the next piece's loads are
// issued into registers right after the barrier and fly while this piece is mixed; each wave then
// takes rows wave, wave + WV, ... in pairs and walks their partner lists (from the plan record,
// copied to LDS when that costs no occupancy) two partners a step, in matching order with the self
// term last -- the same FMA chain as every other kernel.  The partner walk is latency-bound per
// wave, so the waves sharing one staged piece set the rate: 4 -> 16 waves per piece took 96-150
// slots from 2.2-2.3 to 4.4 TB/s (tools/sessions/r3_s39.sh).
constexpr int kWideMaxSlots = 156;

// BIG: staging registers for up to kWideMaxSlots slots at VEC = 4 / 2 (wider pieces for big slot
// counts, with the LDS that takes -- mx_mix_set "wide_lds_kb").
// PLDS: the round's plan record is copied into LDS behind the pieces (when it fits), so the partner
// walk reads slots with ds_read instead of a global load per step.
// TPB: workgroup size (mx_mix_set "wide_tpb"): more waves share one staged piece, so more rows'
// partner walks run at once per byte of LDS.
template <int VEC, bool BIG, int TPB>
constexpr int wide_regs() {
    return ((BIG ? kWideMaxSlots : VEC == 4 ? 40 : VEC == 2 ? 80 : kWideMaxSlots) + TPB / 64 - 1) / (TPB / 64);
}
template <int VEC, bool NT, bool BIG, bool PLDS, int TPB, bool PF2 = false>
__global__ __launch_bounds__(TPB) void mix_kernel_wide(float* const* __restrict__ seg_ptrs,
                                                        const int64_t* __restrict__ seg_len,
                                                        const int64_t* __restrict__ tile_off,
                                                        const uint8_t* __restrict__ seg_vec, int nseg,
                                                        int64_t total_tiles, int tile_cols, int n_slots,
                                                        const int32_t* __restrict__ plan, int64_t iter,
                                                        const int64_t* __restrict__ iter_dev, int n_local, int M,
                                                        float alpha) {
    using F = typename VT<VEC>::type;
    constexpr int PW = 64 * VEC;              // columns per piece
    constexpr int NR = wide_regs<VEC, BIG, TPB>();   // staged vectors per lane
    constexpr int WV = TPB / 64;
    extern __shared__ __attribute__((aligned(16))) float wlds_raw[];
    F* wlds = reinterpret_cast<F*>(wlds_raw);  // [n_slots][64] vectors
    iter = round_of(iter, iter_dev);
    if (iter < 0) return;
    const int32_t* rec = plan + iter * mx::plan_words(n_local, M);
    if (rec[0] == 0) return;                  // all flags zero
    if constexpr (PLDS) {
        const int64_t W = mx::plan_words(n_local, M);
        int32_t* pl = reinterpret_cast<int32_t*>(wlds_raw + (int64_t)n_slots * 64 * VEC);
        for (int64_t i = threadIdx.x; i < W; i += TPB) pl[i] = rec[i];
        __syncthreads();
        rec = pl;
    }
    peer_acquire(rec[2]);
    const int n_remote = rec[1];
    const bool idle = (rec[2] & 1) != 0;
    const int32_t* deg = rec + mx::kPlanHeader;
    const float* sw = reinterpret_cast<const float*>(deg + n_local);
    const int32_t* src = deg + 2 * n_local;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int pieces = tile_cols / PW;
    const int64_t work = total_tiles * pieces;
    const int nj = (n_slots + WV - 1) / WV;      // staged vectors per lane (slot = wave + WV j)
    // VEC-wide accesses wherever the slot's row pointer is VEC * 4-byte aligned (a scalar test;
    // the seg_vec byte would be a vector-memory round trip per piece)
    struct Geo {
        float* const* ptrs;
        int64_t col0, lim;
    };
    auto alv = [](const float* p) { return ((uintptr_t)p & (VEC * sizeof(float) - 1)) == 0; };
    auto geo = [&](int64_t wi) {
        const int64_t tile = wi / pieces;
        int lo = 0, hi = nseg;
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (tile_off[mid] <= tile) lo = mid; else hi = mid;
        }
        Geo g;
        g.ptrs = seg_ptrs + (int64_t)lo * n_slots;
        g.col0 = (tile - tile_off[lo]) * tile_cols + (wi % pieces) * PW;
        g.lim = seg_len[lo];
        return g;
    };
    auto needed = [&](int k) {
        return k < n_local ? (deg[k] > 0 || idle) : (k - n_local < n_remote);
    };
    F RS[PF2 ? 2 : 1][NR];
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, PF2 ? 1 : 0>;
    auto stage_to = [&](auto setc, const Geo& g) {
        constexpr int S = decltype(setc)::value;
#pragma unroll
        for (int j = 0; j < NR; ++j) {
            const int k = wave + WV * j;                    // wave-uniform slot
            if (j < nj && k < n_slots && needed(k)) {
                const int64_t c = g.col0 + (int64_t)lane * VEC;
                if (alv(g.ptrs[k]) && c + VEC <= g.lim) {
                    RS[S][j] = ld<NT, F>(g.ptrs[k] + c);
                } else {
#pragma unroll
                    for (int t = 0; t < VEC; ++t) RS[S][j][t] = (c + t < g.lim) ? ld1(g.ptrs[k] + c + t) : 0.0f;
                }
            }
        }
    };
    auto park = [&](auto setc) {
        constexpr int S = decltype(setc)::value;
#pragma unroll
        for (int j = 0; j < NR; ++j) {
            const int k = wave + WV * j;
            if (j < nj && k < n_slots && needed(k)) wlds[k * 64 + lane] = RS[S][j];
        }
    };
    auto mix_piece = [&](const Geo& cur) {
            // this wave's rows in pairs (r, r + WV): the two partner walks interleaved, two partners per
            // step, so four slot reads and four piece reads are in flight at once (no branch between
            // them); each row's FMA order is unchanged (partners in matching order, then the self term)
            const int64_t c = cur.col0 + (int64_t)lane * VEC;
            auto finish = [&](int r, F acc) {
                const F xs = wlds[r * 64 + lane];
                const float s = sw[r];
    #pragma unroll
                for (int t = 0; t < VEC; ++t) acc[t] = __builtin_fmaf(s, xs[t], acc[t]);
                if (c < cur.lim) store_one<VEC, NT>(cur.ptrs[r], c, cur.lim, alv(cur.ptrs[r]) && c + VEC <= cur.lim, acc);
            };
            auto tail = [&](const int32_t* sr, int e, int d, F& acc) {
                for (; e + 2 <= d; e += 2) {
                    const int s0 = __builtin_amdgcn_readfirstlane(sr[e]);
                    const int s1 = __builtin_amdgcn_readfirstlane(sr[e + 1]);
                    const F x0 = wlds[s0 * 64 + lane];
                    const F x1 = wlds[s1 * 64 + lane];
    #pragma unroll
                    for (int t = 0; t < VEC; ++t) acc[t] = __builtin_fmaf(alpha, x0[t], acc[t]);
    #pragma unroll
                    for (int t = 0; t < VEC; ++t) acc[t] = __builtin_fmaf(alpha, x1[t], acc[t]);
                }
                if (e < d) {
                    const F x0 = wlds[__builtin_amdgcn_readfirstlane(sr[e]) * 64 + lane];
    #pragma unroll
                    for (int t = 0; t < VEC; ++t) acc[t] = __builtin_fmaf(alpha, x0[t], acc[t]);
                }
            };
            for (int ra = wave; ra < n_local; ra += 2 * WV) {
                const int rb = ra + WV;
                const bool hb = rb < n_local;
                const int da = __builtin_amdgcn_readfirstlane(deg[ra]);
                const int db = hb ? __builtin_amdgcn_readfirstlane(deg[rb]) : 0;
                const int32_t* sa = src + (int64_t)ra * M;
                const int32_t* sb = src + (int64_t)rb * M;
                F a, b;
    #pragma unroll
                for (int t = 0; t < VEC; ++t) a[t] = b[t] = 0.0f;
                const int dm = da < db ? da : db;
                int e = 0;
                for (; e + 2 <= dm; e += 2) {
                    const int a0 = __builtin_amdgcn_readfirstlane(sa[e]);
                    const int a1 = __builtin_amdgcn_readfirstlane(sa[e + 1]);
                    const int b0 = __builtin_amdgcn_readfirstlane(sb[e]);
                    const int b1 = __builtin_amdgcn_readfirstlane(sb[e + 1]);
                    const F xa0 = wlds[a0 * 64 + lane];
                    const F xa1 = wlds[a1 * 64 + lane];
                    const F xb0 = wlds[b0 * 64 + lane];
                    const F xb1 = wlds[b1 * 64 + lane];
    #pragma unroll
                    for (int t = 0; t < VEC; ++t) {
                        a[t] = __builtin_fmaf(alpha, xa0[t], a[t]);
                        b[t] = __builtin_fmaf(alpha, xb0[t], b[t]);
                    }
    #pragma unroll
                    for (int t = 0; t < VEC; ++t) {
                        a[t] = __builtin_fmaf(alpha, xa1[t], a[t]);
                        b[t] = __builtin_fmaf(alpha, xb1[t], b[t]);
                    }
                }
                tail(sa, e, da, a);
                tail(sb, e, db, b);
                if (da > 0 || idle) finish(ra, a);
                if (hb && (db > 0 || idle)) finish(rb, b);
            }
    };
    int64_t wi = blockIdx.x;
    if (wi >= work) return;
    Geo cur = geo(wi);
    stage_to(I0{}, cur);
    if constexpr (!PF2) {
        for (; wi < work; wi += gridDim.x) {
            park(I0{});
            __syncthreads();
            Geo nxt = cur;
            if (wi + gridDim.x < work) {       // the next piece's loads fly while this one is mixed
                nxt = geo(wi + gridDim.x);
                stage_to(I0{}, nxt);
            }
            mix_piece(cur);
            __syncthreads();                  // the piece is read by every wave before restaging
            cur = nxt;
        }
    } else {
        // piece i in register set i % 2; after it is parked in LDS the set takes piece i + 2
        Geo cur2 = cur;
        if (wi + gridDim.x < work) {
            cur2 = geo(wi + gridDim.x);
            stage_to(I1{}, cur2);
        }
        auto step = [&](auto setc, Geo& gi, int64_t w) {
            park(setc);
            __syncthreads();
            const Geo here = gi;
            if (w + 2 * (int64_t)gridDim.x < work) {
                gi = geo(w + 2 * (int64_t)gridDim.x);
                stage_to(setc, gi);
            }
            mix_piece(here);
            __syncthreads();
        };
        for (; wi < work; wi += 2 * (int64_t)gridDim.x) {
            step(I0{}, cur, wi);
            if (wi + gridDim.x < work) step(I1{}, cur2, wi + gridDim.x);
        }
    }
}

struct Cfg {
    int vec, ns;
};

int g_ns48 = 0;      // 33-48 slots: a 48-slot row-kernel class (48 KB tiles) instead of the 64-slot one

Cfg pick(int n_slots) {
    if (n_slots <= 8) return {4, 8};
    if (n_slots <= 16) return {4, 16};
    if (n_slots <= 32) return {2, 32};
    if (n_slots <= 48 && g_ns48) return {1, 48};
    if (n_slots <= 64) return {1, 64};
    if (n_slots <= kWideMaxSlots) return {1, 0};    // wide kernel only (256-column layout tiles)
    return {0, 0};
}

// tuning state (mx_mix_set / mx_mix_get); defaults from tools/mixtune.py sweeps on MI355X
// (8 x 25.6M graph-0 rounds): register-indexed + non-temporal + tile stride; with global (not
// flat) loads 2 WGs/CU beat 3 / 4 by 5-9 % (fewer concurrent DRAM streams, latency still hidden)
// and ran at 0.94x the time of torch's copy_ of the same bytes; 2 / 4 accesses per lane per row
// and prefetch were 3-5 % slower; balanced contiguous chunks 20-30 % slower (each workgroup
// streaming its own far-apart range loses the chip-wide DRAM row locality of the tile sweep).
struct Tune {
    int blocks_per_cu = 2;
    int unroll = 1;      // 1, 2 or 4 accesses per lane per row per tile (NS = 8 configs only; LDS kernel <= 2)
    int nontemporal = 2;  // 1 / 0: streaming hints on / off; 2 = auto (row kernel: off for rows of
                          // 32-320 MB, about the Infinity Cache; every other kernel: on)
    int prefetch = 0;
    int regidx = 1;      // 1: register-indexed kernel (n_slots <= 8; wider spills), 0: LDS-column kernel
    int chunked = 0;     // single-segment layouts: 1 = equal contiguous chunk per workgroup, 0 = tile stride
    int grid = 0;        // > 0: exact persistent grid size (overrides blocks_per_cu)
    int readlane_min = 32;  // LDS kernel: slot counts >= this fetch a step's slots with one read + v_readlane
    int rows = 2;        // row-per-wave kernel: 2 = every slot count (<= 8 slots with unroll 1 / 2),
                         // 1 = 9-64 slots only (<= 8: register-indexed / LDS-column), 0 = never
    int split = 0;       // row kernel sub-tiles per layout tile: 0 = auto (enough work items for
                         // the persistent grid), 1 / 2 / 4 = forced (capped by the geometry)
    int wide_lds_kb = 158;  // wide kernel (65-156 slots): LDS per piece (KB); more -> wider pieces, fewer WGs per CU
    int rows_tpb = 256;     // row kernel, 32-64 slots (unsplit tiles): workgroup size 256 / 512 / 1024
    int wide_tpb = 1024;    // wide kernel: workgroup size (256 / 512 / 1024)
    int wide_pf2 = 1;       // wide kernel, 1024 threads: two pieces' loads in flight (two register sets)
    int wide_per_cu = 0;    // wide kernel: workgroups per CU cap (0 = 4; fewer when the LDS does not fit)
    int wide_plan_lds = 1;  // wide kernel: the plan record in LDS (when <= 32 KB) instead of global loads
    int rows_pf2 = 2;    // row kernel, persistent grids of 32-64 slots: two tiles' loads in flight -- 1 on,
                         // 0 off, 2 auto: when at most 5/8 of the class's slots are staged (ER(64)'s N = 8
                         // share, 35 of 64 slots: 0.874 -> 0.927 of the headline kernel's HBM rate; all 64
                         // slots staged: 1.058 -> 0.971, tools/er_share.py, profiles/r03c_er_share_pf2.log)
    int flat_small = 256;  // row kernel: rounds of at most flat_small x the persistent grid's work items
                         // launch one workgroup per item instead (a second pass over the persistent
                         // grid is a second memory round trip on latency-bound short rows); 0 = never
    int mid_bpc = 4;       // row kernel, 8 slots, rows of at most mid_tiles x CUs layout tiles: a persistent
    int mid_tiles = 8;     // grid of mid_bpc workgroups per CU instead of the flat one (0 = off)
    int spec = 1;          // row kernel, 8 local slots and no receive slots, flat grid, streaming
                           // hints, rounds of > 64 MB: rounds with a caller-supplied active-row hint
                           // load those rows' tiles before the plan record (1 on, 0 off)
    int spec_wgpc = 5;     // ... at this many workgroups per CU (dynamic LDS cap; 0 = no cap)
    int spec_glds = 1;     // ... staging those tiles with LDS-DMA (global_load_lds) instead of registers
                           // (512-column sub-tiles: headline 0.2627 -> 0.2591 ms, WRN-28-10 rows
                           // 0.3792 -> 0.3712 ms; profiles/r06t_glds_ab.json)
};
Tune g_tune;

// accesses per lane per slot per tile: the NS = 8 kernels take 1, 2 or 4 (the LDS one 1 or 2)
int unroll_for(int ns) {
    if (ns != 8) return 1;
    if (!g_tune.regidx && g_tune.unroll > 2) return 2;
    return g_tune.unroll;
}

int cu_count() {
    static int v = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess) return 256;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 256;
        return n > 0 ? n : 256;
    }();
    return v;
}

// grid: CUs x blocks_per_cu persistent workgroups, never more than there are tiles; a single
// segment is split into equal contiguous chunks (chunked = 1)
inline int64_t grid_target() {
    return g_tune.grid > 0 ? (int64_t)g_tune.grid : (int64_t)cu_count() * g_tune.blocks_per_cu;
}
inline int64_t grid_for(int64_t total_tiles) {
    int64_t grid = grid_target();
    if (grid > total_tiles) grid = total_tiles;
    return grid < 1 ? 1 : grid;
}

// 8 slots, mid-sized rows (0.4-2M params: a few work items per CU): a persistent grid of mid_bpc
// workgroups per CU, each with its next item's loads in flight, beats one workgroup per item by 7-13 %
// (graph-replayed rounds, tools/small_cfg.py; equal at 181k, the flat grid 1-3 % ahead from 4M on)
inline bool rows_mid(int ns, int64_t total_tiles) {
    return ns == 8 && g_tune.mid_bpc > 0 && g_tune.flat_small > 0 && g_tune.grid == 0 &&
           total_tiles <= (int64_t)g_tune.mid_tiles * cu_count();
}

// row kernel sub-tiles per layout tile: a sub-tile keeps >= 256 columns (one wave pass), and
// auto picks the smallest split giving the persistent grid 1.5 work items per workgroup
// (measured, 8 slots: 651 tiles run 11 % faster as 1302 sub-tiles, 977 tiles 5 % slower as 1954)
int row_split(int ns, int64_t total_tiles) {
    const int cap = ns >= 48 ? 1 : (ns == 32 ? 2 : 4);
    if (g_tune.split > 0) return g_tune.split < cap ? g_tune.split : cap;
    int s = 1;
    if (rows_mid(ns, total_tiles)) {
        while (s < cap && 2 * total_tiles * s < 3 * (int64_t)cu_count() * g_tune.mid_bpc) s *= 2;
        return s;
    }
    while (s < cap && 2 * total_tiles * s < 3 * grid_target()) s *= 2;
    // with one workgroup per work item (flat_small), 512-column sub-tiles beat whole 1024-column
    // tiles at every size measured for 8 slots (2M-36.5M params: -1 to -6 %; headline 283.8 ->
    // 272.3 us, tools/split_sweep.py); persistent grids keep whole tiles (split 2 was slower there)
    if (s < 2 && ns <= 16 && g_tune.flat_small > 0 && g_tune.grid == 0 &&
        2 * total_tiles <= (int64_t)g_tune.flat_small * grid_target())
        s = 2;
    return s;
}

// per-call options of the row kernel's SPEC form, set by gossip_mix for the launch it dispatches
struct RowsOpt {
    uint64_t hint = 0;       // local rows whose tiles are loaded before the plan record arrives
    int wg_per_cu = 0;       // SPEC launches: workgroups per CU (0 = as many as fit)
};
thread_local RowsOpt g_rows_opt;
std::atomic<int64_t> g_spec_launches{0};   // SPEC launches so far (mx_mix_get "spec_launches": tests)

template <int VEC, int NS, int U, bool NT, bool PF>
int launch(float* const* seg_ptrs, const int64_t* seg_len, const int64_t* tile_off,
           const uint8_t* seg_vec, int nseg, int n_slots, const int32_t* plan, int64_t iter, const int64_t* iter_dev,
           int n_local, int M, float alpha, int64_t total_tiles, hipStream_t st) {
    const int mode = ((nseg == 1 && g_tune.chunked) ? 1 : 0) | (NS >= g_tune.readlane_min ? 2 : 0);
    hipLaunchKernelGGL((mix_kernel<VEC, NS, U, NT, PF>), dim3((unsigned)grid_for(total_tiles)), dim3(kTPB),
                       0, st, seg_ptrs, seg_len, tile_off, seg_vec, nseg, total_tiles, n_slots, plan,
                       iter, iter_dev, n_local, M, alpha, mode);
    MX_LAUNCH_CHECK();
    return MX_OK;
}

template <int NS, int TW, bool NT, int SPLIT = 1, bool PF2 = false, int TPB = kTPB, bool SPEC = false, bool GL = false>
int launch_rows(float* const* seg_ptrs, const int64_t* seg_len, const int64_t* tile_off,
                const uint8_t* seg_vec, int nseg, int n_slots, const int32_t* plan, int64_t iter, const int64_t* iter_dev,
                int n_local, int M, float alpha, int64_t total_tiles, hipStream_t st) {
    const int64_t work = total_tiles * SPLIT;
    // one workgroup per item only for 8-16 slots: with 32 / 64 slots (narrower tiles, longer partner
    // walks) the persistent grid stays faster (ER(32): 286 vs 350 us, ER(64): 324 vs 426 us)
    const int64_t mid = rows_mid(NS, total_tiles) ? (int64_t)cu_count() * g_tune.mid_bpc : 0;
    const int64_t grid = mid ? (work < mid ? work : mid)
                         : (NS <= 16 && g_tune.flat_small > 0 && g_tune.grid == 0 &&
                            work <= (int64_t)g_tune.flat_small * grid_target()) ? work : grid_for(work);
    // SPEC launches cap the workgroups per CU (g_rows_opt.wg_per_cu) with dynamic LDS on top of
    // the kernel's static LDS: fewer tiles in flight per CU, each issued at once
    size_t pad = 0;
    if (SPEC && g_rows_opt.wg_per_cu > 0) {
        static const int stat = [] {                           // static LDS of this instantiation
            hipFuncAttributes fa{};
            return hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(
                       mix_kernel_rows<NS, TW, NT, SPLIT, PF2, TPB, SPEC, GL>)) == hipSuccess ? (int)fa.sharedSizeBytes : 0;
        }();
        pad = mx::lds_cap_pad(stat, g_rows_opt.wg_per_cu);
    }
    hipLaunchKernelGGL((mix_kernel_rows<NS, TW, NT, SPLIT, PF2, TPB, SPEC, GL>), dim3((unsigned)grid), dim3(TPB),
                       pad, st, seg_ptrs, seg_len, tile_off, seg_vec, nseg, total_tiles, n_slots, plan,
                       iter, iter_dev, n_local, M, alpha, g_rows_opt.hint);
    MX_LAUNCH_CHECK();
    return MX_OK;
}

template <int NS, int U, bool NT, bool PF>
int launch_reg(float* const* seg_ptrs, const int64_t* seg_len, const int64_t* tile_off,
               const uint8_t* seg_vec, int nseg, int n_slots, const int32_t* plan, int64_t iter, const int64_t* iter_dev,
               int n_local, int M, float alpha, int64_t total_tiles, hipStream_t st) {
    hipLaunchKernelGGL((mix_kernel_reg<NS, U, NT, PF>), dim3((unsigned)grid_for(total_tiles)), dim3(kTPB),
                       0, st, seg_ptrs, seg_len, tile_off, seg_vec, nseg, total_tiles, n_slots, plan,
                       iter, iter_dev, n_local, M, alpha, (nseg == 1 && g_tune.chunked) ? 1 : 0);
    MX_LAUNCH_CHECK();
    return MX_OK;
}

}  // namespace

extern "C" int mx_mix_tile(int n_slots) {
    const Cfg c = pick(n_slots);
    if (c.vec > 0 && c.ns == 0) return kTPB;           // wide kernel: 256-column tiles
    return c.vec * kTPB * unroll_for(c.ns);
}

extern "C" int mx_mix_set(const char* key, int value) {
    MX_CHECK(key, "mx_mix_set: null key");
    int* slot = nullptr;
    if (!strcmp(key, "blocks_per_cu")) {
        MX_CHECK(value >= 1 && value <= 64, "mx_mix_set: blocks_per_cu %d", value);
        slot = &g_tune.blocks_per_cu;
    } else if (!strcmp(key, "unroll")) {
        MX_CHECK(value == 1 || value == 2 || value == 4, "mx_mix_set: unroll %d", value);
        slot = &g_tune.unroll;
    } else if (!strcmp(key, "nontemporal")) {
        slot = &g_tune.nontemporal;
        value = value == 2 ? 2 : (value ? 1 : 0);
    } else if (!strcmp(key, "prefetch")) {
        slot = &g_tune.prefetch;
        value = value ? 1 : 0;
    } else if (!strcmp(key, "regidx")) {
        slot = &g_tune.regidx;
        value = value ? 1 : 0;
    } else if (!strcmp(key, "readlane_min")) {
        MX_CHECK(value >= 8 && value <= 128, "mx_mix_set: readlane_min %d", value);
        slot = &g_tune.readlane_min;
    } else if (!strcmp(key, "grid")) {
        MX_CHECK(value >= 0 && value <= 65536, "mx_mix_set: grid %d", value);
        slot = &g_tune.grid;
    } else if (!strcmp(key, "chunked")) {
        slot = &g_tune.chunked;
        value = value ? 1 : 0;
    } else if (!strcmp(key, "rows")) {
        MX_CHECK(value >= 0 && value <= 2, "mx_mix_set: rows %d", value);
        slot = &g_tune.rows;
    } else if (!strcmp(key, "split")) {
        MX_CHECK(value == 0 || value == 1 || value == 2 || value == 4, "mx_mix_set: split %d", value);
        slot = &g_tune.split;
    } else if (!strcmp(key, "wide_lds_kb")) {
        MX_CHECK(value >= 8 && value <= 158, "mx_mix_set: wide_lds_kb %d", value);
        slot = &g_tune.wide_lds_kb;
    } else if (!strcmp(key, "rows_tpb")) {
        MX_CHECK(value == 256 || value == 512 || value == 1024, "mx_mix_set: rows_tpb %d", value);
        slot = &g_tune.rows_tpb;
    } else if (!strcmp(key, "wide_pf2")) {
        MX_CHECK(value == 0 || value == 1, "mx_mix_set: wide_pf2 %d", value);
        slot = &g_tune.wide_pf2;
    } else if (!strcmp(key, "wide_tpb")) {
        MX_CHECK(value == 256 || value == 512 || value == 1024, "mx_mix_set: wide_tpb %d", value);
        slot = &g_tune.wide_tpb;
    } else if (!strcmp(key, "wide_per_cu")) {
        MX_CHECK(value >= 0 && value <= 8, "mx_mix_set: wide_per_cu %d", value);
        slot = &g_tune.wide_per_cu;
    } else if (!strcmp(key, "wide_plan_lds")) {
        MX_CHECK(value == 0 || value == 1, "mx_mix_set: wide_plan_lds %d", value);
        slot = &g_tune.wide_plan_lds;
    } else if (!strcmp(key, "rows_pf2")) {
        MX_CHECK(value >= 0 && value <= 2, "mx_mix_set: rows_pf2 %d", value);
        slot = &g_tune.rows_pf2;
    } else if (!strcmp(key, "mid_bpc")) {
        MX_CHECK(value >= 0 && value <= 16, "mx_mix_set: mid_bpc %d", value);
        slot = &g_tune.mid_bpc;
    } else if (!strcmp(key, "mid_tiles")) {
        MX_CHECK(value >= 0 && value <= 1024, "mx_mix_set: mid_tiles %d", value);
        slot = &g_tune.mid_tiles;

    } else if (!strcmp(key, "spec")) {
        slot = &g_tune.spec;
        value = value ? 1 : 0;
    } else if (!strcmp(key, "spec_glds")) {
        slot = &g_tune.spec_glds;
        value = value ? 1 : 0;
    } else if (!strcmp(key, "spec_wgpc")) {
        MX_CHECK(value >= 0 && value <= 32, "mx_mix_set: spec_wgpc %d", value);
        slot = &g_tune.spec_wgpc;
    } else if (!strcmp(key, "mean_wgpc")) {
        MX_CHECK(value >= 0 && value <= 32, "mx_mix_set: mean_wgpc %d", value);
        slot = &mx::g_mean_wgpc;
    } else if (!strcmp(key, "flat_small")) {
        MX_CHECK(value >= 0 && value <= 4096, "mx_mix_set: flat_small %d", value);
        slot = &g_tune.flat_small;
    } else if (!strcmp(key, "ns48")) {
        slot = &g_ns48;
        value = value ? 1 : 0;
    }
    MX_CHECK(slot, "mx_mix_set: unknown key '%s'", key);
    *slot = value;
    return MX_OK;
}

extern "C" int mx_mix_get(const char* key) {
    if (!key) return MX_ERR_INVALID;
    if (!strcmp(key, "blocks_per_cu")) return g_tune.blocks_per_cu;
    if (!strcmp(key, "unroll")) return g_tune.unroll;
    if (!strcmp(key, "nontemporal")) return g_tune.nontemporal;
    if (!strcmp(key, "prefetch")) return g_tune.prefetch;
    if (!strcmp(key, "regidx")) return g_tune.regidx;
    if (!strcmp(key, "chunked")) return g_tune.chunked;
    if (!strcmp(key, "grid")) return g_tune.grid;
    if (!strcmp(key, "readlane_min")) return g_tune.readlane_min;
    if (!strcmp(key, "rows")) return g_tune.rows;
    if (!strcmp(key, "split")) return g_tune.split;
    if (!strcmp(key, "flat_small")) return g_tune.flat_small;
    if (!strcmp(key, "spec")) return g_tune.spec;
    if (!strcmp(key, "spec_wgpc")) return g_tune.spec_wgpc;
    if (!strcmp(key, "spec_glds")) return g_tune.spec_glds;
    if (!strcmp(key, "mean_wgpc")) return mx::g_mean_wgpc;
    if (!strcmp(key, "spec_launches")) return (int)(g_spec_launches.load() & 0x7fffffff);
    if (!strcmp(key, "mid_bpc")) return g_tune.mid_bpc;
    if (!strcmp(key, "mid_tiles")) return g_tune.mid_tiles;
    if (!strcmp(key, "rows_pf2")) return g_tune.rows_pf2;
    if (!strcmp(key, "wide_lds_kb")) return g_tune.wide_lds_kb;
    if (!strcmp(key, "wide_plan_lds")) return g_tune.wide_plan_lds;
    if (!strcmp(key, "wide_per_cu")) return g_tune.wide_per_cu;
    if (!strcmp(key, "wide_tpb")) return g_tune.wide_tpb;
    if (!strcmp(key, "wide_pf2")) return g_tune.wide_pf2;
    if (!strcmp(key, "rows_tpb")) return g_tune.rows_tpb;
    if (!strcmp(key, "ns48")) return g_ns48;
    mx::set_error("mx_mix_get: unknown key '%s'", key);
    return MX_ERR_INVALID;
}

// mirrors mx_gossip_mix's dispatch (for M <= 32 matchings; more always take mix_kernel_wide)
extern "C" const char* mx_mix_kernel_name(int n_slots) {
    const Cfg c = pick(n_slots);
    if (c.vec == 0) return "";
    if (c.ns == 0) return "mix_kernel_wide";
    if ((g_tune.rows && c.ns >= 16) || (g_tune.rows == 2 && unroll_for(8) <= 2)) return "mix_kernel_rows";
    if (g_tune.regidx && c.ns == 8) return "mix_kernel_reg";
    return "mix_kernel";
}

extern "C" int mx_mix_layout(const int64_t* seg_len_host, int nseg, int n_slots, int64_t* tile_off_host) {
    MX_CHECK(seg_len_host && tile_off_host && nseg >= 1, "mx_mix_layout: bad arguments");
    const int tile = mx_mix_tile(n_slots);
    MX_CHECK(tile > 0, "mx_mix_layout: n_slots=%d exceeds %d", n_slots, kWideMaxSlots);
    tile_off_host[0] = 0;
    for (int s = 0; s < nseg; ++s) {
        MX_CHECK(seg_len_host[s] >= 0, "mx_mix_layout: negative length");
        tile_off_host[s + 1] = tile_off_host[s] + (seg_len_host[s] + tile - 1) / tile;
    }
    return MX_OK;
}

namespace {
int gossip_mix(float* const* seg_ptrs_dev, const int64_t* seg_len_dev, const int64_t* tile_off_dev,
               const uint8_t* seg_vec_dev, int nseg, int64_t total_tiles, int n_slots, const int32_t* plan_dev,
               int64_t iter, const int64_t* iter_dev, int n_local, int M, float alpha, void* stream,
               uint64_t hint = 0);
}

extern "C" int mx_gossip_mix(float* const* seg_ptrs_dev, const int64_t* seg_len_dev,
                             const int64_t* tile_off_dev, const uint8_t* seg_vec_dev, int nseg,
                             int64_t total_tiles, int n_slots, const int32_t* plan_dev,
                             int64_t iter, int n_local, int M, float alpha, void* stream) {
    return gossip_mix(seg_ptrs_dev, seg_len_dev, tile_off_dev, seg_vec_dev, nseg, total_tiles, n_slots, plan_dev,
                      iter, nullptr, n_local, M, alpha, stream);
}

extern "C" int mx_gossip_mix_packed(const mx_mix_call* c, int64_t iter, void* stream) {
    MX_CHECK(c, "mx_gossip_mix_packed: null call record");
    MX_CHECK(!c->need_host || (iter >= 0 && iter < c->n_iters), "mx_gossip_mix_packed: iter %lld outside [0, %lld)",
             (long long)iter, (long long)c->n_iters);
    return gossip_mix(c->seg_ptrs_dev, c->seg_len_dev, c->tile_off_dev, c->seg_vec_dev, c->nseg, c->total_tiles,
                      c->n_slots, c->plan_dev, iter, nullptr, c->n_local, c->M, c->alpha, stream,
                      c->need_host ? c->need_host[iter] : 0);
}

extern "C" int mx_gossip_mix_at(float* const* seg_ptrs_dev, const int64_t* seg_len_dev,
                                const int64_t* tile_off_dev, const uint8_t* seg_vec_dev, int nseg,
                                int64_t total_tiles, int n_slots, const int32_t* plan_dev,
                                const int64_t* iter_dev, int64_t n_iters, int n_local, int M, float alpha,
                                void* stream) {
    MX_CHECK(iter_dev, "mx_gossip_mix_at: null iteration counter");
    return gossip_mix(seg_ptrs_dev, seg_len_dev, tile_off_dev, seg_vec_dev, nseg, total_tiles, n_slots, plan_dev,
                      n_iters, iter_dev, n_local, M, alpha, stream);
}

namespace {
__global__ void advance_kernel(int64_t* it, int64_t by) {
    if (threadIdx.x == 0 && blockIdx.x == 0) it[0] += by;
}
}  // namespace

namespace {
__global__ void expand_kernel(int64_t* it, int64_t* ctrs, int n) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const int64_t base = it[0];
    for (int j = 0; j < n; ++j) ctrs[j] = base + j;
    it[0] = base + n;
}
}  // namespace

// K graph-replayable rounds for one launch of bookkeeping: ctrs[j] = *iter_dev + j, then
// *iter_dev += n; the K mixing launches that follow read ctrs[0..K-1] (one counter each).
extern "C" int mx_iter_expand(int64_t* iter_dev, int64_t* ctrs, int n, void* stream) {
    MX_CHECK(iter_dev && ctrs && n >= 1, "mx_iter_expand: bad arguments");
    hipLaunchKernelGGL(expand_kernel, dim3(1), dim3(64), 0, mx::as_stream(stream), iter_dev, ctrs, n);
    MX_LAUNCH_CHECK();
    return MX_OK;
}

extern "C" int mx_iter_advance(int64_t* iter_dev, int64_t by, void* stream) {
    MX_CHECK(iter_dev, "mx_iter_advance: null counter");
    hipLaunchKernelGGL(advance_kernel, dim3(1), dim3(64), 0, mx::as_stream(stream), iter_dev, by);
    MX_LAUNCH_CHECK();
    return MX_OK;
}

namespace {
int gossip_mix(float* const* seg_ptrs_dev, const int64_t* seg_len_dev, const int64_t* tile_off_dev,
               const uint8_t* seg_vec_dev, int nseg, int64_t total_tiles, int n_slots, const int32_t* plan_dev,
               int64_t iter, const int64_t* iter_dev, int n_local, int M, float alpha, void* stream,
               uint64_t hint) {
    MX_CHECK(seg_ptrs_dev && seg_len_dev && tile_off_dev && seg_vec_dev && plan_dev,
             "mx_gossip_mix: null pointer");
    MX_CHECK(nseg >= 1 && n_local >= 1 && n_slots >= n_local, "mx_gossip_mix: nseg=%d n_local=%d n_slots=%d",
             nseg, n_local, n_slots);
    MX_CHECK(M >= 1, "mx_gossip_mix: M=%d", M);
    MX_CHECK(iter >= 0, "mx_gossip_mix: iter < 0");
    const Cfg c = pick(n_slots);
    MX_CHECK(c.vec > 0, "mx_gossip_mix: n_slots=%d exceeds %d", n_slots, kWideMaxSlots);
    hipStream_t st = mx::as_stream(stream);
    if (total_tiles <= 0) return MX_OK;
    if (c.ns == 0 || M > kMaxM) {             // wide kernel: > 64 slots or > 32 matchings
        const int tile_cols = mx_mix_tile(n_slots);
        // the widest piece (64 x VEC columns of every slot) within the LDS budget (default 40 KB:
        // 4 workgroups per CU); the persistent grid as many per CU as that LDS allows (<= 4)
        const size_t budget = (size_t)g_tune.wide_lds_kb * 1024;
        int vec = 1;
        if ((size_t)n_slots * 64 * 4 * sizeof(float) <= budget) vec = 4;
        else if ((size_t)n_slots * 64 * 2 * sizeof(float) <= budget) vec = 2;
        const size_t plan_bytes = (size_t)mx::plan_words(n_local, M) * sizeof(int32_t);
        const size_t piece_bytes = (size_t)n_slots * 64 * vec * sizeof(float);
        auto fit = [](size_t b) { return std::min<int64_t>(4, (int64_t)((159 * 1024) / b)); };
        // the plan goes to LDS only when it costs no workgroup per CU (occupancy beats ds_read here)
        const bool plds = g_tune.wide_plan_lds && plan_bytes <= 32 * 1024 &&
                          piece_bytes + plan_bytes <= 158 * 1024 && fit(piece_bytes + plan_bytes) == fit(piece_bytes);
        const size_t lds = (size_t)n_slots * 64 * vec * sizeof(float) + (plds ? plan_bytes : 0);
        MX_CHECK(lds <= 158 * 1024, "mx_gossip_mix: wide kernel LDS %zu", lds);
        const int tpb = g_tune.wide_tpb;
        int64_t per_cu = (int64_t)((159 * 1024) / lds);
        int64_t cap = g_tune.wide_per_cu > 0 ? g_tune.wide_per_cu : 4;
        if (cap > 2048 / tpb) cap = 2048 / tpb;  // 32 waves per CU
        per_cu = per_cu > cap ? cap : per_cu < 1 ? 1 : per_cu;
        int64_t grid = (int64_t)cu_count() * per_cu;
        const int64_t work = total_tiles * (tile_cols / (64 * vec));
        if (grid > work) grid = work;
        const bool nt = g_tune.nontemporal != 0;
        const bool big = (vec == 4 && n_slots > 40) || (vec == 2 && n_slots > 80);
        MX_CHECK(n_slots <= (big || vec == 1 ? kWideMaxSlots : vec == 4 ? 40 : 80), "mx_gossip_mix: wide staging");
#define MX_WIDE1(V, N, B, PL, T, F2)                                                                           \
    do {                                                                                                      \
        static bool big_lds = false;          /* once per instantiation: the most the kernel may ask */   \
        if (lds > 64 * 1024 && !big_lds) {                                                                    \
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(mix_kernel_wide<V, N, B, PL, T, F2>),     \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 158 * 1024);               \
            big_lds = true;                                                                                   \
        }                                                                                                     \
        hipLaunchKernelGGL((mix_kernel_wide<V, N, B, PL, T, F2>), dim3((unsigned)(grid < 1 ? 1 : grid)),      \
                           dim3(T), lds, st, seg_ptrs_dev, seg_len_dev, tile_off_dev, seg_vec_dev, nseg,      \
                           total_tiles, tile_cols, n_slots, plan_dev, iter, iter_dev, n_local, M, alpha);     \
    } while (0)
#define MX_WIDE2(V, N, B, PL)                                                                                 \
    do {                                                                                                      \
        if (tpb == 1024 && g_tune.wide_pf2) MX_WIDE1(V, N, B, PL, 1024, true);                               \
        else if (tpb == 1024) MX_WIDE1(V, N, B, PL, 1024, false);                                            \
        else if (tpb == 512) MX_WIDE1(V, N, B, PL, 512, false);                                              \
        else MX_WIDE1(V, N, B, PL, 256, false);                                                              \
    } while (0)
#define MX_WIDE(V, N, B)                                                                                      \
    do {                                                                                                      \
        if (plds) MX_WIDE2(V, N, B, true); else MX_WIDE2(V, N, B, false);                                     \
    } while (0)
        if (vec == 4 && big) { if (nt) MX_WIDE(4, true, true); else MX_WIDE(4, false, true); }
        else if (vec == 4) { if (nt) MX_WIDE(4, true, false); else MX_WIDE(4, false, false); }
        else if (vec == 2 && big) { if (nt) MX_WIDE(2, true, true); else MX_WIDE(2, false, true); }
        else if (vec == 2) { if (nt) MX_WIDE(2, true, false); else MX_WIDE(2, false, false); }
        else { if (nt) MX_WIDE(1, true, false); else MX_WIDE(1, false, false); }
#undef MX_WIDE
#undef MX_WIDE2
#undef MX_WIDE1
        MX_LAUNCH_CHECK();
        return MX_OK;
    }
    const int key = (g_tune.nontemporal ? 1 : 0) | (g_tune.prefetch ? 2 : 0);
#define MX_ARGS seg_ptrs_dev, seg_len_dev, tile_off_dev, seg_vec_dev, nseg, n_slots, plan_dev, iter, \
                iter_dev, n_local, M, alpha, total_tiles, st
#define MX_DISPATCH(V, N, U)                                                  \
    switch (key) {                                                            \
        case 0: return launch<V, N, U, false, false>(MX_ARGS);                \
        case 1: return launch<V, N, U, true, false>(MX_ARGS);                 \
        case 2: return launch<V, N, U, false, true>(MX_ARGS);                 \
        default: return launch<V, N, U, true, true>(MX_ARGS);                 \
    }
#define MX_DISPATCH_REG(N, U)                                                 \
    switch (key) {                                                            \
        case 0: return launch_reg<N, U, false, false>(MX_ARGS);               \
        case 1: return launch_reg<N, U, true, false>(MX_ARGS);                \
        case 2: return launch_reg<N, U, false, U == 1>(MX_ARGS);              \
        default: return launch_reg<N, U, true, U == 1>(MX_ARGS);              \
    }
    if ((g_tune.rows && c.ns >= 16) || (g_tune.rows == 2 && unroll_for(8) <= 2)) {
        // auto: rows of 32-320 MB (about the 256 MB Infinity Cache) keep ordinary (cacheable)
        // accesses -- back-to-back rounds then find them on die (8 x 2M params 25.1 -> 23.7 us,
        // 8 x 8M 90.3 -> 75.2 us, 8 x 10M 111.5 -> 107.7 us); above, the streaming hints win
        // (8 x 12M 138.9 -> 130.8 us, headline 294 -> 272 us), and below, where the rows fit in the
        // L2s, too (8 x 181k / 666k: 5-7 % slower with ordinary accesses; tools/sessions/r2_s80.sh)
        const int64_t ws = total_tiles * (int64_t)mx_mix_tile(n_slots) * n_slots * 4;
        const bool nt = g_tune.nontemporal == 2 ? (ws <= ((int64_t)32 << 20) || ws > ((int64_t)320 << 20))
                                                : g_tune.nontemporal != 0;
        if (c.ns == 8 && unroll_for(8) == 2)
            return nt ? launch_rows<8, 2048, true>(MX_ARGS) : launch_rows<8, 2048, false>(MX_ARGS);
        const int sp = row_split(c.ns, total_tiles);
#define MX_ROWS(N, TW, S) (nt ? launch_rows<N, TW, true, S>(MX_ARGS) : launch_rows<N, TW, false, S>(MX_ARGS))
        if (c.ns == 8) {
            // SPEC (knob "spec"): a round whose local active rows the caller passed (hint, from the
            // host's copy of the flags: mx_gossip_mix_packed) loads their first tile before the plan
            // record arrives, at spec_wgpc workgroups per CU -- 8-slot rounds of > 64 MB on the flat
            // grid with streaming hints (auto hints: > 320 MB; 8 x 14.8M-60M params: -0.5 to -3.5 %,
            // the headline 0.2700 -> 0.2637 ms; neutral at 8 x 4M; tools/occ_sweep.py, profiles/r06t_*)
            const int64_t work = total_tiles * sp;
            const bool flat = !rows_mid(8, total_tiles) && g_tune.flat_small > 0 && g_tune.grid == 0 &&
                              work <= (int64_t)g_tune.flat_small * grid_target();
            // only when every slot is a local row: receive slots (RCCL slab, or a peer's HBM under the
            // pull transport, read over xGMI) keep the uncapped launch measured at N > 1
            if (nt && hint && g_tune.spec && flat && n_slots == n_local && ws > ((int64_t)64 << 20)) {
                g_rows_opt.hint = hint;
                g_rows_opt.wg_per_cu = g_tune.spec_wgpc;
                ++g_spec_launches;
                if (g_tune.spec_glds && sp == 2) return launch_rows<8, 512, true, 2, false, kTPB, true, true>(MX_ARGS);
                return sp == 4 ? launch_rows<8, 256, true, 4, false, kTPB, true>(MX_ARGS)
                               : sp == 2 ? launch_rows<8, 512, true, 2, false, kTPB, true>(MX_ARGS)
                                         : launch_rows<8, 1024, true, 1, false, kTPB, true>(MX_ARGS);
            }
            return sp == 4 ? MX_ROWS(8, 256, 4) : sp == 2 ? MX_ROWS(8, 512, 2) : MX_ROWS(8, 1024, 1);
        }
        if (c.ns == 16) return sp == 4 ? MX_ROWS(16, 256, 4) : sp == 2 ? MX_ROWS(16, 512, 2) : MX_ROWS(16, 1024, 1);
#define MX_ROWSP(N, TW, S)                                                                                  \
    ((g_tune.rows_pf2 == 1 || (g_tune.rows_pf2 == 2 && 8 * n_slots <= 5 * (N)))                                  \
         ? (nt ? launch_rows<N, TW, true, S, true>(MX_ARGS) : launch_rows<N, TW, false, S, true>(MX_ARGS))     \
         : MX_ROWS(N, TW, S))
#define MX_ROWST(N, TW, T)                                                                                  \
    ((g_tune.rows_pf2 == 1 || (g_tune.rows_pf2 == 2 && 8 * n_slots <= 5 * (N)))                                  \
         ? (nt ? launch_rows<N, TW, true, 1, true, T>(MX_ARGS) : launch_rows<N, TW, false, 1, true, T>(MX_ARGS)) \
         : (nt ? launch_rows<N, TW, true, 1, false, T>(MX_ARGS) : launch_rows<N, TW, false, 1, false, T>(MX_ARGS)))
#define MX_ROWSW(N, TW)                                                                                     \
    (g_tune.rows_tpb == 1024 ? MX_ROWST(N, TW, 1024) : g_tune.rows_tpb == 512 ? MX_ROWST(N, TW, 512) : MX_ROWSP(N, TW, 1))
        if (c.ns == 32) return sp == 2 ? MX_ROWSP(32, 256, 2) : MX_ROWSW(32, 512);
        if (c.ns == 48) return MX_ROWSW(48, 256);
        return MX_ROWSW(64, 256);
#undef MX_ROWSW
#undef MX_ROWST
#undef MX_ROWSP
#undef MX_ROWS
    }
    if (g_tune.regidx && c.ns == 8) {
        if (unroll_for(8) == 4) { MX_DISPATCH_REG(8, 4) }
        if (unroll_for(8) == 2) { MX_DISPATCH_REG(8, 2) }
        MX_DISPATCH_REG(8, 1)
    }
    switch (c.ns) {
        case 8:
            if (unroll_for(8) == 2) { MX_DISPATCH(4, 8, 2) }
            MX_DISPATCH(4, 8, 1)
        case 16:
            MX_DISPATCH(4, 16, 1)
        case 32:
            MX_DISPATCH(2, 32, 1)
        default:
            MX_DISPATCH(1, 64, 1)
    }
#undef MX_DISPATCH
#undef MX_DISPATCH_REG
#undef MX_ARGS
}
}  // namespace
