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
#include "mx_common.h"

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

template <bool NT, typename F>
__device__ __forceinline__ F ld(const float* p) {
    if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const F*>(p));
    else return *reinterpret_cast<const F*>(p);
}

template <bool NT, typename F>
__device__ __forceinline__ void st(float* p, const F& v) {
    if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<F*>(p));
    else *reinterpret_cast<F*>(p) = v;
}

// VEC floats per lane access (16 B for VEC = 4), NS slots (LDS rows), U accesses per lane per
// row per tile (U * 256 * VEC floats per tile), NT: non-temporal (streaming) loads/stores.
template <int VEC, int NS, int U, bool NT, bool PF>
__global__ __launch_bounds__(kTPB) void mix_kernel(float* const* __restrict__ seg_ptrs,
                                                   const int64_t* __restrict__ seg_len,
                                                   const int64_t* __restrict__ tile_off,
                                                   const uint8_t* __restrict__ seg_vec, int nseg,
                                                   int64_t total_tiles, int n_slots,
                                                   const int32_t* __restrict__ plan, int64_t iter,
                                                   int n_local, int M, float alpha) {
    using F = typename VT<VEC>::type;
    constexpr int TILE = kTPB * VEC * U;
    __shared__ F lds[NS][U][kTPB];
    __shared__ int32_t sp[mx::kPlanHeader + 2 * NS + NS * kMaxM];

    const int tid = threadIdx.x;
    const int64_t W = mx::plan_words(n_local, M);
    const int32_t* rec = plan + iter * W;
    for (int i = tid; i < W; i += kTPB) sp[i] = rec[i];
    __syncthreads();
    if (sp[0] == 0) return;  // all flags zero: the reference returns before any I/O

    const int n_remote = sp[1];
    const int32_t* deg = sp + mx::kPlanHeader;
    const float* sw = reinterpret_cast<const float*>(deg + n_local);
    const int32_t* src = deg + 2 * n_local;
    uint64_t need = 0;
    for (int r = 0; r < n_local; ++r)
        if (deg[r] > 0) need |= 1ull << r;
    for (int k = 0; k < n_remote; ++k) need |= 1ull << (n_local + k);

    // tile -> (segment, first column of this lane, full-vector flag)
    auto locate = [&](int64_t tile, int& seg, int64_t& c0, bool& full) {
        seg = 0;
        if (nseg > 1) {
            int lo = 0, hi = nseg;
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (tile_off[mid] <= tile) lo = mid; else hi = mid;
            }
            seg = lo;
        }
        const int64_t len = seg_len[seg];
        c0 = (tile - tile_off[seg]) * TILE + (int64_t)tid * VEC;
        full = (c0 + (int64_t)(U - 1) * kTPB * VEC + VEC <= len) && seg_vec[seg];
    };
    F v[NS][U];
    auto load = [&](int seg, int64_t c0, bool full) {
        const int64_t len = seg_len[seg];
        float* const* ptrs = seg_ptrs + (int64_t)seg * n_slots;
#pragma unroll
        for (int k = 0; k < NS; ++k) {
            if ((need >> k) & 1ull) {
                const float* p = ptrs[k] + c0;
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    if (full) {
                        v[k][u] = ld<NT, F>(p + u * kTPB * VEC);
                    } else {
                        const int64_t c = c0 + (int64_t)u * kTPB * VEC;
#pragma unroll
                        for (int j = 0; j < VEC; ++j)
                            v[k][u][j] = (c + j < len) ? p[u * kTPB * VEC + j] : 0.0f;
                    }
                }
            }
        }
    };

    int64_t tile = blockIdx.x;
    if (tile >= total_tiles) return;
    int seg;
    int64_t c0;
    bool full;
    locate(tile, seg, c0, full);
    load(seg, c0, full);
    while (true) {
#pragma unroll
        for (int k = 0; k < NS; ++k)
            if ((need >> k) & 1ull) {
#pragma unroll
                for (int u = 0; u < U; ++u) lds[k][u][tid] = v[k][u];
            }
        // registers are free again: with PF, start streaming the next tile before this one is
        // mixed and stored, so its loads are older than this tile's stores in vmcnt order
        const int64_t next = tile + gridDim.x;
        int nseg_i = 0;
        int64_t nc0 = 0;
        bool nfull = false;
        if (PF && next < total_tiles) {
            locate(next, nseg_i, nc0, nfull);
            load(nseg_i, nc0, nfull);
        }
        const int64_t len = seg_len[seg];
        float* const* ptrs = seg_ptrs + (int64_t)seg * n_slots;
        for (int r = 0; r < n_local; ++r) {
            const int d = deg[r];
            if (d == 0) continue;
            F acc[U];
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int j = 0; j < VEC; ++j) acc[u][j] = 0.0f;
            for (int e = 0; e < d; ++e) {
                const int sl = src[r * M + e];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const F x = lds[sl][u][tid];
#pragma unroll
                    for (int j = 0; j < VEC; ++j) acc[u][j] = __builtin_fmaf(alpha, x[j], acc[u][j]);
                }
            }
            const float s = sw[r];
            float* p = ptrs[r] + c0;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const F xs = lds[r][u][tid];
#pragma unroll
                for (int j = 0; j < VEC; ++j) acc[u][j] = __builtin_fmaf(s, xs[j], acc[u][j]);
                if (full) {
                    st<NT, F>(p + u * kTPB * VEC, acc[u]);
                } else {
                    const int64_t c = c0 + (int64_t)u * kTPB * VEC;
#pragma unroll
                    for (int j = 0; j < VEC; ++j)
                        if (c + j < len) p[u * kTPB * VEC + j] = acc[u][j];
                }
            }
        }
        if (next >= total_tiles) break;
        tile = next;
        if (PF) {
            seg = nseg_i;
            c0 = nc0;
            full = nfull;
        } else {
            locate(tile, seg, c0, full);
            load(seg, c0, full);
        }
    }
}


// Register-indexed variant (VEC = 4): the tile of every slot is kept in ONE register vector of
// NS*4 floats; the wave-uniform partner slot indexes it through s_set_gpr_idx (VGPR indexing
// mode), so no LDS is used and occupancy is bounded by VGPRs only.  PF double-buffers the
// vector so the next tile's loads are in flight while this one is mixed and stored.
template <int NS>
using RegVec = float __attribute__((ext_vector_type(NS * 4)));

template <int NS, bool NT, bool PF>
__global__ __launch_bounds__(kTPB) void mix_kernel_reg(float* const* __restrict__ seg_ptrs,
                                                       const int64_t* __restrict__ seg_len,
                                                       const int64_t* __restrict__ tile_off,
                                                       const uint8_t* __restrict__ seg_vec, int nseg,
                                                       int64_t total_tiles, int n_slots,
                                                       const int32_t* __restrict__ plan, int64_t iter,
                                                       int n_local, int M, float alpha) {
    using F = typename VT<4>::type;
    constexpr int TILE = kTPB * 4;
    __shared__ int32_t sp[mx::kPlanHeader + 2 * NS + NS * kMaxM];
    const int tid = threadIdx.x;
    const int64_t W = mx::plan_words(n_local, M);
    const int32_t* rec = plan + iter * W;
    for (int i = tid; i < W; i += kTPB) sp[i] = rec[i];
    __syncthreads();
    if (sp[0] == 0) return;
    const int n_remote = sp[1];
    const int32_t* deg = sp + mx::kPlanHeader;
    const float* sw = reinterpret_cast<const float*>(deg + n_local);
    const int32_t* src = deg + 2 * n_local;
    uint64_t need = 0;
    for (int r = 0; r < n_local; ++r)
        if (deg[r] > 0) need |= 1ull << r;
    for (int k = 0; k < n_remote; ++k) need |= 1ull << (n_local + k);

    auto locate = [&](int64_t tile, int& seg, int64_t& c0, bool& full) {
        seg = 0;
        if (nseg > 1) {
            int lo = 0, hi = nseg;
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (tile_off[mid] <= tile) lo = mid; else hi = mid;
            }
            seg = lo;
        }
        c0 = (tile - tile_off[seg]) * TILE + (int64_t)tid * 4;
        full = (c0 + 4 <= seg_len[seg]) && seg_vec[seg];
    };
    auto load = [&](RegVec<NS>& a, int seg, int64_t c0, bool full) {
        const int64_t len = seg_len[seg];
        float* const* ptrs = seg_ptrs + (int64_t)seg * n_slots;
#pragma unroll
        for (int k = 0; k < NS; ++k) {
            if ((need >> k) & 1ull) {
                const float* p = ptrs[k] + c0;
                if (full) {
                    const F q = ld<NT, F>(p);
                    a[4 * k + 0] = q[0];
                    a[4 * k + 1] = q[1];
                    a[4 * k + 2] = q[2];
                    a[4 * k + 3] = q[3];
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j) a[4 * k + j] = (c0 + j < len) ? p[j] : 0.0f;
                }
            }
        }
    };

    int64_t tile = blockIdx.x;
    if (tile >= total_tiles) return;
    int seg;
    int64_t c0;
    bool full;
    locate(tile, seg, c0, full);
    RegVec<NS> cur, nxt;
    load(cur, seg, c0, full);
    while (true) {
        const int64_t next = tile + gridDim.x;
        int nseg_i = 0;
        int64_t nc0 = 0;
        bool nfull = false;
        if (PF && next < total_tiles) {
            locate(next, nseg_i, nc0, nfull);
            load(nxt, nseg_i, nc0, nfull);
        }
        const int64_t len = seg_len[seg];
        float* const* ptrs = seg_ptrs + (int64_t)seg * n_slots;
        for (int r = 0; r < n_local; ++r) {
            const int d = deg[r];
            if (d == 0) continue;
            F acc = {0.0f, 0.0f, 0.0f, 0.0f};
            for (int e = 0; e < d; ++e) {
                const int s4 = 4 * __builtin_amdgcn_readfirstlane(src[r * M + e]);
                acc[0] = __builtin_fmaf(alpha, cur[s4 + 0], acc[0]);
                acc[1] = __builtin_fmaf(alpha, cur[s4 + 1], acc[1]);
                acc[2] = __builtin_fmaf(alpha, cur[s4 + 2], acc[2]);
                acc[3] = __builtin_fmaf(alpha, cur[s4 + 3], acc[3]);
            }
            const int r4 = 4 * __builtin_amdgcn_readfirstlane(r);
            const float s = sw[r];
            acc[0] = __builtin_fmaf(s, cur[r4 + 0], acc[0]);
            acc[1] = __builtin_fmaf(s, cur[r4 + 1], acc[1]);
            acc[2] = __builtin_fmaf(s, cur[r4 + 2], acc[2]);
            acc[3] = __builtin_fmaf(s, cur[r4 + 3], acc[3]);
            float* p = ptrs[r] + c0;
            if (full) {
                st<NT, F>(p, acc);
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (c0 + j < len) p[j] = acc[j];
            }
        }
        if (next >= total_tiles) break;
        tile = next;
        if (PF) {
            seg = nseg_i;
            c0 = nc0;
            full = nfull;
            cur = nxt;
        } else {
            locate(tile, seg, c0, full);
            load(cur, seg, c0, full);
        }
    }
}

struct Cfg {
    int vec, ns;
};

Cfg pick(int n_slots) {
    if (n_slots <= 8) return {4, 8};
    if (n_slots <= 16) return {4, 16};
    if (n_slots <= 32) return {2, 32};
    if (n_slots <= 64) return {1, 64};
    return {0, 0};
}

// tuning state (mx_mix_tune); defaults chosen from measurements on MI355X
struct Tune {
    int blocks_per_cu = 4;
    int unroll = 1;      // 1 or 2 accesses per lane per row per tile (NS = 8 config only)
    int nontemporal = 1;
    int prefetch = 0;
    int regidx = 0;      // 1: register-indexed kernel (n_slots <= 8; wider spills), 0: LDS-column kernel
};
Tune g_tune;

int unroll_for(int ns) { return (ns == 8 && !g_tune.regidx) ? g_tune.unroll : 1; }

int cu_count() {
    static int v = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess) return 256;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 256;
        return n > 0 ? n : 256;
    }();
    return v;
}

template <int VEC, int NS, int U, bool NT, bool PF>
int launch(float* const* seg_ptrs, const int64_t* seg_len, const int64_t* tile_off,
           const uint8_t* seg_vec, int nseg, int n_slots, const int32_t* plan, int64_t iter,
           int n_local, int M, float alpha, int64_t total_tiles, hipStream_t st) {
    int64_t grid = (int64_t)cu_count() * g_tune.blocks_per_cu;
    if (grid > total_tiles) grid = total_tiles;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL((mix_kernel<VEC, NS, U, NT, PF>), dim3((unsigned)grid), dim3(kTPB), 0, st, seg_ptrs,
                       seg_len, tile_off, seg_vec, nseg, total_tiles, n_slots, plan, iter, n_local,
                       M, alpha);
    MX_LAUNCH_CHECK();
    return MX_OK;
}
template <int NS, bool NT, bool PF>
int launch_reg(float* const* seg_ptrs, const int64_t* seg_len, const int64_t* tile_off,
               const uint8_t* seg_vec, int nseg, int n_slots, const int32_t* plan, int64_t iter,
               int n_local, int M, float alpha, int64_t total_tiles, hipStream_t st) {
    int64_t grid = (int64_t)cu_count() * g_tune.blocks_per_cu;
    if (grid > total_tiles) grid = total_tiles;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL((mix_kernel_reg<NS, NT, PF>), dim3((unsigned)grid), dim3(kTPB), 0, st, seg_ptrs,
                       seg_len, tile_off, seg_vec, nseg, total_tiles, n_slots, plan, iter, n_local,
                       M, alpha);
    MX_LAUNCH_CHECK();
    return MX_OK;
}

}  // namespace

extern "C" int mx_mix_tile(int n_slots) {
    const Cfg c = pick(n_slots);
    return c.vec * kTPB * unroll_for(c.ns);
}

extern "C" int mx_mix_tune(int blocks_per_cu, int unroll, int nontemporal, int prefetch, int regidx) {
    MX_CHECK(blocks_per_cu >= 1 && blocks_per_cu <= 64, "mx_mix_tune: blocks_per_cu %d", blocks_per_cu);
    MX_CHECK(unroll == 1 || unroll == 2, "mx_mix_tune: unroll %d", unroll);
    g_tune.blocks_per_cu = blocks_per_cu;
    g_tune.unroll = unroll;
    g_tune.nontemporal = nontemporal ? 1 : 0;
    g_tune.prefetch = prefetch ? 1 : 0;
    g_tune.regidx = regidx ? 1 : 0;
    return MX_OK;
}

extern "C" int mx_mix_layout(const int64_t* seg_len_host, int nseg, int n_slots, int64_t* tile_off_host) {
    MX_CHECK(seg_len_host && tile_off_host && nseg >= 1, "mx_mix_layout: bad arguments");
    const int tile = mx_mix_tile(n_slots);
    MX_CHECK(tile > 0, "mx_mix_layout: n_slots=%d exceeds 64", n_slots);
    tile_off_host[0] = 0;
    for (int s = 0; s < nseg; ++s) {
        MX_CHECK(seg_len_host[s] >= 0, "mx_mix_layout: negative length");
        tile_off_host[s + 1] = tile_off_host[s] + (seg_len_host[s] + tile - 1) / tile;
    }
    return MX_OK;
}

extern "C" int mx_gossip_mix(float* const* seg_ptrs_dev, const int64_t* seg_len_dev,
                             const int64_t* tile_off_dev, const uint8_t* seg_vec_dev, int nseg,
                             int64_t total_tiles, int n_slots, const int32_t* plan_dev,
                             int64_t iter, int n_local, int M, float alpha, void* stream) {
    MX_CHECK(seg_ptrs_dev && seg_len_dev && tile_off_dev && seg_vec_dev && plan_dev,
             "mx_gossip_mix: null pointer");
    MX_CHECK(nseg >= 1 && n_local >= 1 && n_slots >= n_local, "mx_gossip_mix: nseg=%d n_local=%d n_slots=%d",
             nseg, n_local, n_slots);
    MX_CHECK(M >= 1 && M <= kMaxM, "mx_gossip_mix: M=%d outside [1, %d]", M, kMaxM);
    MX_CHECK(iter >= 0, "mx_gossip_mix: iter < 0");
    const Cfg c = pick(n_slots);
    MX_CHECK(c.vec > 0, "mx_gossip_mix: n_slots=%d exceeds 64", n_slots);
    hipStream_t st = mx::as_stream(stream);
    if (total_tiles <= 0) return MX_OK;
    const int key = (g_tune.nontemporal ? 1 : 0) | (g_tune.prefetch ? 2 : 0);
#define MX_ARGS seg_ptrs_dev, seg_len_dev, tile_off_dev, seg_vec_dev, nseg, n_slots, plan_dev, iter, \
                n_local, M, alpha, total_tiles, st
#define MX_DISPATCH(V, N, U)                                                  \
    switch (key) {                                                            \
        case 0: return launch<V, N, U, false, false>(MX_ARGS);                \
        case 1: return launch<V, N, U, true, false>(MX_ARGS);                 \
        case 2: return launch<V, N, U, false, true>(MX_ARGS);                 \
        default: return launch<V, N, U, true, true>(MX_ARGS);                 \
    }
#define MX_DISPATCH_REG(N)                                                    \
    switch (key) {                                                            \
        case 0: return launch_reg<N, false, false>(MX_ARGS);                  \
        case 1: return launch_reg<N, true, false>(MX_ARGS);                   \
        case 2: return launch_reg<N, false, true>(MX_ARGS);                   \
        default: return launch_reg<N, true, true>(MX_ARGS);                   \
    }
    if (g_tune.regidx && c.ns == 8) { MX_DISPATCH_REG(8) }
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
