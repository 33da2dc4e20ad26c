// choco.hip -- ChocoSGD compressed gossip on the GPU.
//
// mx_topk_abs_diff  = compressors.get_top_k (compressors.py:3-19) applied to
//                     send = x - x_hat (ChocoCommunicator.prepare_comm_buffer, communicator.py:188-190)
// mx_choco_apply    = ChocoCommunicator.averaging (communicator.py:200-230)
//
// Top-k (k largest |x - x_hat|, ties at the threshold resolved towards the lowest indices,
// output in index order) with ONE full streaming pass over x / x_hat:
//   S  sample_kernel   12-bit histogram of the magnitude key's top digit (bits 19..30: exponent +
//                      4 mantissa bits) over every S-th 1024-element piece (S = 1: all of them);
//   B  compact_kernel  THE full pass.  Every block resolves the candidate floor b_lo from the
//                      sample (S = 1: exactly the digit of the k-th largest key; S > 1: k scaled
//                      to the sample with a 25 % + 4 sigma margin), then, one 4096-element chunk
//                      per block iteration, stores every key whose digit is >= b_lo as (value,
//                      chunk-local index) into the chunk's own region in index order (wave scans
//                      + one barrier), counts its top digit into the 12-bit candidate histogram
//                      and adds the block's kept count to the row's candidate total;
//                      in the (sample-dependent, rare) case that fewer than k were kept, the
//                      first candidate pass re-runs the compaction with b_lo = 0 (into a histogram
//                      of its own) on its own blocks before histogramming (a row grid barrier in
//                      that path only) -- the result is exact either way;
//   C  cand_hist<10>, cand_hist<9>: the 10- and 9-bit digits of the candidates matching the
//      prefix resolved so far; every block of a pass re-resolves the previous histograms itself
//      (find_bin, read-only), so no one-block select launches sit between the passes;
//      cand_mark resolves the exact threshold key T and the number of its ties to take, and
//      counts > T / == T per chunk and per block (contiguous chunk ranges); write_cand places each
//      chunk's output from those (block totals before it + a few chunk counts, no scan launch;
//      a last-block scan tail was tried and dropped: the device-scope fence every block then needs
//      writes back and invalidates the XCD's L2) and emits the selected candidates in index order
//      (values = x - x_hat, int64 indices) and, optionally, the message's per-4096-element tile
//      bounds that mx_choco_apply reads (the output offset of every chunk), and re-zeroes the
//      histograms / counters for the next call.
// Everything stays on the device; no host round trip.  All local workers' rows are processed by
// the same launches (blockIdx.y = row): 6 launches per call for any number of rows (the fallback
// compaction that sampling may need rides in the first candidate pass: no launch of its own).
//
// Work invariant: the histograms and the candidate total are zero on entry (the
// caller zero-fills the scratch once; every call leaves it that way), so no zeroing launch runs.
#include "mx_common.h"

#include <mutex>

namespace {
constexpr int kTPB = 256;
constexpr int kWaves = kTPB / 64;
constexpr int kSub = 1024;                   // elements per wave step = 4 quads x 64 lanes
constexpr int kSubQuads = kSub / 4;
constexpr int kChunk = kWaves * kSub;        // elements per chunk = one block (candidate region)
constexpr int kTopBits = 12, kTopShift = 19;
constexpr int kTopBins = 1 << kTopBits;
constexpr int kMidBits = 10, kMidShift = 9;  // bits 9..18
constexpr int kLowBits = 9;                  // bits 0..8
constexpr int64_t kSampleTarget = 1 << 18;   // sampled elements per row (auto stride)

// fine sampled floor ("fine_floor"): a window of kWinBins top digits around the last call's floor
// digit, each split into kFineSub sub-bins (key bits 13..18), sampled beside the 12-bit histogram
constexpr int kWinBins = 4, kFineSub = 64, kFineShift = 13;
constexpr int kFineBins = kWinBins * kFineSub;
constexpr int kHistWords = 3 * kTopBins + (1 << kMidBits) + (1 << kLowBits) + kFineBins;   // hs, h12, h12f, h10, h9, hsf

struct SelState {
    uint32_t b0;          // lowest top digit kept as a candidate (b_lo)
    uint32_t T;           // exact threshold key (cand_mark / select_kernel)
    int64_t need;         // ties of T to take (cand_mark / select_kernel)
    unsigned long long cand_n;   // candidates kept by the first compact_kernel pass (zero on entry)
    uint32_t bar;         // arrivals at the row's grid barriers (zeroed by the compaction pass)
    uint32_t err;         // sticky: a row barrier's bounded wait expired (select_kernel)
    // floor hint (mx_topk_set "floor_hint"): the last call's exact k-th key's top digit and the
    // row's adaptive margin below it, written by the call's threshold pass; call / fallback counts
    uint32_t hint_digit, hint_ok, margin;
    uint32_t n_calls, n_fallbacks;
    uint32_t last_cand;   // the last call's candidate count (keys kept by its first compaction)
    uint32_t win_digit;   // the last call's floor digit (fine_floor's window; b0 itself is rewritten
                          // by the compaction while its other blocks still read the window)
    int32_t scan;         // row 0 only: mx_topk_check's result (first row with `err` set, or -1)
};
static_assert(sizeof(SelState) <= 64, "SelState must fit its 64-byte slot");

// Per-chunk counters and per-block totals are 64-byte records, each written whole by one store
// instruction (a record half-written by two kernels / two blocks is a partial-sector write).  Padding
// the candidate regions' last lines the same way measured neutral (same-box A/B) and is not done.
constexpr int kRec = 8;                      // int64 words per record
// Candidate regions (one per chunk, filled from its start, ~1-6 % used) are strided 256 B beyond
// their 16 / 8 KB so the region heads every pass touches spread over the HBM channels instead of
// all sitting at the same offset of 16 KB-aligned windows.
constexpr int kCvLd = kChunk + 64;           // floats per value region
constexpr int kClLd = kChunk + 128;          // uint16 per index region

struct WorkLayout {
    size_t hist, state, cnt, bt, cval, cloc, pub, total;
};

// select_kernel's per-block published histograms (one row: kSelMaxB blocks at most)
constexpr int kSelMaxB = 32;
constexpr int kPub10 = 1 << kMidBits;            // words per block: its 10-bit histogram
constexpr int kPub9 = (1 << kLowBits) + 16;      // its 9-bit histogram, then its count above the 22-bit prefix

__host__ __device__ inline int64_t n_chunks(int64_t P) { return (P + kChunk - 1) / kChunk; }
__host__ __device__ inline int64_t n_subs(int64_t P) { return (P + kSub - 1) / kSub; }

__host__ __device__ inline WorkLayout layout(int64_t P) {
    const int64_t nc = n_chunks(P);
    WorkLayout w;
    w.hist = 0;
    w.state = w.hist + sizeof(uint32_t) * kHistWords;
    w.cnt = w.state + 64;
    w.bt = w.cnt + sizeof(int64_t) * kRec * (size_t)nc;           // cand_mark block totals (<= nc blocks)
    w.cval = (w.bt + sizeof(int64_t) * kRec * (size_t)nc + 255) / 256 * 256;
    w.cloc = w.cval + sizeof(float) * (size_t)nc * kCvLd;
    w.pub = (w.cloc + sizeof(uint16_t) * (size_t)nc * kClLd + 255) / 256 * 256;
    w.total = w.pub + sizeof(uint32_t) * (size_t)kSelMaxB * (kPub10 + kPub9);
    return w;
}

// A batch of rows: input row r at x + r*ld (x_hat likewise, may be null); its output message at
// out + r*out_ld (values) and + idx_off (int64 indices); its scratch at work + r*work_ld.
struct Rows {
    const float* x;
    const float* xh;
    int64_t ld;
    char* out;
    int64_t out_ld, idx_off;
    char* work;
    int64_t work_ld;
    int64_t P, k;
    int64_t bnd_off;      // int32 tile bounds at out + r*out_ld + bnd_off (< 0: not written)
    int32_t hint;         // floor_hint margin in 12-bit bins (< 0: sampled floor)
    int32_t fine;         // fine_floor: 1 = refine the sampled floor inside the window (sub-bins)
};

struct RowView {
    const float* x;
    const float* xh;
    uint32_t* hs;         // sampled top digits
    uint32_t* h12;        // candidates' top digits
    uint32_t* h12f;       // the same, of the fallback pass (keeps every key)
    uint32_t* h10;        // next 10 bits of the candidates in the threshold bin
    uint32_t* h9;         // last 9 bits
    uint32_t* hsf;        // fine sampled sub-bins of the window (fine_floor)
    SelState* st;
    int64_t* cnt;
    int64_t* bt;          // cand_mark block totals (keys > T, keys == T)
    float* cval;
    uint16_t* cloc;
    float* vals;
    int64_t* idx;
};

__device__ __forceinline__ RowView row_view(const Rows& R, int r) {
    const WorkLayout w = layout(R.P);
    char* wb = R.work + (int64_t)r * R.work_ld;
    RowView v;
    v.x = R.x + (int64_t)r * R.ld;
    v.xh = R.xh ? R.xh + (int64_t)r * R.ld : nullptr;
    v.hs = reinterpret_cast<uint32_t*>(wb + w.hist);
    v.h12 = v.hs + kTopBins;
    v.h12f = v.h12 + kTopBins;
    v.h10 = v.h12f + kTopBins;
    v.h9 = v.h10 + (1 << kMidBits);
    v.hsf = v.h9 + (1 << kLowBits);
    v.st = reinterpret_cast<SelState*>(wb + w.state);
    v.cnt = reinterpret_cast<int64_t*>(wb + w.cnt);
    v.bt = reinterpret_cast<int64_t*>(wb + w.bt);
    v.cval = reinterpret_cast<float*>(wb + w.cval);
    v.cloc = reinterpret_cast<uint16_t*>(wb + w.cloc);
    v.vals = reinterpret_cast<float*>(R.out + (int64_t)r * R.out_ld);
    v.idx = reinterpret_cast<int64_t*>(R.out + (int64_t)r * R.out_ld + R.idx_off);
    return v;
}

__device__ __forceinline__ RowView row_view(const Rows& R) { return row_view(R, blockIdx.y); }

__device__ __forceinline__ uint32_t key_of(float d) { return __float_as_uint(d) & 0x7fffffffu; }

__device__ __forceinline__ float diff_at(const float* x, const float* xh, int64_t i) {
    return xh ? __fsub_rn(x[i], xh[i]) : x[i];
}

typedef float f4 __attribute__((ext_vector_type(4)));

// 16-byte streaming access; NT = non-temporal hint (compile-time: a runtime choice measured 24 %
// slower whatever its value, the prefetching loops lose their schedule)
template <bool NT>
__device__ __forceinline__ f4 ld4(const f4* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st4(f4 v, f4* p) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// elements 4q .. 4q+3 of x - x_hat (16-byte non-temporal loads when the rows are aligned);
// returns how many of them are < P
__device__ __forceinline__ int load_quad(const float* x, const float* xh, int64_t q, int64_t P, bool vec,
                                         float (&d)[4]) {
    const int64_t i0 = 4 * q;
    if (vec && i0 + 4 <= P) {
        const f4 a = __builtin_nontemporal_load(reinterpret_cast<const f4*>(x) + q);
        if (xh) {
            const f4 b = __builtin_nontemporal_load(reinterpret_cast<const f4*>(xh) + q);
#pragma unroll
            for (int c = 0; c < 4; ++c) d[c] = __fsub_rn(a[c], b[c]);
        } else {
#pragma unroll
            for (int c = 0; c < 4; ++c) d[c] = a[c];
        }
        return 4;
    }
    int n = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int64_t i = i0 + c;
        d[c] = 0.0f;
        if (i < P) {
            d[c] = diff_at(x, xh, i);
            ++n;
        }
    }
    return n;
}

// set bits of a wave mask in the lanes below this one
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// inclusive scan of a per-lane count over the wave, in DPP lane moves (no LDS round trips: the
// ds_bpermute form of __shfl_up costs six dependent LDS latencies per scan): row_shr 1 / 2 / 4 / 8
// within each 16-lane row (zeros shifted in), then row_bcast:15 / row_bcast:31 carry the row
// totals into the rows above
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);   // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}

// the same over 64-bit counts: both halves moved by the same DPP pattern give the source lane's
// 64-bit value
template <int CTRL, int ROWS, bool BC>
__device__ __forceinline__ int64_t dpp64(int64_t v) {
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, ROWS, 0xf, BC);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)((uint64_t)v >> 32), CTRL, ROWS, 0xf, BC);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

__device__ __forceinline__ int64_t wave_incl_scan64(int64_t v) {
    v += dpp64<0x111, 0xf, true>(v);
    v += dpp64<0x112, 0xf, true>(v);
    v += dpp64<0x114, 0xf, true>(v);
    v += dpp64<0x118, 0xf, true>(v);
    v += dpp64<0x142, 0xa, false>(v);
    v += dpp64<0x143, 0xc, false>(v);
    return v;
}

__device__ __forceinline__ int64_t lane63(int64_t v) {
    const int lo = __builtin_amdgcn_readlane((int)(uint32_t)v, 63);
    const int hi = __builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), 63);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// The fine window's first top digit: kWinBins digits from one below the last call's floor digit (the
// floor moves by a fraction of a digit per round; a miss just leaves that round's floor a whole
// digit); -1 = no window (fine_floor off, or no call yet).  The sampling pass and the compaction
// read the same state, so they agree.
__device__ __forceinline__ int fine_window(const Rows& R, const RowView& v) {
    if (!R.fine || !v.st->hint_ok) return -1;
    const int d = (int)v.st->win_digit - 1;
    return d < 0 ? 0 : d > kTopBins - kWinBins ? kTopBins - kWinBins : d;
}

// ---- S: top-digit histogram over every S-th 1024-element piece, one wave per sampled piece;
// this block takes pieces (bx + i gx) * kWaves + wave into its LDS histogram h (zeroed here), and
// with a fine window w0 >= 0 the keys of digits [w0, w0 + kWinBins) also into the sub-bins hf
__device__ __forceinline__ void sample_into(const Rows& R, const RowView& v, int64_t S, int64_t bx, int64_t gx, uint32_t* h,
                                            uint32_t* hf = nullptr, int w0 = -1) {
    for (int i = threadIdx.x; i < kTopBins; i += kTPB) h[i] = 0;
    if (w0 >= 0)
        for (int i = threadIdx.x; i < kFineBins; i += kTPB) hf[i] = 0;
    __syncthreads();
    const bool vec = (((uintptr_t)v.x | (uintptr_t)v.xh) & 15) == 0;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t nsamp = (n_subs(R.P) + S - 1) / S;
    for (int64_t u = bx * kWaves + wave; u < nsamp; u += gx * kWaves) {
        const int64_t q0 = u * S * kSubQuads;
        float d[4][4];
        int n[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) n[j] = load_quad(v.x, v.xh, q0 + j * 64 + lane, R.P, vec, d[j]);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (c < n[j]) {
                    const uint32_t key = key_of(d[j][c]);
                    atomicAdd(&h[key >> kTopShift], 1u);
                    const uint32_t wd = (key >> kTopShift) - (uint32_t)w0;
                    if (w0 >= 0 && wd < (uint32_t)kWinBins)
                        atomicAdd(&hf[wd * kFineSub + ((key >> kFineShift) & (kFineSub - 1))], 1u);
                }
    }
    __syncthreads();
}

__global__ __launch_bounds__(kTPB) void sample_kernel(Rows R, int64_t S) {
    const RowView v = row_view(R);
    __shared__ uint32_t h[kTopBins];
    __shared__ uint32_t hf[kFineBins];
    const int w0 = fine_window(R, v);
    sample_into(R, v, S, blockIdx.x, gridDim.x, h, hf, w0);
    for (int i = threadIdx.x; i < kTopBins; i += kTPB)
        if (h[i]) atomicAdd(&v.hs[i], h[i]);
    if (w0 >= 0)
        for (int i = threadIdx.x; i < kFineBins; i += kTPB)
            if (hf[i]) atomicAdd(&v.hsf[i], hf[i]);
}

typedef __attribute__((address_space(1))) uint32_t g_u32;

__device__ __forceinline__ void st_sc1(uint32_t* p, uint32_t v) {
    __hip_atomic_store((g_u32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_sc1(const uint32_t* p) {
    return __hip_atomic_load((g_u32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr uint64_t kSpinTicks = 1ull << 28;    // ~2.7 s of the 100 MHz constant clock
// the bounded waits' deadline (mx_topk_set "spin_ticks": a test knob -- 0 makes every wait that has
// to wait at all expire, so the error path can be exercised on purpose)
__device__ uint64_t g_spin_ticks_dev = kSpinTicks;
// compaction trace (mx_topk_set "compact_trace" 1, diagnostic): per workgroup of the last one-row
// compaction launch, the constant clock at its start, after its floor is resolved, and at its end
constexpr int kTraceBlocks = 8192;
__device__ uint64_t g_ctrace[kTraceBlocks * 3];
__device__ int g_ctrace_on = 0;
__device__ __forceinline__ void ctrace(int slot) {
    const int b = blockIdx.x;
    if (g_ctrace_on && threadIdx.x == 0 && blockIdx.y == 0 && b < kTraceBlocks)
        g_ctrace[3 * b + slot] = (uint64_t)wall_clock64();
}

// block-uniform values the compiler cannot prove uniform (they come through LDS): into SGPRs
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ int64_t uni(int64_t x) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)x >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// one thread: poll a counter (`sc1` loads) until `target`; false when the bounded wait expired
__device__ __forceinline__ bool wait_count(const uint32_t* ctr, uint32_t target) {
    const uint64_t t0 = wall_clock64();
    while (ld_sc1(ctr) < target) {
        __builtin_amdgcn_s_sleep(2);
        if ((uint64_t)wall_clock64() - t0 > g_spin_ticks_dev) return false;
    }
    return true;
}

// A finished histogram's bins, kPer per thread, in registers (the boundary search walks registers,
// not dependent global loads).  With fewer bins than threads, thread t holds bin NBINS-1-t (threads
// past NBINS hold empty bins).
template <int NBINS, int TPB = kTPB>
struct Bins {
    static constexpr int kPer = NBINS >= TPB ? NBINS / TPB : 1;
    uint32_t c[kPer];                                    // bins NBINS-1-(t*kPer+j), top first
};

// this thread's kPer bins of a finished histogram (vector loads into registers)
template <int NBINS, int TPB = kTPB>
__device__ __forceinline__ void load_bins(const uint32_t* __restrict__ hist, Bins<NBINS, TPB>& b) {
    const int t = threadIdx.x;
    constexpr int kPer = Bins<NBINS, TPB>::kPer;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        if constexpr (NBINS >= TPB) b.c[j] = hist[NBINS - 1 - (t * kPer + j)];   // unpredicated: vector loads
        else b.c[j] = t < NBINS ? hist[NBINS - 1 - t] : 0u;
    }
}

// Block-wide, over bins already in registers: the bin holding the need-th largest key, scanning
// bins from the top; *rem = rank of that key inside its bin.  bin 0 / rem = need - total when the
// histogram holds fewer than `need` keys.  Read-only (every block of a kernel resolves the same
// answer), so no separate one-block select launch sits between the passes.  Wave scans in DPP,
// one barrier to combine the waves, one to publish.
template <int NBINS, int TPB = kTPB>
__device__ void scan_bins(const Bins<NBINS, TPB>& bs, int64_t need, int* bin, int64_t* rem, int64_t* total) {
    constexpr int kPer = Bins<NBINS, TPB>::kPer;
    constexpr int kW = TPB / 64;
    __shared__ int64_t wsum[kW];
    __shared__ int s_bin;
    __shared__ int64_t s_rem;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    int64_t mine = 0;
#pragma unroll
    for (int j = 0; j < kPer; ++j) mine += bs.c[j];
    int64_t incl = wave_incl_scan64(mine);               // inclusive scan over the wave (DPP)
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    int64_t base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kW; ++w) {
        base += w < wave ? wsum[w] : 0;
        tot += wsum[w];
    }
    incl += base;
    const int64_t before = incl - mine;
    if (tot >= need && before < need && incl >= need) {  // exactly one thread holds the boundary
        int64_t acc = before;
        int b = -1;
        int64_t r = 0;
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            if (b < 0 && acc + bs.c[j] >= need) {
                b = NBINS - 1 - (t * kPer + j);
                r = need - acc;
            }
            acc += bs.c[j];
        }
        s_bin = b;
        s_rem = r;
    }
    __syncthreads();
    *total = tot;
    if (tot < need || need <= 0) {
        *bin = 0;
        *rem = need <= 0 ? need : need - tot;
    } else {
        *bin = s_bin;
        *rem = s_rem;
    }
    __syncthreads();                                     // the shared answer may be reused
}

template <int NBINS>
__device__ void find_bin(const uint32_t* __restrict__ hist, int64_t need, int* bin, int64_t* rem,
                         int64_t* total) {
    Bins<NBINS> bs;
    load_bins<NBINS>(hist, bs);
    scan_bins<NBINS>(bs, need, bin, rem, total);
}

// Threshold resolved so far from the finished candidate histograms: `stages` of 12 / 10 / 9 bits.
struct Resolved {
    uint32_t prefix, mask;
    int64_t need;                                        // keys still to take at/below prefix
};

// Every histogram a stage will need is loaded up front -- the 12-bit one of both the first and the
// fallback compaction (which one holds the candidates depends on the candidate count, itself a
// load) -- so the stages cost one memory round trip, not one each; the scans follow in registers.
__device__ Resolved resolve(const RowView& v, int64_t k, int stages) {
    Bins<kTopBins> a12, f12;
    Bins<1 << kMidBits> b10;
    Bins<1 << kLowBits> b9;
    const unsigned long long cand_n = v.st->cand_n;
    load_bins<kTopBins>(v.h12, a12);
    load_bins<kTopBins>(v.h12f, f12);
    if (stages >= 2) load_bins<1 << kMidBits>(v.h10, b10);
    if (stages >= 3) load_bins<1 << kLowBits>(v.h9, b9);
    const bool fb = cand_n < (unsigned long long)k;      // the fallback pass ran for this row
    if (fb) {
#pragma unroll
        for (int j = 0; j < Bins<kTopBins>::kPer; ++j) a12.c[j] = f12.c[j];
    }
    Resolved z{0u, 0u, k};
    int b;
    int64_t rem, tot;
    scan_bins<kTopBins>(a12, z.need, &b, &rem, &tot);
    z.prefix = (uint32_t)b << kTopShift;
    z.mask = 0xfffu << kTopShift;
    z.need = rem;
    if (stages >= 2) {
        scan_bins<1 << kMidBits>(b10, z.need, &b, &rem, &tot);
        z.prefix |= (uint32_t)b << kMidShift;
        z.mask |= ((1u << kMidBits) - 1) << kMidShift;
        z.need = rem;
    }
    if (stages >= 3) {
        scan_bins<1 << kLowBits>(b9, z.need, &b, &rem, &tot);
        z.prefix |= (uint32_t)b;
        z.mask = 0xffffffffu;
        z.need = rem;
    }
    return z;
}

// ---- B: persistent blocks, one 4096-element chunk per block iteration; keys with top digit >=
// b_lo -> (value, local index) in the chunk's region, in index order (wave w, step j, lane l
// holds elements 4(c*1024 + 256w + 64j + l) .. +3), and their top digits into the 12-bit
// candidate histogram.  b_lo comes from the sampled histogram (every block resolves it): S = 1 the
// exact digit of the k-th largest key; S > 1 k scaled to the sample with a 25 % + 4 sigma margin.
// The next chunk's x / x_hat loads are issued before the current chunk is ranked and written.
// cnt[kRec c + 0..3] = {0, candidates > T, candidates == T, candidates}, + 4 words of padding.
// fallback = 1: runs only if fewer than k candidates were kept, then keeps every key.
// BAL: a wave's output offsets from ballots + mbcnt (one row: 117.5 -> 115.5 us per round) or from
// shuffle scans (several rows: 650 vs 655 us with ballots, whose 64-bit masks spill SGPRs)
// LOOP: candidate stores in a loop over the lane's kept elements (mx_topk_set "compact_store" 1)
// PF2: two whole chunks in flight per wave instead of one (a second register buffer, +32 VGPRs)
// The compaction's candidate floor (a 12-bit top digit; block-uniform, every thread calls it).
// S >= 1: from the sampled histogram -- S = 1 the exact digit of the k-th largest key, S > 1 k scaled
// to the sample with a 25 % + 4 sigma margin.  S = 0 (floor_hint): the previous call's exact k-th
// key's digit lowered by the row's adaptive margin (no sampling launch); the first call on a scratch
// has no hint and keeps every key.  A floor too high is caught by the candidate count (fallback).
// Returned as a KEY floor (keys >= it are kept): a digit's first key, or with fine_floor, when the
// floor's digit falls in the window, that digit's sub-bin holding the wanted sampled rank.
__device__ uint32_t floor_key(const Rows& R, const RowView& v, int64_t S, double frac) {
    if (S == 0) {
        if (!v.st->hint_ok) return 0u;
        const uint32_t m = v.st->margin ? v.st->margin : (uint32_t)(R.hint > 0 ? R.hint : 1);
        const uint32_t d = v.st->hint_digit;
        return (d > m ? d - m : 0u) << kTopShift;
    }
    int64_t want = R.k;
    if (S > 1) {
        const double e = (double)R.k * frac;
        want = (int64_t)ceil(1.25 * e + 4.0 * sqrt(e) + 16.0);
    }
    int b;
    int64_t rem, tot;
    find_bin<kTopBins>(v.hs, want, &b, &rem, &tot);
    if (tot < want) return 0u;                              // too few sampled keys: keep everything
    const int w0 = fine_window(R, v);                       // block-uniform
    if (w0 >= 0 && b >= w0 && b < w0 + kWinBins) {
        int sb;
        int64_t rem2, tot2;
        find_bin<kFineSub>(v.hsf + (b - w0) * kFineSub, rem, &sb, &rem2, &tot2);
        if (tot2 >= rem) return ((uint32_t)b << kTopShift) | ((uint32_t)sb << kFineShift);
    }
    return (uint32_t)b << kTopShift;
}

// The same floor with its inputs loaded ahead (compact_run): the sampled histogram and every window
// sub-bin are loaded BEFORE the first chunk's x / x_hat loads are issued.  Loads return in issue
// order, so histogram loads issued after the chunk's (the old order) waited for its HBM latency, and
// the window's sub-bins were a second dependent round trip after that: the block's floor was ready
// ~4 us after its start, ~2 us after its first chunk (profiles/r05h_compact_trace.log).  Thread
// (wave w, lane l) holds window slot w's sub-bin 63 - l (kTPB / 64 == kWinBins waves), so the
// sub-bin is found by one wave scan instead of a second block-wide load and scan.
static_assert(kTPB / 64 == kWinBins && kFineSub == 64, "one wave per window slot, one lane per sub-bin");
#ifndef MX_FLOOR_EARLY
#define MX_FLOOR_EARLY 1      // 0: the round-4 order (floor resolved after the first chunk's loads), for A/B builds
#endif
struct FloorIn {
    Bins<kTopBins> hs;
    uint32_t sub;
};

// (unconditional -- a branch here would join with register moves that wait for the loads; with the
// floor hint (S = 0) the loaded bins are simply unused)
__device__ __forceinline__ void floor_load(const RowView& v, FloorIn& fi) {
    load_bins<kTopBins>(v.hs, fi.hs);
    fi.sub = v.hsf[(threadIdx.x >> 6) * kFineSub + kFineSub - 1 - (threadIdx.x & 63)];
}

__device__ uint32_t floor_key_loaded(const Rows& R, const RowView& v, int64_t S, double frac, const FloorIn& fi) {
    if (S == 0) return floor_key(R, v, S, frac);
    const double e = (double)R.k * frac;
    const int64_t want = S > 1 ? (int64_t)ceil(1.25 * e + 4.0 * sqrt(e) + 16.0) : R.k;
    int b;
    int64_t rem, tot;
    scan_bins<kTopBins>(fi.hs, want, &b, &rem, &tot);
    if (tot < want) return 0u;                              // too few sampled keys: keep everything
    const int w0 = fine_window(R, v);                       // block-uniform
    if (w0 >= 0 && b >= w0 && b < w0 + kWinBins) {
        __shared__ int s_sb;
        if (threadIdx.x == 0) s_sb = -1;
        __syncthreads();
        if ((int)(threadIdx.x >> 6) == b - w0) {             // wave-uniform
            const int64_t incl = wave_incl_scan64((int64_t)fi.sub);
            if (incl - (int64_t)fi.sub < rem && incl >= rem) s_sb = kFineSub - 1 - (int)(threadIdx.x & 63);
        }
        __syncthreads();
        const int sb = s_sb;
        if (sb >= 0) return ((uint32_t)b << kTopShift) | ((uint32_t)sb << kFineShift);
    }
    return (uint32_t)b << kTopShift;
}

// After the threshold pass resolved T (one thread per row): the next call's floor hint, the margin
// adapted (a fallback widens it by 4 bins, a candidate set above 4 k narrows it by one), counts.
// cn = this call's candidate count (keys kept by the first compaction).
__device__ void record_round(const Rows& R, SelState* st, uint32_t T, unsigned long long cn) {
    const bool fb = cn < (unsigned long long)R.k;
    uint32_t m = st->margin ? st->margin : (uint32_t)(R.hint > 0 ? R.hint : 1);
    if (fb) m = m + 4 < 255 ? m + 4 : 255;
    else if (cn > 4ull * (unsigned long long)R.k && m > 1) m -= 1;
    st->margin = m;
    st->hint_digit = T >> kTopShift;
    st->hint_ok = 1;
    st->n_calls += 1;
    st->n_fallbacks += fb ? 1u : 0u;
    st->last_cand = (uint32_t)(cn < 0xffffffffull ? cn : 0xffffffffull);
    st->win_digit = st->b0;               // this call's floor digit (written by its compaction)
}

template <bool BAL, bool LOOP, bool PF2 = false>
__device__ void compact_run(const Rows& R, const RowView& v, int64_t S, double frac, int fallback, int64_t bx,
                            int64_t gx) {
    __shared__ uint32_t wtot[2][kWaves];
    __shared__ uint32_t h[kTopBins];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t nc = n_chunks(R.P);
    const bool vec = (((uintptr_t)v.x | (uintptr_t)v.xh) & 15) == 0;
    const f4* x4 = reinterpret_cast<const f4*>(v.x);
    const f4* h4 = reinterpret_cast<const f4*>(v.xh);
    auto whole = [&](int64_t c) { return vec && (c + 1) * kChunk <= R.P; };
    f4 ax[4], ah[4];                               // raw loads of the next full chunk
    f4 px[4], ph[4];                               // PF2: and of the one after
    auto issue_to = [&](f4 (&X)[4], f4 (&H)[4], int64_t c) {
        const int64_t q0 = c * (kChunk / 4) + wave * kSubQuads + lane;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            X[j] = __builtin_nontemporal_load(x4 + q0 + j * 64);
            H[j] = h4 ? __builtin_nontemporal_load(h4 + q0 + j * 64) : f4{0.0f, 0.0f, 0.0f, 0.0f};
        }
    };
    auto issue = [&](int64_t c) { issue_to(ax, ah, c); };
    if (!fallback) ctrace(0);
    FloorIn fi;
    if (MX_FLOOR_EARLY && !fallback) floor_load(v, fi);   // ahead of the chunk loads (floor_key_loaded)
    int64_t c = bx;
    if (c < nc && whole(c)) issue(c);              // the first chunk flies while b_lo is resolved
    if constexpr (PF2) {
        if (c + gx < nc && whole(c + gx)) issue_to(px, ph, c + gx);
    }

    uint32_t b_lo = 0, fkey = 0;                   // floor: keys >= fkey (digit b_lo) are kept
    if (!fallback) {
        fkey = MX_FLOOR_EARLY ? floor_key_loaded(R, v, S, frac, fi) : floor_key(R, v, S, frac);
        b_lo = fkey >> kTopShift;
        if (bx == 0 && threadIdx.x == 0) {
            v.st->b0 = b_lo;
            v.st->bar = 0;                                  // the selection's row barriers start here
        }
    }
    if (!fallback) ctrace(1);
    // only digits >= b_lo are ever counted: zero and flush just those bins (b_lo is near the top)
    const int h0 = (int)(b_lo & ~(uint32_t)(kTPB - 1));
    for (int i = h0 + threadIdx.x; i < kTopBins; i += kTPB) h[i] = 0;
    uint32_t kept = 0;                             // this block's candidates (thread 0)
    __syncthreads();                               // h zeroed
    // whole chunks (prefetched one ahead in registers) and the partial / unaligned ones run in two
    // separate loops over the same per-chunk step: one loop holding both load paths made the
    // waitcnt pass wait for the next chunk's loads in the middle of every iteration
    const int64_t nfull = vec ? R.P / kChunk : 0;  // chunks whole(c) holds for: [0, nfull)
    int par = 0;
    auto step = [&](int64_t c, float (&d)[4][4], const int (&n)[4]) {
        uint32_t keep = 0;                           // bit 4j + e: element e of step j is kept
        uint32_t ex[4], wt[4];                       // kept in lower lanes / in the wave, per step
        uint32_t tot = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            ex[j] = 0;
            wt[j] = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t key = key_of(d[j][e]);
                const uint32_t dg = key >> kTopShift;
                const bool f = e < n[j] && key >= fkey;
                keep |= (f ? 1u : 0u) << (4 * j + e);
                if constexpr (BAL) {                    // ballots + mbcnt instead of a shuffle scan
                    const uint64_t b = __ballot(f);
                    ex[j] += lanes_below(b);
                    wt[j] += (uint32_t)__popcll(b);
                } else {
                    ex[j] += f;                         // this lane's count; scanned below
                }
                if (f) atomicAdd(&h[dg], 1u);
            }
            if constexpr (!BAL) {
                const uint32_t incl = wave_incl_scan(ex[j]);
                wt[j] = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
                ex[j] = incl - ex[j];
            }
            tot += wt[j];
        }
        if (lane == 0) wtot[par][wave] = tot;
        __syncthreads();                             // double-buffered by parity: one barrier
        uint32_t pos = 0, all = 0;
        for (int w = 0; w < kWaves; ++w) {
            pos += w < wave ? wtot[par][w] : 0;
            all += wtot[par][w];
        }
        float* cv = v.cval + c * kCvLd;
        uint16_t* cl = v.cloc + c * kClLd;
        if constexpr (LOOP) {
            // one store pair per kept element of the lane, the wave looping as often as its
            // fullest lane keeps (1-2 at 1 % density) instead of 16 masked store pairs
            uint32_t base[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                base[j] = pos + ex[j];
                pos += wt[j];
            }
            for (uint32_t rem = keep; rem; rem &= rem - 1) {
                const int b = __builtin_ctz(rem);
                const int j = b >> 2;
                float val = d[0][0];
                uint32_t bj = base[0];
#pragma unroll
                for (int t = 1; t < 16; ++t) val = b == t ? d[t >> 2][t & 3] : val;
#pragma unroll
                for (int t = 1; t < 4; ++t) bj = j == t ? base[t] : bj;
                const uint32_t p = bj + __popc(keep & ((1u << b) - 1) & (0xfu << (4 * j)));
                cv[p] = val;
                cl[p] = (uint16_t)(kSub * wave + 4 * (64 * j + lane) + (b & 3));
            }
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                uint32_t p = pos + ex[j];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if ((keep >> (4 * j + e)) & 1u) {
                        cv[p] = d[j][e];
                        cl[p] = (uint16_t)(kSub * wave + 4 * (64 * j + lane) + e);
                        ++p;
                    }
                }
                pos += wt[j];
            }
        }
        if (wave == 0 && lane < kRec) v.cnt[kRec * c + lane] = lane == 3 ? all : 0;   // the whole record
        if (threadIdx.x == 0) kept += all;
        par ^= 1;
    };
    if constexpr (PF2) {
        const int n[4] = {4, 4, 4, 4};
        for (; c < nfull; c += 2 * gx) {
            {
                float d[4][4];
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int e = 0; e < 4; ++e) d[j][e] = h4 ? __fsub_rn(ax[j][e], ah[j][e]) : ax[j][e];
                if (c + 2 * gx < nfull) issue_to(ax, ah, c + 2 * gx);
                step(c, d, n);
            }
            if (c + gx >= nfull) {                 // the stride sequence's next chunk is past the whole ones
                c += gx;
                break;
            }
            {
                float d[4][4];
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int e = 0; e < 4; ++e) d[j][e] = h4 ? __fsub_rn(px[j][e], ph[j][e]) : px[j][e];
                if (c + 3 * gx < nfull) issue_to(px, ph, c + 3 * gx);
                step(c + gx, d, n);
            }
        }
    } else {
        for (; c < nfull; c += gx) {
            float d[4][4];
            const int n[4] = {4, 4, 4, 4};
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) d[j][e] = h4 ? __fsub_rn(ax[j][e], ah[j][e]) : ax[j][e];
            if (c + gx < nfull) issue(c + gx);
            step(c, d, n);
        }
    }
    for (; c < nc; c += gx) {
        float d[4][4];
        int n[4];
        const int64_t q0 = c * (kChunk / 4) + wave * kSubQuads;
#pragma unroll
        for (int j = 0; j < 4; ++j) n[j] = load_quad(v.x, v.xh, q0 + j * 64 + lane, R.P, vec, d[j]);
        step(c, d, n);
    }
    __syncthreads();
    uint32_t* out = fallback ? v.h12f : v.h12;
    for (int i = h0 + threadIdx.x; i < kTopBins; i += kTPB)
        if (h[i]) atomicAdd(&out[i], h[i]);
    if (!fallback && threadIdx.x == 0 && kept) atomicAdd(&v.st->cand_n, (unsigned long long)kept);
    if (!fallback) ctrace(2);
}

template <bool BAL, bool LOOP, bool PF2 = false>
__global__ __launch_bounds__(kTPB) void compact_kernel(Rows R, int64_t S, double frac) {
    const RowView v = row_view(R);
    compact_run<BAL, LOOP, PF2>(R, v, S, frac, 0, blockIdx.x, gridDim.x);
}

// The same pass with wave-owned chunks (mx_topk_set "compact_wave" 1): every wave streams whole
// chunks of its own -- gw, gw + GW, ... (gw = the wave's index over the grid) -- in four
// 1024-element sub-steps, each the 4 quads per lane of one wave step above, the next sub-step's
// loads in flight while one is ranked.  A chunk's candidates are placed from the wave's own
// running count, so the waves of a block never wait for each other (no barrier per chunk); they
// share only the LDS histogram, flushed once at the end.  Output identical to compact_kernel's
// (same regions, same index order, same counts and histograms).
template <bool BAL>
__global__ __launch_bounds__(kTPB) void compact_wave_kernel(Rows R, int64_t S, double frac) {
    const RowView v = row_view(R);
    __shared__ uint32_t h[kTopBins];
    __shared__ uint32_t wk[kWaves];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t nc = n_chunks(R.P);
    const int64_t gw = (int64_t)blockIdx.x * kWaves + wave, GW = (int64_t)gridDim.x * kWaves;
    const bool vec = (((uintptr_t)v.x | (uintptr_t)v.xh) & 15) == 0;
    const f4* x4 = reinterpret_cast<const f4*>(v.x);
    const f4* h4 = reinterpret_cast<const f4*>(v.xh);
    const int64_t nfull = vec ? R.P / kChunk : 0;  // whole, aligned chunks: [0, nfull)
    auto chunk_of = [&](int64_t s) { return gw + (s >> 2) * GW; };
    f4 ax[4], ah[4];
    auto issue = [&](int64_t s) {
        const int64_t q0 = chunk_of(s) * (kChunk / 4) + (s & 3) * kSubQuads + lane;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            ax[j] = __builtin_nontemporal_load(x4 + q0 + j * 64);
            ah[j] = h4 ? __builtin_nontemporal_load(h4 + q0 + j * 64) : f4{0.0f, 0.0f, 0.0f, 0.0f};
        }
    };
    int64_t s = 0;
    if (chunk_of(0) < nfull) issue(0);             // in flight while b_lo is resolved
    uint32_t b_lo = 0, fkey = 0;
    {
        fkey = floor_key(R, v, S, frac);
        b_lo = fkey >> kTopShift;
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            v.st->b0 = b_lo;
            v.st->bar = 0;
        }
    }
    const int h0 = (int)(b_lo & ~(uint32_t)(kTPB - 1));
    for (int i = h0 + threadIdx.x; i < kTopBins; i += kTPB) h[i] = 0;
    __syncthreads();
    uint32_t run = 0, kept = 0;                    // the current chunk's candidates so far / the wave's
    auto sub = [&](int64_t s, float (&d)[4][4], const int (&n)[4]) {
        const int64_t c = chunk_of(s);
        const int u = (int)(s & 3);
        uint32_t keep = 0, ex[4], wt[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            ex[j] = 0;
            wt[j] = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t key = key_of(d[j][e]);
                const uint32_t dg = key >> kTopShift;
                const bool f = e < n[j] && key >= fkey;
                keep |= (f ? 1u : 0u) << (4 * j + e);
                if constexpr (BAL) {
                    const uint64_t b = __ballot(f);
                    ex[j] += lanes_below(b);
                    wt[j] += (uint32_t)__popcll(b);
                } else {
                    ex[j] += f;
                }
                if (f) atomicAdd(&h[dg], 1u);
            }
            if constexpr (!BAL) {
                const uint32_t incl = wave_incl_scan(ex[j]);
                wt[j] = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
                ex[j] = incl - ex[j];
            }
        }
        float* cv = v.cval + c * kCvLd;
        uint16_t* cl = v.cloc + c * kClLd;
        uint32_t base[4], pos = run;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            base[j] = pos + ex[j];
            pos += wt[j];
        }
        for (uint32_t rem = keep; rem; rem &= rem - 1) {
            const int b = __builtin_ctz(rem);
            const int j = b >> 2;
            float val = d[0][0];
            uint32_t bj = base[0];
#pragma unroll
            for (int t = 1; t < 16; ++t) val = b == t ? d[t >> 2][t & 3] : val;
#pragma unroll
            for (int t = 1; t < 4; ++t) bj = j == t ? base[t] : bj;
            const uint32_t p = bj + __popc(keep & ((1u << b) - 1) & (0xfu << (4 * j)));
            cv[p] = val;
            cl[p] = (uint16_t)(kSub * u + 4 * (64 * j + lane) + (b & 3));
        }
        run = pos;
        if (u == 3) {                              // the chunk is complete: its whole record
            if (lane < kRec) v.cnt[kRec * c + lane] = lane == 3 ? run : 0;
            kept += run;
            run = 0;
        }
    };
    for (; chunk_of(s) < nfull; ++s) {
        float d[4][4];
        const int n[4] = {4, 4, 4, 4};
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) d[j][e] = h4 ? __fsub_rn(ax[j][e], ah[j][e]) : ax[j][e];
        if (chunk_of(s + 1) < nfull) issue(s + 1);
        sub(s, d, n);
    }
    for (; chunk_of(s) < nc; ++s) {                // partial / unaligned chunks
        float d[4][4];
        int n[4];
        const int64_t q0 = chunk_of(s) * (kChunk / 4) + (s & 3) * kSubQuads;
#pragma unroll
        for (int j = 0; j < 4; ++j) n[j] = load_quad(v.x, v.xh, q0 + j * 64 + lane, R.P, vec, d[j]);
        sub(s, d, n);
    }
    if (lane == 0) wk[wave] = kept;
    __syncthreads();
    for (int i = h0 + threadIdx.x; i < kTopBins; i += kTPB)
        if (h[i]) atomicAdd(&v.h12[i], h[i]);
    if (threadIdx.x == 0) {
        uint32_t all = 0;
        for (int w = 0; w < kWaves; ++w) all += wk[w];
        if (all) atomicAdd(&v.st->cand_n, (unsigned long long)all);
    }
}

// Every block of this row's grid has arrived (rare path only: the fallback compaction inside the
// first candidate pass).  Producers: every wave's stores drained and released at agent scope, then
// one arrival per block on the row's counter; the poller's agent-scope acquire then covers the
// workgroup behind the barrier.  A grid barrier needs every block of the row co-resident: the host
// caps this pass's grid (all rows together) at 7/8 of what the chip holds of this kernel at once
// (occupancy query x CUs; the margin leaves room for e.g. RCCL's kernels beside it, N > 1), and
// the wait itself is BOUNDED: past kSpinTicks (~2.7 s) the row's sticky `err` word is set and the
// block goes on (the row's output is then undefined, never a hang; mx_topk_check reports it).
__device__ void row_grid_barrier(SelState* st, unsigned blocks) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(&st->bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!wait_count(&st->bar, blocks)) st_sc1(&st->err, 1u);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
}

// counts and first candidates of two chunk regions, loaded one step ahead by the candidate passes
struct RegionPair {
    int64_t n1, n2;
    float a1, a2;
};

// candidate histogram of the next digit (10 bits at 9, or 9 bits at 0) among candidates matching
// the prefix resolved so far; one wave per chunk region; LDS histogram flushed once per block
// The first candidate pass (BITS = 10) also stands in for the fallback compaction: with a
// sampled floor (S > 1) a row whose compaction kept fewer than k keys is compacted again here, by
// this pass's own blocks, keeping every key (into the fallback histogram), and the row's blocks
// meet at a grid barrier before histogramming -- a rare path, so the common one pays no launch.
template <int BITS, bool BAL, bool LOOP>
__global__ __launch_bounds__(kTPB) void cand_hist(Rows R, int64_t S, double frac) {
    const RowView v = row_view(R);
    if constexpr (BITS == kMidBits) {
        if (S != 1 && v.st->cand_n < (unsigned long long)R.k) {    // block-uniform (sampled or hinted floor)
            compact_run<BAL, LOOP>(R, v, S, frac, 1, blockIdx.x, gridDim.x);
            row_grid_barrier(v.st, gridDim.x);
        }
    }
    constexpr int NB = 1 << BITS;
    constexpr int stages = BITS == kMidBits ? 1 : 2;
    constexpr int shift = BITS == kMidBits ? kMidShift : 0;
    __shared__ uint32_t h[NB];
    const int64_t nchunks = n_chunks(R.P);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // two chunk regions per step, their counts and first 64 candidates loaded together (the
    // region is allocated whatever the count, lanes past it are ignored): one memory round trip
    // instead of a count -> candidates chain per region -- this pass reads them cold.  The first
    // step's loads fly while the histograms are resolved, each later step's during the one before.
    const int64_t stride = (int64_t)gridDim.x * kWaves;
    auto load = [&](int64_t c) {
        RegionPair q{0, 0, 0.0f, 0.0f};
        if (c < nchunks) {
            q.n1 = v.cnt[kRec * c + 3];
            q.a1 = v.cval[c * kCvLd + lane];
        }
        if (c + stride < nchunks) {
            q.n2 = v.cnt[kRec * (c + stride) + 3];
            q.a2 = v.cval[(c + stride) * kCvLd + lane];
        }
        return q;
    };
    int64_t c = (int64_t)blockIdx.x * kWaves + wave;
    RegionPair cur = load(c);
    const Resolved z = resolve(v, R.k, stages);
    for (int i = threadIdx.x; i < NB; i += kTPB) h[i] = 0;
    __syncthreads();
    auto add = [&](float d) {
        const uint32_t key = key_of(d);
        if ((key & z.mask) == z.prefix) atomicAdd(&h[(key >> shift) & (NB - 1)], 1u);
    };
    for (; c < nchunks; c += 2 * stride) {
        const RegionPair nx = load(c + 2 * stride);
        const int64_t c2 = c + stride;
        if (lane < cur.n1) add(cur.a1);
        for (int64_t i = 64 + lane; i < cur.n1; i += 64) add(v.cval[c * kCvLd + i]);
        if (lane < cur.n2) add(cur.a2);
        for (int64_t i = 64 + lane; i < cur.n2; i += 64) add(v.cval[c2 * kCvLd + i]);
        cur = nx;
    }
    __syncthreads();
    uint32_t* out = BITS == kMidBits ? v.h10 : v.h9;
    for (int i = threadIdx.x; i < NB; i += kTPB)
        if (h[i]) atomicAdd(&out[i], h[i]);
}

// the exact threshold key T and how many of its ties to take; per chunk region (one wave each)
// the counts of candidates > T and == T, written without atomics
// Block j owns the contiguous chunks [j*G, (j+1)*G) and also writes its totals to bt[2j], bt[2j+1],
// so write_cand can place any chunk's output from <= gridDim.x block totals plus < G chunk counts
// (no separate scan launch).
__global__ __launch_bounds__(kTPB) void cand_mark(Rows R, int64_t G) {
    const RowView v = row_view(R);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t nchunks = n_chunks(R.P);
    const int64_t c0 = (int64_t)blockIdx.x * G, c1 = c0 + G < nchunks ? c0 + G : nchunks;
    auto load = [&](int64_t c) {                 // two regions per step (as cand_hist), one step ahead
        RegionPair q{0, 0, 0.0f, 0.0f};
        if (c < c1) {
            q.n1 = v.cnt[kRec * c + 3];
            q.a1 = v.cval[c * kCvLd + lane];
        }
        if (c + kWaves < c1) {
            q.n2 = v.cnt[kRec * (c + kWaves) + 3];
            q.a2 = v.cval[(c + kWaves) * kCvLd + lane];
        }
        return q;
    };
    RegionPair cur = load(c0 + wave);            // in flight while the three histograms are resolved
    const Resolved z = resolve(v, R.k, 3);
    const uint32_t T = z.prefix;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        v.st->T = T;
        v.st->need = z.need;
        record_round(R, v.st, T, v.st->cand_n);
    }
    __shared__ uint32_t sg[kWaves], se[kWaves];
    uint32_t wg = 0, we = 0;
    auto count = [&](int64_t c, int64_t nc, float a) {     // a = candidate `lane` (speculative)
        uint32_t g = 0, e = 0;                   // wave-uniform: ballot counts per 64 candidates
        {
            const bool in = lane < nc;
            const uint32_t key = key_of(a);
            g += (uint32_t)__popcll(__ballot(in && key > T));
            e += (uint32_t)__popcll(__ballot(in && key == T));
        }
        for (int64_t i0 = 64; i0 < nc; i0 += 64) {
            const bool in = i0 + lane < nc;
            const uint32_t key = in ? key_of(v.cval[c * kCvLd + i0 + lane]) : 0u;
            g += (uint32_t)__popcll(__ballot(in && key > T));
            e += (uint32_t)__popcll(__ballot(in && key == T));
        }
        wg += g;
        we += e;
        if (lane < kRec) v.cnt[kRec * c + lane] = lane == 1 ? g : lane == 2 ? e : lane == 3 ? nc : 0;
    };
    for (int64_t c = c0 + wave; c < c1; c += 2 * kWaves) {
        const RegionPair nx = load(c + 2 * kWaves);
        count(c, cur.n1, cur.a1);
        if (c + kWaves < c1) count(c + kWaves, cur.n2, cur.a2);
        cur = nx;
    }
    if (lane == 0) {
        sg[wave] = wg;
        se[wave] = we;
    }
    __syncthreads();
    if (threadIdx.x < kRec) {                      // the whole 64-B record
        int64_t bg = 0, be = 0;
        for (int w = 0; w < kWaves; ++w) {
            bg += sg[w];
            be += se[w];
        }
        v.bt[kRec * blockIdx.x + threadIdx.x] = threadIdx.x == 0 ? bg : threadIdx.x == 1 ? be : 0;
    }
}

__device__ __forceinline__ int64_t wave_sum64(int64_t v) { return lane63(wave_incl_scan64(v)); }

// ---- C: one wave per chunk region: the candidates are already in index order, so a wave scan
// of the tie flags ranks the ties and a wave scan of the selection flags places the output.
// The block's chunks start at c_first; keys > T and ties before it = the cand_mark block totals of
// the blocks wholly before it (bt) + the chunk counts of its own cand_mark block before c_first,
// summed by the whole block; each wave then adds the (< kWaves) chunks of this block before its own.
__global__ __launch_bounds__(kTPB) void write_cand(Rows R, int64_t G) {
    const RowView v = row_view(R);
    const uint32_t T = v.st->T;
    const int64_t need_eq = v.st->need;
    // nothing reads the histograms or the candidate total any more: re-zero them for the next call
    for (int64_t i = (int64_t)blockIdx.x * kTPB + threadIdx.x; i < kHistWords; i += (int64_t)gridDim.x * kTPB)
        v.hs[i] = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        v.st->cand_n = 0;
        v.st->bar = 0;
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t c_first = (int64_t)blockIdx.x * kWaves;
    const int64_t c = c_first + wave;
    const int64_t nchunks = n_chunks(R.P);
    const bool live = c < nchunks;                 // this wave's region: count + first 64 candidates
    const int64_t nc = live ? v.cnt[kRec * c + 3] : 0;  // loaded up front (speculatively), in flight
    const float a0 = live ? v.cval[c * kCvLd + lane] : 0.0f;          // with the prefix loads
    const uint32_t l0 = live ? v.cloc[c * kClLd + lane] : 0u;
    const int64_t J = c_first / G, nitems = J + (c_first - J * G);
    int64_t g = 0, e = 0;
    for (int64_t i = threadIdx.x; i < nitems; i += kTPB) {
        if (i < J) {
            g += v.bt[kRec * i];
            e += v.bt[kRec * i + 1];
        } else {
            const int64_t cc = J * G + (i - J);
            g += v.cnt[kRec * cc + 1];
            e += v.cnt[kRec * cc + 2];
        }
    }
    g = wave_sum64(g);
    e = wave_sum64(e);
    __shared__ int64_t rg[kWaves], re[kWaves];
    if (lane == 0) {
        rg[wave] = g;
        re[wave] = e;
    }
    __syncthreads();
    if (!live) return;
    int64_t gt = 0, eq = 0;
    for (int w = 0; w < kWaves; ++w) {
        gt += rg[w];
        eq += re[w];
    }
    for (int64_t cc = c_first; cc < c; ++cc) {
        gt += v.cnt[kRec * cc + 1];
        eq += v.cnt[kRec * cc + 2];
    }
    int64_t run_out = gt + (eq < need_eq ? eq : need_eq), run_eq = eq;
    if (R.bnd_off >= 0 && lane == 0) {             // chunk c is apply tile c: its first entry
        int32_t* bnd = reinterpret_cast<int32_t*>(R.out + (int64_t)blockIdx.y * R.out_ld + R.bnd_off);
        bnd[c] = (int32_t)(run_out < R.k ? run_out : R.k);
        if (c == nchunks - 1) bnd[nchunks] = (int32_t)R.k;
    }
    for (int64_t i0 = 0; i0 < nc; i0 += 64) {
        const int64_t i = i0 + lane;
        const bool in = i < nc;
        const float d = !in ? 0.0f : i0 == 0 ? a0 : v.cval[c * kCvLd + i];
        const uint32_t key = key_of(d);
        const bool eq = in && key == T;
        const uint64_t be = __ballot(eq);          // flag ranks by ballot + mbcnt (exclusive counts)
        const uint32_t eex = lanes_below(be);
        const bool sel = in && (key > T || (eq && run_eq + (int64_t)eex < need_eq));
        const uint64_t bs = __ballot(sel);
        const int64_t pos = run_out + lanes_below(bs);
        if (sel && pos < R.k) {                    // (< k by construction; the guard keeps a corrupted
            v.vals[pos] = d;                       // scratch from writing outside the message)
            v.idx[pos] = c * kChunk + (i0 == 0 ? l0 : v.cloc[c * kClLd + i]);
        }
        run_out += __popcll(bs);
        run_eq += __popcll(be);
    }
}

// ---- D: the whole selection after the compaction in ONE launch (mx_topk_set "select" 1): the work
// of cand_hist<10>, cand_hist<9>, cand_mark and write_cand by B blocks of 1024 threads per row (one
// per CU) that meet at two row barriers instead of three kernel boundaries, with every candidate
// read from memory once.
//   load   the block's contiguous chunk regions [cb, ce) -- wave w owns chunks cb + w + 16 i -- the
//          first 128 candidates of each of up to kSelRC regions per wave cached in LDS; the 12-bit
//          candidate histogram resolved (bin b12, rank need1) while they fly
//   pass 1 10-bit digits (bits 9..18) of the candidates in bin b12 -> the block's histogram,
//          published to its slot (`sc1` stores); barrier 1; every block sums the B slots (`sc1`
//          loads) and resolves bin b10, rank need2
//   pass 2 9-bit digits of the candidates matching the 22-bit prefix -> the block's histogram, and
//          its count of keys above the prefix; barrier 2; every block sums the slots -> the exact
//          threshold key T and the ties to take, and from the slots of the blocks before it, its
//          own output base (keys > T and ties before its first chunk)
//   write  the counts > T / == T of every chunk, one block-wide scan in chunk order, then every
//          region's selected candidates in index order and its tile bound (write_cand's loop)
// Measured (tools/select_trace.py stage clocks, one row of the VGG-16 share, 29 blocks): load +
// 12-bit resolve 5.2 us, pass 1 1.6, barrier 1.8, 10-bit sums 2.6, pass 2 2.2, barrier 2.4, bases
// 3.3, write 7.6: 26.7 us, about the four passes' own kernel time (27.6 us), and the rounds are
// slower (one row 100.6 -> 103.9 us, 8 rows 608 -> 638 us, same box): the row's work sits on 29
// CUs instead of the whole chip, and each barrier costs what a kernel boundary does.  Not the
// default (mx_topk_set "select" 1 selects it); kept tested as the measured answer to "one launch".
// Hand-off protocol (MI355X_MICROARCH.md, "Valid forms", table row 1): the published words are
// `sc1` stores, every storing wave waits `vmcnt(0)`, a workgroup barrier, then one lane's agent-scope
// add to the row's counter; the consumer polls it with an `sc1` load, a workgroup barrier, then
// `sc1` loads of the slots; one workgroup per CU (the launch's LDS holds the CU).  The rare
// sampled-floor fallback (fewer than k candidates kept) re-compacts every key here, by these blocks,
// behind a fenced row barrier.  Every wait is bounded (the row's `err` word is set on expiry: the
// output is then undefined, never a hang); the row's blocks are co-resident (the host launches at
// most half the chip's CUs' worth of blocks at once).
constexpr int kSelTPB = 1024;
constexpr int kSelWaves = kSelTPB / 64;
constexpr int kSelRC = 8;                      // chunk regions per wave cached in LDS (128 candidates each)
// thread 0: poll the row's arrival counter until `target` (bounded: the row's error word is set)
__device__ __forceinline__ void spin_until(SelState* st, uint32_t target) {
    if (!wait_count(&st->bar, target)) st_sc1(&st->err, 1u);
}

// after this block's `sc1` publishing stores: arrive, wait for the row's other blocks
__device__ __forceinline__ void sel_barrier(SelState* st, uint32_t target) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add((g_u32*)&st->bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        spin_until(st, target);
    }
    __syncthreads();
}

// after plain stores (the fallback compaction): release, arrive, wait, acquire
__device__ __forceinline__ void sel_barrier_fenced(SelState* st, uint32_t target) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_fetch_add((g_u32*)&st->bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        spin_until(st, target);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
}

// block-wide sum of one value per thread (all threads receive it)
__device__ __forceinline__ int64_t sel_block_sum(int64_t x) {
    __shared__ int64_t part[kSelWaves];
    x = wave_sum64(x);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = x;
    __syncthreads();
    int64_t s = 0;
#pragma unroll
    for (int w = 0; w < kSelWaves; ++w) s += part[w];
    __syncthreads();
    return s;
}

__global__ __launch_bounds__(kSelTPB) void select_kernel(Rows R, int row0, int B, int64_t S, int trace) {
    // the launch's LDS caches the first 128 candidates of each of the wave's first kSelRC regions
    // (each wave reads back only its own regions: no barrier between a fill and its reads); its
    // size also holds the CU for this one workgroup
    extern __shared__ uint32_t sel_lds[];
    float* lv = reinterpret_cast<float*>(sel_lds);                           // [kSelRC][16][128]
    uint16_t* ll = reinterpret_cast<uint16_t*>(lv + kSelRC * kSelWaves * 128);   // the same, locations
    __shared__ int cnl[kSelRC][kSelWaves];
    const int r = row0 + (int)blockIdx.y;
    const RowView v = row_view(R, r);
    uint32_t* pub10 = reinterpret_cast<uint32_t*>(R.work + (int64_t)r * R.work_ld + layout(R.P).pub);
    uint32_t* pub9 = pub10 + kSelMaxB * kPub10;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // mx_topk_set("select_trace", 1): thread 0 of every block stores the constant clock at the stage
    // boundaries into the spare words of its 9-bit slot (a diagnostic; off by default)
    auto stamp = [&](int i) {
        if (trace && threadIdx.x == 0) pub9[blockIdx.x * kPub9 + (1 << kLowBits) + 1 + i] = (uint32_t)wall_clock64();
    };
    stamp(0);   // wave-uniform: region addresses in SGPRs
    const int b = blockIdx.x;
    const int64_t nc = n_chunks(R.P);
    const int64_t G = (nc + B - 1) / B;
    const int64_t cb = b * G < nc ? b * G : nc, ce = cb + G < nc ? cb + G : nc;
    const int iters = (int)((ce - cb + kSelWaves - 1) / kSelWaves);
    const int ncache = iters < kSelRC ? iters : kSelRC;
    __shared__ uint32_t h[kTopBins];

    // the wave's cached regions (speculative loads, all in flight together: a region is allocated
    // whatever its count, dead regions alias the block's first)
    auto load_cache = [&]() {
        float a0[kSelRC], a1[kSelRC];
        uint32_t l0[kSelRC], l1[kSelRC];
        int n[kSelRC];
#pragma unroll
        for (int i = 0; i < kSelRC; ++i) {
            const int64_t c = cb + (int64_t)i * kSelWaves + wave;
            const bool live = i < ncache && c < ce;
            const int64_t cc = live ? c : (cb < nc ? cb : 0);
            n[i] = live ? (int)v.cnt[kRec * cc + 3] : 0;
            a0[i] = v.cval[cc * kCvLd + lane];
            a1[i] = v.cval[cc * kCvLd + 64 + lane];
            l0[i] = v.cloc[cc * kClLd + lane];
            l1[i] = v.cloc[cc * kClLd + 64 + lane];
        }
#pragma unroll
        for (int i = 0; i < kSelRC; ++i) {
            const int o = (i * kSelWaves + wave) * 128;
            lv[o + lane] = a0[i];
            lv[o + 64 + lane] = a1[i];
            ll[o + lane] = (uint16_t)l0[i];
            ll[o + 64 + lane] = (uint16_t)l1[i];
            if (lane == 0) cnl[i][wave] = n[i];
        }
    };
    load_cache();
    const unsigned long long cand_n = v.st->cand_n;
    Bins<kTopBins, kSelTPB> a12, f12;
    load_bins<kTopBins, kSelTPB>(v.h12, a12);
    load_bins<kTopBins, kSelTPB>(v.h12f, f12);
    const bool fb = S != 1 && cand_n < (unsigned long long)R.k;  // row-uniform
    uint32_t bar0 = 0;
    if (fb) {
        // keep every key of this block's chunks, in index order, digits into the fallback histogram
        for (int i = tid; i < kTopBins; i += kSelTPB) h[i] = 0;
        __syncthreads();
        const bool vec = (((uintptr_t)v.x | (uintptr_t)v.xh) & 15) == 0;
        for (int64_t c = cb; c < ce; ++c) {
            for (int u = tid; u < kChunk / 4; u += kSelTPB) {
                float d[4];
                const int n = load_quad(v.x, v.xh, c * (kChunk / 4) + u, R.P, vec, d);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (e < n) {
                        v.cval[c * kCvLd + 4 * u + e] = d[e];
                        v.cloc[c * kClLd + 4 * u + e] = (uint16_t)(4 * u + e);
                        atomicAdd(&h[key_of(d[e]) >> kTopShift], 1u);
                    }
                }
            }
            const int64_t len = R.P - c * kChunk < kChunk ? R.P - c * kChunk : kChunk;
            if (wave == 0 && lane < kRec) v.cnt[kRec * c + lane] = lane == 3 ? len : 0;
        }
        __syncthreads();
        for (int i = tid; i < kTopBins; i += kSelTPB)
            if (h[i]) atomicAdd(&v.h12f[i], h[i]);
        bar0 = (uint32_t)B;
        sel_barrier_fenced(v.st, bar0);
        load_cache();
        load_bins<kTopBins, kSelTPB>(v.h12f, f12);
    }
    // 12-bit stage (the compaction's histogram, or the fallback's)
    int b12, b10, b9;
    int64_t need, tot;
    if (fb) {
#pragma unroll
        for (int j = 0; j < Bins<kTopBins, kSelTPB>::kPer; ++j) a12.c[j] = f12.c[j];
    }
    scan_bins<kTopBins, kSelTPB>(a12, R.k, &b12, &need, &tot);
    b12 = uni(b12);
    need = uni(need);
    stamp(1);

    // every candidate of the wave's i-th region, in 64-wide steps (cached ones from LDS)
    auto region_of = [&](int i) { return cb + (int64_t)i * kSelWaves + wave; };
    auto count_of = [&](int i) {
        if (i < ncache) return cnl[i][wave];
        const int64_t c = region_of(i);
        return c < ce ? (int)v.cnt[kRec * c + 3] : 0;
    };
    auto val_of = [&](int i, int j) {
        return i < ncache && j < 128 ? lv[(i * kSelWaves + wave) * 128 + j] : v.cval[region_of(i) * kCvLd + j];
    };
    auto loc_of = [&](int i, int j) {
        return i < ncache && j < 128 ? (uint32_t)ll[(i * kSelWaves + wave) * 128 + j]
                                     : (uint32_t)v.cloc[region_of(i) * kClLd + j];
    };
    // the cached regions' counts and both 64-wide slots, all read from LDS at once (one latency,
    // not a chain per region; regions past ncache were cached with count 0); tails past 128 and
    // uncached regions from memory
    int rn[kSelRC];
    float ra0[kSelRC], ra1[kSelRC];
    auto read_cache = [&]() {
#pragma unroll
        for (int i = 0; i < kSelRC; ++i) {
            const int o = (i * kSelWaves + wave) * 128;
            rn[i] = cnl[i][wave];
            ra0[i] = lv[o + lane];
            ra1[i] = lv[o + 64 + lane];
        }
    };
    auto for_regions = [&](auto&& f) {
        read_cache();
#pragma unroll
        for (int i = 0; i < kSelRC; ++i) {
            if (lane < rn[i]) f(ra0[i]);
            if (64 + lane < rn[i]) f(ra1[i]);
        }
#pragma unroll
        for (int i = 0; i < kSelRC; ++i)
            for (int j = 128 + lane; j < rn[i]; j += 64) f(v.cval[region_of(i) * kCvLd + j]);
        for (int i = ncache; i < iters; ++i) {
            const int64_t c = region_of(i);
            const int n = c < ce ? (int)v.cnt[kRec * c + 3] : 0;
            for (int j = lane; j < n; j += 64) f(v.cval[c * kCvLd + j]);
        }
    };

    // pass 1: 10-bit digits of bin b12; keys above bin b12 counted
    for (int i = tid; i < (1 << kMidBits); i += kSelTPB) h[i] = 0;
    __syncthreads();
    uint32_t gt = 0;
    for_regions([&](float d) {
        const uint32_t key = key_of(d);
        const uint32_t dg = key >> kTopShift;
        gt += dg > (uint32_t)b12;
        if (dg == (uint32_t)b12) atomicAdd(&h[(key >> kMidShift) & ((1u << kMidBits) - 1)], 1u);
    });
    __syncthreads();
    stamp(2);
    for (int i = tid; i < kPub10; i += kSelTPB) st_sc1(&pub10[b * kPub10 + i], h[i]);
    sel_barrier(v.st, bar0 + B);
    stamp(3);
    if (b == 0) {                                // nothing reads the 12-bit histograms or the
        for (int i = tid; i < 3 * kTopBins; i += kSelTPB) v.hs[i] = 0;   // candidate total any more
        for (int i = tid; i < kFineBins; i += kSelTPB) v.hsf[i] = 0;
        if (tid == 0) v.st->cand_n = 0;
    }
    {
        Bins<1 << kMidBits, kSelTPB> s10;        // thread t: bins 1023 - (2t + j), summed over the row's blocks
        constexpr int kPer = Bins<1 << kMidBits, kSelTPB>::kPer;
        uint32_t xs[kPer][kSelMaxB];             // every slot's load in flight at once (a summing loop
#pragma unroll                                   // waits one round trip per slot)
        for (int j = 0; j < kPer; ++j)
#pragma unroll
            for (int q = 0; q < kSelMaxB; ++q)
                xs[j][q] = ld_sc1(&pub10[(q < B ? q : 0) * kPub10 + (1 << kMidBits) - 1 - (tid * kPer + j)]);
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            uint32_t acc = 0;
#pragma unroll
            for (int q = 0; q < kSelMaxB; ++q) acc += q < B ? xs[j][q] : 0u;
            s10.c[j] = acc;
        }
        scan_bins<1 << kMidBits, kSelTPB>(s10, need, &b10, &need, &tot);
        b10 = uni(b10);
        need = uni(need);
    }
    stamp(4);
    const uint32_t pre22 = ((uint32_t)b12 << kMidBits) | (uint32_t)b10;   // key >> 9 of the prefix

    // pass 2: 9-bit digits of the keys matching the 22-bit prefix; keys above it counted
    for (int i = tid; i < (1 << kLowBits); i += kSelTPB) h[i] = 0;
    __syncthreads();
    for_regions([&](float d) {
        const uint32_t key = key_of(d);
        if ((key >> kTopShift) == (uint32_t)b12) {
            const uint32_t hi = key >> kMidShift;
            gt += hi > pre22;
            if (hi == pre22) atomicAdd(&h[key & ((1u << kLowBits) - 1)], 1u);
        }
    });
    const int64_t gt_blk = sel_block_sum(gt);  // its barriers also order the LDS histogram
    stamp(5);
    if (tid < (1 << kLowBits)) st_sc1(&pub9[b * kPub9 + tid], h[tid]);
    if (tid == 0) st_sc1(&pub9[b * kPub9 + (1 << kLowBits)], (uint32_t)gt_blk);
    sel_barrier(v.st, bar0 + 2 * B);
    stamp(6);
    int64_t base_gt, base_eq;
    {
        Bins<1 << kLowBits, kSelTPB> s9;         // thread t < 512: bin 511 - t
        uint32_t all = 0, before = 0;
        if (tid < (1 << kLowBits)) {
            uint32_t xs[kSelMaxB];
#pragma unroll
            for (int q = 0; q < kSelMaxB; ++q) xs[q] = ld_sc1(&pub9[(q < B ? q : 0) * kPub9 + (1 << kLowBits) - 1 - tid]);
#pragma unroll
            for (int q = 0; q < kSelMaxB; ++q) {
                all += q < B ? xs[q] : 0u;
                before += q < b ? xs[q] : 0u;
            }
        }
        s9.c[0] = all;
        scan_bins<1 << kLowBits, kSelTPB>(s9, need, &b9, &need, &tot);
        b9 = uni(b9);
        need = uni(need);
        const int bin = (1 << kLowBits) - 1 - tid;
        int64_t g = tid < (1 << kLowBits) && bin > b9 ? before : 0;
        if (tid < b) g += ld_sc1(&pub9[tid * kPub9 + (1 << kLowBits)]);
        base_gt = uni(sel_block_sum(g));
        base_eq = uni(sel_block_sum(tid < (1 << kLowBits) && bin == b9 ? before : 0));
    }
    stamp(7);
    const uint32_t T = (pre22 << kMidShift) | (uint32_t)b9;
    const int64_t need_eq = need;
    if (b == 0 && tid == 0) {
        v.st->T = T;
        v.st->need = need_eq;
        record_round(R, v.st, T, cand_n);
    }

    int32_t* bnd = R.bnd_off >= 0 ? reinterpret_cast<int32_t*>(R.out + (int64_t)r * R.out_ld + R.bnd_off) : nullptr;
    // one 64-wide step of a chunk's candidates in index order: ties ranked, the selected placed
    auto put = [&](int64_t c, float d, uint32_t loc, bool in, int64_t& run_out, int64_t& run_e) {
        const uint32_t key = key_of(d);
        const bool eq = in && key == T;
        const uint64_t be = __ballot(eq);
        const bool sel = in && (key > T || (eq && run_e + (int64_t)lanes_below(be) < need_eq));
        const uint64_t bs = __ballot(sel);
        const int64_t pos = run_out + lanes_below(bs);
        if (sel && pos < R.k) {
            v.vals[pos] = d;
            v.idx[pos] = c * kChunk + loc;
        }
        run_out += __popcll(bs);
        run_e += __popcll(be);
    };
    auto chunk_start = [&](int64_t c, int64_t gt_before, int64_t eq_before) {
        const int64_t run_out = gt_before + (eq_before < need_eq ? eq_before : need_eq);
        if (bnd && lane == 0) {
            bnd[c] = (int32_t)(run_out < R.k ? run_out : R.k);
            if (c == nc - 1) bnd[nc] = (int32_t)R.k;
        }
        return run_out;
    };
    if (iters <= kSelRC) {
        // every chunk cached: counts > T / == T of all of them at once, ONE block-wide exclusive
        // scan in chunk order (chunk cb + 16 i + w is entry 16 i + w), then every region placed
        // independently of the others
        __shared__ uint32_t sg[kSelRC * kSelWaves], se[kSelRC * kSelWaves];
        read_cache();
#pragma unroll
        for (int i = 0; i < kSelRC; ++i) {
            uint32_t g = (uint32_t)__popcll(__ballot(lane < rn[i] && key_of(ra0[i]) > T)) +
                         (uint32_t)__popcll(__ballot(64 + lane < rn[i] && key_of(ra1[i]) > T));
            uint32_t e = (uint32_t)__popcll(__ballot(lane < rn[i] && key_of(ra0[i]) == T)) +
                         (uint32_t)__popcll(__ballot(64 + lane < rn[i] && key_of(ra1[i]) == T));
            if (rn[i] > 128) {                       // a long region's tail (wave-uniform, rare)
                uint32_t tg = 0, te = 0;
                for (int j = 128 + lane; j < rn[i]; j += 64) {
                    const uint32_t key = key_of(v.cval[region_of(i) * kCvLd + j]);
                    tg += key > T;
                    te += key == T;
                }
                g += (uint32_t)wave_sum64(tg);
                e += (uint32_t)wave_sum64(te);
            }
            if (lane == 0) {
                sg[i * kSelWaves + wave] = g;
                se[i * kSelWaves + wave] = e;
            }
        }
        __syncthreads();
        static_assert(kSelRC * kSelWaves == 128, "one wave scans the block's chunk counts, two per lane");
        if (wave == 0) {
            const uint32_t g0 = sg[2 * lane], g1 = sg[2 * lane + 1], e0 = se[2 * lane], e1 = se[2 * lane + 1];
            const uint32_t gx = wave_incl_scan(g0 + g1) - (g0 + g1), ex = wave_incl_scan(e0 + e1) - (e0 + e1);
            sg[2 * lane] = gx;
            sg[2 * lane + 1] = gx + g0;
            se[2 * lane] = ex;
            se[2 * lane + 1] = ex + e0;
        }
        __syncthreads();
        // placement: everything it reads is in LDS (re-read per region rather than held across the
        // scan); a long region's tail (rare) reads memory after its region's stores.  Nothing loaded
        // from memory may still be in flight when the loop starts: the waitcnt pass would otherwise
        // wait for every output store at the loop head (vmcnt counts stores too)
        __builtin_amdgcn_s_waitcnt(0x0f70);      // vmcnt(0) (expcnt / lgkmcnt left alone)
        for (int i = 0; i < ncache; ++i) {
            const int64_t c = region_of(i);
            if (c >= ce) continue;
            const int o = (i * kSelWaves + wave) * 128;
            const int n = cnl[i][wave];
            int64_t run_e = base_eq + se[i * kSelWaves + wave];
            int64_t run_out = chunk_start(c, base_gt + sg[i * kSelWaves + wave], run_e);
            put(c, lv[o + lane], ll[o + lane], lane < n, run_out, run_e);
            if (n > 64) put(c, lv[o + 64 + lane], ll[o + 64 + lane], 64 + lane < n, run_out, run_e);
            for (int i0 = 128; i0 < n; i0 += 64) {
                const bool in = i0 + lane < n;
                put(c, in ? v.cval[c * kCvLd + i0 + lane] : 0.0f, in ? v.cloc[c * kClLd + i0 + lane] : 0u, in,
                    run_out, run_e);
            }
        }
    } else {
        // more regions than cached: per 16 chunks (one per wave), counts scanned across the waves
        __shared__ uint32_t xg[2][kSelWaves], xe[2][kSelWaves];
        int64_t run_gt = base_gt, run_eq = base_eq;
        int par = 0;
        for (int it = 0; it < iters; ++it) {
            const int64_t c = region_of(it);
            const int n = count_of(it);
            uint32_t g = 0, e = 0;
            for (int j = lane; j < n; j += 64) {
                const uint32_t key = key_of(val_of(it, j));
                g += key > T;
                e += key == T;
            }
            g = (uint32_t)wave_sum64(g);
            e = (uint32_t)wave_sum64(e);
            if (lane == 0) {
                xg[par][wave] = g;
                xe[par][wave] = e;
            }
            __syncthreads();
            int64_t pg = 0, pe = 0, ag = 0, ae = 0;
#pragma unroll
            for (int w = 0; w < kSelWaves; ++w) {
                pg += w < wave ? xg[par][w] : 0u;
                pe += w < wave ? xe[par][w] : 0u;
                ag += xg[par][w];
                ae += xe[par][w];
            }
            if (c < ce) {
                int64_t run_e = run_eq + pe;
                int64_t run_out = chunk_start(c, run_gt + pg, run_e);
                for (int i0 = 0; i0 < n; i0 += 64) {
                    const int i = i0 + lane;
                    const bool in = i < n;
                    put(c, in ? val_of(it, i) : 0.0f, in ? loc_of(it, i) : 0u, in, run_out, run_e);
                }
            }
            run_gt += ag;
            run_eq += ae;
            par ^= 1;
        }
    }
    __syncthreads();
    stamp(8);
}

// ------------------------------------------------------------------------------- apply
// ChocoCommunicator.averaging (communicator.py:200-230) fused into one pass per state tile.
// Row r's tile [t0, t0 + kTile) of s and x_hat is staged in LDS; every message that touches the
// tile is applied there in the reference order (partners in matching order, then the own
// message), then the dense update x = fma(-g, x_hat, fma(g, s, x)) streams x through once and
// only the 64-byte granules of s / x_hat that a message touched are written back.  Per element
// the rounding sequence is exactly the reference's; HBM traffic is x read + written, s and
// x_hat read once, their dirty granules written, and the messages read once.
//
// Messages are index-sorted, so the entries of message `slot` inside tile t are the range
// [bnd[t], bnd[t+1]) of the bounds the sender's write_cand stored after the message's indices
// (tile t = top-k chunk t: bnd[t] is that chunk's output offset).
constexpr int kTile = 4096;                    // elements per apply tile (16 KB of s + 16 KB of x_hat)

__host__ __device__ inline int64_t n_tiles(int64_t P) { return (P + kTile - 1) / kTile; }

static_assert(kTile == kChunk, "apply tiles are the top-k chunks (the message bounds are chunk offsets)");

struct Msg {
    const float* v;
    const int64_t* ix;
    const int32_t* bnd;
};

// message layout (mx_choco_msg_bytes): vals f32[kpad] | idx int64[k] | bnd int32[ntiles + 1]
// Where message `slot` starts: MsgStride -- one buffer, msg_ld bytes per slot (mx_choco_apply);
// MsgTable -- a device table of int64 addresses, one per slot (mx_choco_apply_slots, the pull
// transport: the local rows' messages here, the partners' in their owners' IPC-mapped snapshot
// buffers); the persistent apply copies either into LDS once per workgroup (MsgTable over LDS).
struct MsgStride {
    const char* m;
    int64_t ld;
    __device__ __forceinline__ const char* base(int slot) const { return m + (int64_t)slot * ld; }
};
struct MsgTable {
    const int64_t* tab;
    __device__ __forceinline__ const char* base(int slot) const { return reinterpret_cast<const char*>(tab[slot]); }
};

template <class MS>
__device__ __forceinline__ Msg msg_at(const MS& ms, int64_t kpad, int64_t k, int slot) {
    const char* b = ms.base(slot);
    return Msg{reinterpret_cast<const float*>(b), reinterpret_cast<const int64_t*>(b + 4 * kpad),
               reinterpret_cast<const int32_t*>(b + 4 * kpad + 8 * k)};
}

// Pull transport (plan word [2] bit 1, mx_plan_set_peer_reads): the partner messages are read from
// peers' IPC-mapped snapshot buffers, which this GPU's L2 may hold as non-local lines from two rounds
// ago.  One system-scope acquire per workgroup before its first message load -- the same protocol
// as the mixing kernels' peer_acquire (mix.hip); block-uniform, nothing for rounds without it.
__device__ __forceinline__ void peer_acquire(int32_t mode_word) {
    if (mode_word & 2) {
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");       // system scope: buffer_inv sc0 sc1
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
    }
}

// The plan record of this round: `rec` itself, or with iter_dev (graph-replayable launches) the
// record of round *iter_dev of the plan table at `rec`; null (launch is a no-op) when that round
// is outside [0, n_iters) or has no active matching -- communicator.py:249-250 skips such rounds.
__device__ __forceinline__ const int32_t* round_rec(const int32_t* rec, const int64_t* iter_dev, int64_t n_iters,
                                                   int64_t words) {
    if (!iter_dev) return rec;
    const int64_t v = *iter_dev;
    if (v < 0 || v >= n_iters) return nullptr;
    const int32_t* r = rec + v * words;
    return r[0] ? r : nullptr;
}

// NT: non-temporal accesses.  Chosen by the row count (mx_topk_set "apply_nt", -1 = auto): with
// several rows the streams are far larger than the Infinity Cache and the hints win (8 rows
// 0.65 ms vs 0.80 ms with ordinary accesses); a single row (config 4's share of one GPU at N = 8)
// runs 123 -> 117 us per round with ordinary accesses, the apply pass then finding part of x /
// x_hat the top-k pass has just read still on die (tools/choco_mall.py).
// GRAN: floats per dirty granule of s / x_hat written back.  16 (64 B) is the one instantiated: 32-B
// granules measured 8 rows 639 -> 715 us per round (same-box A/B; partial non-temporal line writes),
// one row unchanged
template <bool NT, int GRAN, class MS>
__device__ __forceinline__ void apply_tile(float* __restrict__ x, float* __restrict__ xh, float* __restrict__ s,
                                           int64_t ld, int64_t P, const MS& ms, int64_t kpad, int64_t k,
                                           const int32_t* __restrict__ rec, int n_local, int M, float alpha, float g,
                                           float* ls, float* lh, uint8_t* ds, uint8_t* dh, int r, int64_t t) {
    constexpr int kGran = GRAN;
    const int64_t t0 = t * kTile;
    const int len = (int)(P - t0 < kTile ? P - t0 : kTile);
    float* xr = x + (int64_t)r * ld + t0;
    float* sr = s + (int64_t)r * ld + t0;
    float* hr = xh + (int64_t)r * ld + t0;
    const int tid = threadIdx.x;
    const bool vec = len == kTile && (((uintptr_t)xr | (uintptr_t)sr | (uintptr_t)hr) & 15) == 0;
    constexpr int kQ = kTile / 4 / kTPB;       // quads per lane
    f4 xv[kQ];                                 // x is loaded up front: its stream overlaps the
    if (vec) {                                 // message phase instead of following it
#pragma unroll
        for (int j = 0; j < kQ; ++j) {
            const int q = j * kTPB + tid;
            xv[j] = ld4<NT>(reinterpret_cast<const f4*>(xr) + q);
            reinterpret_cast<f4*>(ls)[q] = ld4<NT>(reinterpret_cast<const f4*>(sr) + q);
            reinterpret_cast<f4*>(lh)[q] = ld4<NT>(reinterpret_cast<const f4*>(hr) + q);
        }
    } else {
        for (int i = tid; i < len; i += kTPB) {
            ls[i] = sr[i];
            lh[i] = hr[i];
        }
    }
    for (int i = tid; i < kTile / kGran; i += kTPB) ds[i] = dh[i] = 0;
    __syncthreads();
    const int32_t* deg = rec + mx::kPlanHeader;
    const int d = deg[r];
    const int32_t* src = deg + 2 * n_local + r * M;
    for (int e = 0; e < d; ++e) {              // partners, ascending matching order
        const Msg m = msg_at(ms, kpad, k, src[e]);
        const int lo = max(m.bnd[t], 0), hi = min(m.bnd[t + 1], (int)k);   // clamped: a received
        for (int q = lo + tid; q < hi; q += kTPB) {                        // message is not trusted
            const int c = (int)(m.ix[q] - t0);                             // to stay in range
            if ((unsigned)c >= (unsigned)len) continue;
            ls[c] = __fadd_rn(ls[c], __fmul_rn(alpha, m.v[q]));
            ds[c / kGran] = 1;
        }
        __syncthreads();                       // a later message may touch the same element
    }
    {                                          // own message
        const float sw = __int_as_float(deg[n_local + r]);
        const Msg m = msg_at(ms, kpad, k, r);
        const int lo = max(m.bnd[t], 0), hi = min(m.bnd[t + 1], (int)k);
        for (int q = lo + tid; q < hi; q += kTPB) {
            const int c = (int)(m.ix[q] - t0);
            if ((unsigned)c >= (unsigned)len) continue;
            const float vq = m.v[q];
            ls[c] = __fadd_rn(ls[c], __fmul_rn(sw, vq));
            lh[c] = __fadd_rn(lh[c], vq);
            ds[c / kGran] = 1;
            dh[c / kGran] = 1;
        }
    }
    __syncthreads();
    if (vec) {
#pragma unroll
        for (int j = 0; j < kQ; ++j) {
            const int q = j * kTPB + tid;
            f4 a = xv[j];
            const f4 sv = reinterpret_cast<const f4*>(ls)[q];
            const f4 hv = reinterpret_cast<const f4*>(lh)[q];
#pragma unroll
            for (int c = 0; c < 4; ++c) a[c] = __builtin_fmaf(-g, hv[c], __builtin_fmaf(g, sv[c], a[c]));
            st4<NT>(a, reinterpret_cast<f4*>(xr) + q);
            if (ds[q / (kGran / 4)]) st4<NT>(sv, reinterpret_cast<f4*>(sr) + q);
            if (dh[q / (kGran / 4)]) st4<NT>(hv, reinterpret_cast<f4*>(hr) + q);
        }
    } else {
        for (int i = tid; i < len; i += kTPB) {
            xr[i] = __builtin_fmaf(-g, lh[i], __builtin_fmaf(g, ls[i], xr[i]));
            if (ds[i / kGran]) sr[i] = ls[i];
            if (dh[i / kGran]) hr[i] = lh[i];
        }
    }
}

template <bool NT, int GRAN, bool SP>
__global__ __launch_bounds__(kTPB) void apply_kernel(float* __restrict__ x, float* __restrict__ xh,
                                                     float* __restrict__ s, int64_t ld, int64_t P,
                                                     const char* __restrict__ msgs, int64_t msg_ld,
                                                     int64_t kpad, int64_t k,
                                                     const int32_t* __restrict__ rec_in,
                                                     const int64_t* __restrict__ iter_dev, int64_t n_iters,
                                                     int64_t words, int n_local, int M,
                                                     float alpha, float g) {
    const int32_t* rec = round_rec(rec_in, iter_dev, n_iters, words);
    if (!rec) return;
    peer_acquire(rec[2]);
    __shared__ float ls[kTile], lh[kTile];
    __shared__ uint8_t ds[kTile / GRAN], dh[kTile / GRAN];
    if constexpr (SP)
        apply_tile<NT, GRAN>(x, xh, s, ld, P, MsgTable{reinterpret_cast<const int64_t*>(msgs)}, kpad, k, rec, n_local,
                             M, alpha, g, ls, lh, ds, dh, blockIdx.y, blockIdx.x);
    else
        apply_tile<NT, GRAN>(x, xh, s, ld, P, MsgStride{msgs, msg_ld}, kpad, k, rec, n_local, M, alpha, g, ls, lh,
                             ds, dh, blockIdx.y, blockIdx.x);
}

// The same pass with the message phase's global reads moved under the tile's stream: the plan
// record and every message's tile bounds are wave-uniform (scalar loads, their own counter), and
// the first kTPB entries of up to kPfMsgs messages are loaded per thread right after the x / s /
// x_hat loads and before s / x_hat are staged into LDS, so the ordered LDS updates then run
// without a memory round trip per message (the plain kernel pays two per message: bounds, then
// entries).  Entries past the first kTPB of a message in this tile, and messages past kPfMsgs,
// are loaded as in the plain kernel.  Same order of updates, same results.
constexpr int kPfMsgs = 8;

template <bool NT, class MS>
__device__ __forceinline__ void apply_pf_tile(float* __restrict__ x, float* __restrict__ xh, float* __restrict__ s,
                                              int64_t ld, int64_t P, const MS& ms, int64_t kpad, int64_t k,
                                              const int32_t* __restrict__ rec, int n_local, int M, float alpha,
                                              float g, float* ls, float* lh, uint8_t* ds, uint8_t* dh, int r,
                                              int64_t t) {
    constexpr int kGran = 16;
    const int64_t t0 = t * kTile;
    const int len = (int)(P - t0 < kTile ? P - t0 : kTile);
    float* xr = x + (int64_t)r * ld + t0;
    float* sr = s + (int64_t)r * ld + t0;
    float* hr = xh + (int64_t)r * ld + t0;
    if (!(len == kTile && (((uintptr_t)xr | (uintptr_t)sr | (uintptr_t)hr) & 15) == 0)) {   // partial /
        apply_tile<NT, 16>(x, xh, s, ld, P, ms, kpad, k, rec, n_local, M, alpha, g, ls, lh, ds, dh, r, t);
        return;                                                                         // unaligned tile
    }
    // from here on the whole-tile path is branch-free up to the message phase, so the waitcnt pass
    // can count the loads in flight exactly (a merge of two paths makes it wait for all of them)
    const int tid = threadIdx.x;
    constexpr int kQ = kTile / 4 / kTPB;       // quads per lane
    const int32_t* deg = rec + mx::kPlanHeader;
    const int d = deg[r];
    const int nm = d + 1;                      // partners in matching order, then the own message
    const int32_t* src = deg + 2 * n_local + r * M;
    const float sw = __int_as_float(deg[n_local + r]);
    // lane e < kPfMsgs of every wave: message e's slot, then its bounds in this tile -- two small
    // vector loads issued BEFORE the tile stream (vector loads return in order), so the entry
    // loads that need them can be issued right behind the stream
    const int lane = tid & 63;
    int my_lo = 0, my_hi = 0, my_sl = r;
    {
        const int e = lane < kPfMsgs ? lane : 0;
        const int sl = lane < kPfMsgs && e < d ? src[e] : r;
        my_sl = sl;
        const Msg m = msg_at(ms, kpad, k, sl);
        if (lane < kPfMsgs && e < nm) {
            my_lo = max(m.bnd[t], 0);              // clamped: a received message is not trusted
            my_hi = min(m.bnd[t + 1], (int)k);     // to stay in range
        }
    }
    f4 xv[kQ], sv[kQ], hv[kQ];
#pragma unroll
    for (int j = 0; j < kQ; ++j) {
        const int q = j * kTPB + tid;
        xv[j] = ld4<NT>(reinterpret_cast<const f4*>(xr) + q);
        sv[j] = ld4<NT>(reinterpret_cast<const f4*>(sr) + q);
        hv[j] = ld4<NT>(reinterpret_cast<const f4*>(hr) + q);
    }
    int plo[kPfMsgs], phi[kPfMsgs];
    int64_t pix[kPfMsgs];
    float pv[kPfMsgs];
#pragma unroll
    for (int e = 0; e < kPfMsgs; ++e) {
        plo[e] = __builtin_amdgcn_readlane(my_lo, e);
        phi[e] = __builtin_amdgcn_readlane(my_hi, e);
        const int q = plo[e] + tid < phi[e] ? plo[e] + tid : 0;     // clamped: loads stay unconditional
        const Msg m = msg_at(ms, kpad, k, __builtin_amdgcn_readlane(my_sl, e));
        pix[e] = m.ix[q];
        pv[e] = m.v[q];
    }
#pragma unroll
    for (int j = 0; j < kQ; ++j) {
        const int q = j * kTPB + tid;
        reinterpret_cast<f4*>(ls)[q] = sv[j];
        reinterpret_cast<f4*>(lh)[q] = hv[j];
    }
    for (int i = tid; i < kTile / kGran; i += kTPB) ds[i] = dh[i] = 0;
    __syncthreads();
    auto upd = [&](bool own, int64_t ix, float vq) {
        const int c = (int)(ix - t0);
        if ((unsigned)c >= (unsigned)len) return;
        ls[c] = __fadd_rn(ls[c], __fmul_rn(own ? sw : alpha, vq));
        ds[c / kGran] = 1;
        if (own) {
            lh[c] = __fadd_rn(lh[c], vq);
            dh[c / kGran] = 1;
        }
    };
#pragma unroll
    for (int e = 0; e < kPfMsgs; ++e) {
        if (e >= nm) break;
        const bool own = e == d;
        if (plo[e] + tid < phi[e]) upd(own, pix[e], pv[e]);
        if (phi[e] - plo[e] > kTPB) {
            const Msg m = msg_at(ms, kpad, k, __builtin_amdgcn_readlane(my_sl, e));
            for (int q = plo[e] + kTPB + tid; q < phi[e]; q += kTPB) upd(own, m.ix[q], m.v[q]);
        }
        __syncthreads();                       // a later message may touch the same element
    }
    for (int e = kPfMsgs; e < nm; ++e) {
        const bool own = e == d;
        const Msg m = msg_at(ms, kpad, k, own ? r : src[e]);
        const int lo = max(m.bnd[t], 0), hi = min(m.bnd[t + 1], (int)k);
        for (int q = lo + tid; q < hi; q += kTPB) upd(own, m.ix[q], m.v[q]);
        __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < kQ; ++j) {
        const int q = j * kTPB + tid;
        f4 a = xv[j];
        const f4 s4 = reinterpret_cast<const f4*>(ls)[q];
        const f4 h4 = reinterpret_cast<const f4*>(lh)[q];
#pragma unroll
        for (int c = 0; c < 4; ++c) a[c] = __builtin_fmaf(-g, h4[c], __builtin_fmaf(g, s4[c], a[c]));
        st4<NT>(a, reinterpret_cast<f4*>(xr) + q);
        if (ds[q / (kGran / 4)]) st4<NT>(s4, reinterpret_cast<f4*>(sr) + q);
        if (dh[q / (kGran / 4)]) st4<NT>(h4, reinterpret_cast<f4*>(hr) + q);
    }
}

template <bool NT, bool SP>
__global__ __launch_bounds__(kTPB) void apply_kernel_pf(float* __restrict__ x, float* __restrict__ xh,
                                                        float* __restrict__ s, int64_t ld, int64_t P,
                                                        const char* __restrict__ msgs, int64_t msg_ld,
                                                        int64_t kpad, int64_t k,
                                                        const int32_t* __restrict__ rec_in,
                                                        const int64_t* __restrict__ iter_dev, int64_t n_iters,
                                                        int64_t words, int n_local, int M,
                                                        float alpha, float g) {
    const int32_t* rec = round_rec(rec_in, iter_dev, n_iters, words);
    if (!rec) return;
    peer_acquire(rec[2]);
    __shared__ float ls[kTile], lh[kTile];
    __shared__ uint8_t ds[kTile / 16], dh[kTile / 16];
    if constexpr (SP)
        apply_pf_tile<NT>(x, xh, s, ld, P, MsgTable{reinterpret_cast<const int64_t*>(msgs)}, kpad, k, rec, n_local,
                          M, alpha, g, ls, lh, ds, dh, blockIdx.y, blockIdx.x);
    else
        apply_pf_tile<NT>(x, xh, s, ld, P, MsgStride{msgs, msg_ld}, kpad, k, rec, n_local, M, alpha, g, ls, lh, ds,
                          dh, blockIdx.y, blockIdx.x);
}

// Persistent form (a grid of about the co-resident workgroups, each looping over the tiles
// blockIdx.x, + gridDim.x, ... of row blockIdx.y): per workgroup, not per tile, the pull
// transport's system-scope acquire (peer-reads bit) and the message addresses -- the slot table
// (SP) or the strided addresses -- loaded once into LDS.  The per-tile work is apply_pf_tile's.
constexpr int kLdsSlots = 256;

template <bool NT, bool SP>
__global__ __launch_bounds__(kTPB) void apply_kernel_persist(float* __restrict__ x, float* __restrict__ xh,
                                                             float* __restrict__ s, int64_t ld, int64_t P,
                                                             const char* __restrict__ msgs, int64_t msg_ld,
                                                             int64_t kpad, int64_t k,
                                                             const int32_t* __restrict__ rec_in,
                                                             const int64_t* __restrict__ iter_dev, int64_t n_iters,
                                                             int64_t words, int n_local, int M,
                                                             float alpha, float g, int n_slots, int64_t ntiles) {
    const int32_t* rec = round_rec(rec_in, iter_dev, n_iters, words);
    if (!rec) return;
    peer_acquire(rec[2]);
    __shared__ float ls[kTile], lh[kTile];
    __shared__ uint8_t ds[kTile / 16], dh[kTile / 16];
    __shared__ int64_t ltab[kLdsSlots];
    for (int i = threadIdx.x; i < n_slots; i += kTPB)
        ltab[i] = SP ? reinterpret_cast<const int64_t*>(msgs)[i] : (int64_t)(msgs + (int64_t)i * msg_ld);
    __syncthreads();
    const MsgTable ms{ltab};
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        apply_pf_tile<NT>(x, xh, s, ld, P, ms, kpad, k, rec, n_local, M, alpha, g, ls, lh, ds, dh, blockIdx.y, t);
        __syncthreads();                       // the next tile restages ls / lh / ds / dh
    }
}

unsigned clamp_grid(int64_t n, int64_t per, int64_t cap) {
    int64_t g = (n + per - 1) / per;
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    return (unsigned)g;
}
}  // namespace

int g_sample_stride = 0;   // 0 = auto (about kSampleTarget sampled elements per row)
// host copies of the two device-side knobs, per device: hipMemcpyToSymbol writes the CURRENT
// device's copy of the symbol only, so mx_topk_set applies them to the current device and
// mx_topk_get reports the current device's value (a process driving several GPUs sets
// them per device; setting every device would create a context on each)
constexpr int kMaxDev = 64;
uint64_t g_spin_ticks_host[kMaxDev];       // 0 = never set on that device: kSpinTicks
int g_compact_trace[kMaxDev];
int cur_dev() {
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= kMaxDev) d = 0;
    return d;
}
int g_compact_blocks = 0;     // persistent compaction blocks over all rows; 0 = auto: ~720 for one
                              // row (an even chunk count each), 2560 for several (same-box sweeps: one row 256 / 384 / 512 / 640 /
                              // 1024 / 2048 blocks 131 / 121 / 116.4 / 116.2 / 119 / 134 us per round,
                              // the per-block prologue and flush outweigh the parallelism; 8 rows
                              // 0.667 -> 0.656 ms at 2048, flat from 768 to 3072)
int g_sample_pieces = 1;      // sampled 1024-element pieces per wave (sample_kernel grid)
int g_apply_pf = 1;           // apply pass: 1 message entries prefetched under the tile stream, 0 plain
int g_apply_nt = -1;          // apply pass non-temporal accesses: -1 auto (only with several rows), 0, 1
int g_apply_persist = -1;     // persistent apply (apply_kernel_persist): -1 auto (the slot-table form only), 0, 1
int g_compact_wave = 0;       // compaction with wave-owned chunks: 0 = off (block-owned chunks), c > 0 = about
                              // c chunks per wave
int g_compact_pf2 = 0;        // compaction: 1 = two whole chunks in flight per wave (PF2), 0 = one
int g_compact_store = 1;      // compaction candidate stores: 1 (default) a loop over the lane's kept elements,
                              // 0 one masked store pair per (step, element) (same-box A/B: 8 rows 639 -> 632 us,
                              // one row 114.4 -> 113.2 us)
int g_cand_chunks = 0;        // chunk regions per wave of cand_hist / cand_mark; 0 = auto: 4 for one
                              // row, 8 for several (fewer blocks = fewer histogram flushes: a second
                              // flush of cand_hist<10>'s 1024 bins measured +3.7 us on one row; same-box
                              // sweep 2 -> 4 / 8: one row 121.7 -> 119.6 us, 8 rows 655 -> 640 us)

int g_fine_floor = 1;          // 1: the sampled floor refined to 1/64 of a top digit inside a window around
                               // the last call's k-th key, 0: the digit floor.  Same box, 3 interleaved
                               // repeats (tools/choco_hint.py, profiles/r04b_choco_fine_floor.log): 8 rows
                               // keep 1.35 k candidates instead of 1.5-4.2 k, 629-633 -> 598-613 us per
                               // round with and without drift; one row neutral (102.0-103.2 us)
int g_floor_hint = -1;         // >= 0: candidate floor from the previous call's k-th key minus this many
                               // 12-bit bins (adaptive per row), no sampling launch; -1: sampled floor
unsigned g_hist_grid = 0;      // the last call's cand_hist<10> grid per row, and the co-resident cap it
unsigned g_hist_capacity = 0;  // was held to (blocks of that instantiation the chip holds, x 7/8): mx_topk_get

int g_select = 0;             // selection after the compaction: 0 = the four passes (cand_hist<10>,
                              // cand_hist<9>, cand_mark, write_cand), 1 = one launch (select_kernel; same-box
                              // A/B: one row 100.6 -> 103.9 us, 8 rows 608 -> 638 us per round, not the default)
int g_select_blocks = 0;      // select_kernel blocks per row; 0 = auto (every region cached, <= 32)
int g_select_trace = 0;       // select_kernel stage clocks into the scratch (diagnostic)
constexpr size_t kSelHoldBytes = (size_t)kSelRC * kSelWaves * 128 * 6;   // select_kernel's region cache (96 KB)

// select_kernel blocks one launch may hold: half the chip's CUs (one block per CU; the rest of the
// chip stays free for whatever else runs, so a row's blocks are always co-resident)
int select_capacity() {
    static int cached[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 64;
    if (!cached[dev]) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 2) cus = 128;
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(select_kernel),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSelHoldBytes);
        cached[dev] = cus / 2;
    }
    return cached[dev];
}

// blocks of a cand_hist<10> instantiation the chip holds at once, x 7/8 (room for a neighbour
// kernel such as RCCL's at N > 1), per device and instantiation
int64_t hist_capacity(const void* fn) {
    struct Entry { int dev; const void* fn; int64_t cap; };
    static Entry cache[32];
    static int used = 0;
    static std::mutex mu;                    // host threads may launch on several devices at once
    std::lock_guard<std::mutex> lock(mu);
    int dev = 0;
    (void)hipGetDevice(&dev);
    for (int i = 0; i < used; ++i)
        if (cache[i].dev == dev && cache[i].fn == fn) return cache[i].cap;
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kTPB, 0) != hipSuccess || per_cu < 1) per_cu = 1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 1;
    const int64_t cap = (int64_t)per_cu * cus * 7 / 8 > 0 ? (int64_t)per_cu * cus * 7 / 8 : 1;
    if (used < 32) cache[used++] = Entry{dev, fn, cap};
    return cap;
}

// workgroups of the persistent apply the chip holds at once (x 7/8, as hist_capacity)
int64_t persist_capacity(const void* fn) { return hist_capacity(fn); }

int64_t sample_stride(int64_t P) {
    const int64_t nc = n_chunks(P);
    int64_t S = g_sample_stride > 0 ? g_sample_stride : (nc * kChunk) / kSampleTarget;
    const int64_t ns = n_subs(P);
    if (S < 1) S = 1;
    if (S > ns) S = ns;
    return S;
}

extern "C" size_t mx_topk_work_bytes(int64_t P) { return layout(P < 1 ? 1 : P).total; }

extern "C" int64_t mx_choco_msg_bytes(int64_t P, int64_t k) {
    if (P < 1 || k < 1) return 0;
    return 4 * ((k + 1) / 2 * 2) + 8 * k + 4 * (n_chunks(P) + 1);
}

extern "C" int mx_topk_set(const char* key, int64_t value) {
    MX_CHECK(key, "mx_topk_set: null key");
    if (!strcmp(key, "sample_stride")) {
        MX_CHECK(value >= 0, "mx_topk_set: sample_stride %lld", (long long)value);
        g_sample_stride = (int)value;
        return MX_OK;
    }
    if (!strcmp(key, "compact_blocks")) {
        MX_CHECK(value >= 0 && value <= (1 << 20), "mx_topk_set: compact_blocks %lld", (long long)value);
        g_compact_blocks = (int)value;
        return MX_OK;
    }
    if (!strcmp(key, "cand_chunks")) {
        MX_CHECK(value >= 0 && value <= 4096, "mx_topk_set: cand_chunks %lld", (long long)value);
        g_cand_chunks = (int)value;
        return MX_OK;
    }
    if (!strcmp(key, "apply_nt")) {
        MX_CHECK(value >= -1 && value <= 1, "mx_topk_set: apply_nt %lld", (long long)value);
        g_apply_nt = (int)value;
        return MX_OK;
    }
    if (!strcmp(key, "apply_persist")) {
        MX_CHECK(value >= -1 && value <= 1, "mx_topk_set: apply_persist %lld", (long long)value);
        g_apply_persist = (int)value;
        return MX_OK;
    }
    if (!strcmp(key, "apply_pf")) {
        MX_CHECK(value == 0 || value == 1, "mx_topk_set: apply_pf %lld", (long long)value);
        g_apply_pf = (int)value;
        return MX_OK;
    }
    if (!strcmp(key, "compact_store")) {
        MX_CHECK(value == 0 || value == 1, "mx_topk_set: compact_store %lld", (long long)value);
        g_compact_store = (int)value;
        return MX_OK;
    }
    if (!strcmp(key, "compact_wave")) {
        MX_CHECK(value >= 0 && value <= 1024, "mx_topk_set: compact_wave %lld", (long long)value);
        g_compact_wave = (int)value;
        return MX_OK;
    }
    if (!strcmp(key, "compact_pf2")) {
        MX_CHECK(value == 0 || value == 1, "mx_topk_set: compact_pf2 %lld", (long long)value);
        g_compact_pf2 = (int)value;
        return MX_OK;
    }
    if (!strcmp(key, "select")) {
        MX_CHECK(value == 0 || value == 1, "mx_topk_set: select %lld", (long long)value);
        g_select = (int)value;
        return MX_OK;
    }
    if (!strcmp(key, "fine_floor")) {
        MX_CHECK(value == 0 || value == 1, "mx_topk_set: fine_floor %lld", (long long)value);
        g_fine_floor = (int)value;
        return MX_OK;
    }
    if (!strcmp(key, "floor_hint")) {
        MX_CHECK(value >= -1 && value <= 64, "mx_topk_set: floor_hint %lld (-1 off, 0..64 bins)", (long long)value);
        g_floor_hint = (int)value;
        return MX_OK;
    }
    if (!strcmp(key, "select_trace")) {
        g_select_trace = value != 0;
        return MX_OK;
    }
    if (!strcmp(key, "select_blocks")) {
        MX_CHECK(value >= 0 && value <= kSelMaxB, "mx_topk_set: select_blocks %lld", (long long)value);
        g_select_blocks = (int)value;
        return MX_OK;
    }
    if (!strcmp(key, "compact_trace")) {
        const int on = value != 0;
        MX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_ctrace_on), &on, sizeof(on)));
        g_compact_trace[cur_dev()] = on;
        return MX_OK;
    }
    if (!strcmp(key, "spin_ticks")) {
        MX_CHECK(value >= 0, "mx_topk_set: spin_ticks %lld", (long long)value);
        const uint64_t v = (uint64_t)value;
        MX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_spin_ticks_dev), &v, sizeof(v)));
        g_spin_ticks_host[cur_dev()] = v + 1;        // stored + 1: 0 marks "never set"
        return MX_OK;
    }
    if (!strcmp(key, "sample_pieces")) {
        MX_CHECK(value >= 1 && value <= 1024, "mx_topk_set: sample_pieces %lld", (long long)value);
        g_sample_pieces = (int)value;
        return MX_OK;
    }
    MX_CHECK(false, "mx_topk_set: unknown key '%s'", key);
}

extern "C" int64_t mx_topk_get(const char* key) {
    if (key && !strcmp(key, "spin_ticks")) {
        const uint64_t v = g_spin_ticks_host[cur_dev()];
        return (int64_t)(v ? v - 1 : kSpinTicks);
    }
    if (key && !strcmp(key, "compact_trace")) return g_compact_trace[cur_dev()];
    if (key && !strcmp(key, "sample_stride")) return g_sample_stride;
    if (key && !strcmp(key, "compact_blocks")) return g_compact_blocks;
    if (key && !strcmp(key, "sample_pieces")) return g_sample_pieces;
    if (key && !strcmp(key, "cand_chunks")) return g_cand_chunks;
    if (key && !strcmp(key, "apply_nt")) return g_apply_nt;
    if (key && !strcmp(key, "compact_store")) return g_compact_store;
    if (key && !strcmp(key, "apply_pf")) return g_apply_pf;
    if (key && !strcmp(key, "apply_persist")) return g_apply_persist;
    if (key && !strcmp(key, "compact_pf2")) return g_compact_pf2;
    if (key && !strcmp(key, "compact_wave")) return g_compact_wave;
    if (key && !strcmp(key, "select")) return g_select;
    if (key && !strcmp(key, "select_blocks")) return g_select_blocks;
    if (key && !strcmp(key, "select_trace")) return g_select_trace;
    if (key && !strcmp(key, "hist_grid")) return g_hist_grid;
    if (key && !strcmp(key, "floor_hint")) return g_floor_hint;
    if (key && !strcmp(key, "fine_floor")) return g_fine_floor;
    if (key && !strcmp(key, "hist_capacity")) return g_hist_capacity;
    mx::set_error("mx_topk_get: unknown key '%s'", key ? key : "(null)");
    return MX_ERR_INVALID;
}

extern "C" int mx_topk_abs_diff_rows(const float* x, const float* x_hat, int64_t ld, int nrows, int64_t P,
                                     int64_t k, void* out, int64_t out_ld_bytes, int64_t idx_off_bytes,
                                     int64_t bnd_off_bytes, void* work, int64_t work_ld_bytes, void* stream) {
    MX_CHECK(x && out && work, "mx_topk_abs_diff_rows: null pointer");
    MX_CHECK(P >= 1 && k >= 1 && k <= P && nrows >= 1 && nrows <= 65535 && (nrows == 1 || ld >= P),
             "mx_topk_abs_diff_rows: P=%lld k=%lld nrows=%d ld=%lld", (long long)P, (long long)k, nrows, (long long)ld);
    MX_CHECK(((uintptr_t)(static_cast<char*>(out) + idx_off_bytes)) % 8 == 0 && (nrows == 1 || out_ld_bytes % 8 == 0),
             "mx_topk_abs_diff_rows: int64 index output must be 8-byte aligned");
    MX_CHECK(bnd_off_bytes < 0 || (((uintptr_t)(static_cast<char*>(out) + bnd_off_bytes)) % 4 == 0 &&
                                   (nrows == 1 || out_ld_bytes % 4 == 0) && k < (int64_t)1 << 31),
             "mx_topk_abs_diff_rows: tile bounds must be 4-byte aligned (and k < 2^31)");
    MX_CHECK(work_ld_bytes >= (int64_t)layout(P).total || nrows == 1, "mx_topk_abs_diff_rows: work_ld too small");
    MX_CHECK(((uintptr_t)work) % 256 == 0 && (nrows == 1 || work_ld_bytes % 256 == 0),
             "mx_topk_abs_diff_rows: work must be 256-byte aligned");
    hipStream_t st = mx::as_stream(stream);
    Rows R{x, x_hat, ld, static_cast<char*>(out), out_ld_bytes, idx_off_bytes, static_cast<char*>(work),
           work_ld_bytes, P, k, bnd_off_bytes, (int32_t)g_floor_hint, (int32_t)g_fine_floor};
    const int64_t nc = n_chunks(P);
    // S = 0: the floor comes from the previous call's k-th key (floor_hint), no sampling launch
    const int64_t S = g_floor_hint >= 0 ? 0 : sample_stride(P);
    const int64_t nsamp = S > 0 ? (n_subs(P) + S - 1) / S : 0;
    int64_t sampled = 0;                      // elements in the sampled pieces
    for (int64_t u = 0; u < nsamp; ++u) {
        const int64_t c0 = u * S * kSub;
        sampled += (P - c0 < kSub) ? P - c0 : kSub;
    }
    const double frac = S > 0 ? (double)sampled / (double)P : 1.0;
    MX_CHECK(nc <= 0x7fffffff && P < ((int64_t)1 << 32), "mx_topk_abs_diff_rows: P too large (uint32 histograms)");
    const int cblocks = g_compact_blocks > 0 ? g_compact_blocks : (nrows == 1 ? 640 : 2560);
    unsigned bgrid = clamp_grid(nc, 1, (cblocks + nrows - 1) / nrows);   // persistent
    if (nrows == 1 && g_compact_blocks == 0) {
        // one row: about 720 workgroups dealt whole chunk counts, so no last pass runs on a few
        // (VGG-16 share, 3607 chunks: 722 x 5; same box 101.3 -> 100.1 us per round vs 640)
        const int64_t q = (nc + 360) / 720 > 1 ? (nc + 360) / 720 : 1;
        bgrid = (unsigned)((nc + q - 1) / q);
    }
    const unsigned wgrid = (unsigned)((nc + kWaves - 1) / kWaves);          // one wave per chunk
    const unsigned sgrid = clamp_grid(nsamp > 0 ? nsamp : 1, (int64_t)g_sample_pieces * kWaves, (1024 + nrows - 1) / nrows);
    const int cchunks = g_cand_chunks > 0 ? g_cand_chunks : (nrows == 1 ? 4 : 8);
    const unsigned cgrid = clamp_grid(nc, (int64_t)cchunks * kWaves, (2048 + nrows - 1) / nrows);
#define MX_L(kern, grid, tpb, ...)                                                 \
    hipLaunchKernelGGL(kern, grid, dim3(tpb), 0, st, R, ##__VA_ARGS__);            \
    MX_LAUNCH_CHECK()
    if (S > 0) MX_L(sample_kernel, dim3(sgrid, nrows), kTPB, S);
    auto ck = nrows == 1 ? (g_compact_store ? (g_compact_pf2 ? compact_kernel<true, true, true> : compact_kernel<true, true>)
                                            : compact_kernel<true, false>)
                         : (g_compact_store ? (g_compact_pf2 ? compact_kernel<false, true, true> : compact_kernel<false, true>)
                                            : compact_kernel<false, false>);
    if (g_compact_wave) {
        // wave-owned chunks: about g_compact_wave chunks per wave (1 = one chunk each)
        const int64_t waves = (nc + g_compact_wave - 1) / g_compact_wave;
        const unsigned wg = clamp_grid(waves, kWaves, 65535);
        auto cw = nrows == 1 ? compact_wave_kernel<true> : compact_wave_kernel<false>;
        MX_L(cw, dim3(wg, nrows), kTPB, S, frac);
    } else {
        MX_L(ck, dim3(bgrid, nrows), kTPB, S, frac);
    }
    if (g_select) {
        // the fallback compaction (S > 1, rare) runs inside select_kernel; rows in batches of at
        // most select_capacity() blocks per launch
        // auto: the fewest blocks whose waves hold every region in the LDS cache (one row of the
        // VGG-16 share: 29), at most kSelMaxB
        int64_t Bw = g_select_blocks > 0 ? g_select_blocks : (nc + kSelRC * kSelWaves - 1) / (kSelRC * kSelWaves);
        const int B = (int)(Bw > kSelMaxB ? kSelMaxB : Bw < 1 ? 1 : Bw);
        const int cap = select_capacity();
        const int rpl = cap / B > 0 ? cap / B : 1;
        for (int r0 = 0; r0 < nrows; r0 += rpl) {
            const int nr = nrows - r0 < rpl ? nrows - r0 : rpl;
            hipLaunchKernelGGL(select_kernel, dim3((unsigned)B, (unsigned)nr), dim3(kSelTPB), kSelHoldBytes, st, R, r0,
                               B, S, g_select_trace);
            MX_LAUNCH_CHECK();
        }
        return MX_OK;
    }
    // the fallback compaction (S > 1, rare) runs inside the first candidate pass, behind a row grid
    // barrier: that pass's blocks (every row's) must all be resident at once, so with sampling its
    // grid is capped at 7/8 of the chip's capacity for the instantiation (occupancy query, cached)
    auto h10 = nrows == 1 ? (g_compact_store ? cand_hist<kMidBits, true, true> : cand_hist<kMidBits, true, false>)
                          : (g_compact_store ? cand_hist<kMidBits, false, true> : cand_hist<kMidBits, false, false>);
    unsigned hgrid = cgrid;
    if (S != 1) {
        const int64_t cap = hist_capacity(reinterpret_cast<const void*>(h10));
        MX_CHECK(cap >= nrows, "mx_topk_abs_diff_rows: %d rows exceed the %lld co-resident blocks of the candidate "
                 "pass (its sampled-floor fallback needs every block of a row resident)", nrows, (long long)cap);
        if ((int64_t)hgrid * nrows > cap) hgrid = (unsigned)(cap / nrows);
        g_hist_capacity = (unsigned)cap;
    } else {
        g_hist_capacity = 0;
    }
    g_hist_grid = hgrid;
    MX_L(h10, dim3(hgrid, nrows), kTPB, S, frac);
    MX_L((cand_hist<kLowBits, false, false>), dim3(cgrid, nrows), kTPB, S, frac);
    const int64_t G = (nc + cgrid - 1) / cgrid;    // chunks per cand_mark block
    MX_L(cand_mark, dim3(cgrid, nrows), kTPB, G);
    MX_L(write_cand, dim3(wgrid, nrows), kTPB, G);
#undef MX_L
    return MX_OK;
}

// The rows' sticky error words (a bounded row-barrier wait that expired: the sampled-floor fallback
// in cand_hist<10>, or select_kernel).
namespace {
// one lane: the first row whose error word is set (or -1), every set word cleared; the result goes
// to row 0's SelState.scan (the caller's own scratch: no word shared between calls or streams) and,
// when `flag` is given and a row was set, row + 1 to *flag with a system-scope release (a host-mapped
// word the host reads without synchronising: mx_topk_err_forward)
__global__ void err_scan_kernel(char* work, int64_t work_ld, int nrows, int64_t off, int64_t scan_off,
                                int32_t* flag) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int32_t bad = -1;
    for (int r = 0; r < nrows; ++r) {
        uint32_t* e = reinterpret_cast<uint32_t*>(work + (int64_t)r * work_ld + off);
        if (*e) {
            if (bad < 0) bad = r;
            *e = 0u;
        }
    }
    *reinterpret_cast<int32_t*>(work + scan_off) = bad;
    if (flag && bad >= 0)
        __hip_atomic_store((__attribute__((address_space(1))) int32_t*)flag, bad + 1, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

int launch_err_scan(void* work, int64_t work_ld_bytes, int nrows, int64_t P, int32_t* flag, hipStream_t st) {
    const int64_t off = (int64_t)(layout(P).state + offsetof(SelState, err));
    const int64_t scan_off = (int64_t)(layout(P).state + offsetof(SelState, scan));
    hipLaunchKernelGGL(err_scan_kernel, dim3(1), dim3(64), 0, st, static_cast<char*>(work), work_ld_bytes, nrows, off,
                       scan_off, flag);
    MX_LAUNCH_CHECK();
    return MX_OK;
}
}  // namespace

// Synchronises `stream`, reads and clears the words; MX_ERR_HIP naming the first row if any was set.
extern "C" int mx_topk_check(void* work, int64_t work_ld_bytes, int nrows, int64_t P, void* stream) {
    MX_CHECK(work && nrows >= 1 && P >= 1 && (nrows == 1 || work_ld_bytes >= (int64_t)layout(P).total),
             "mx_topk_check: bad arguments");
    hipStream_t st = mx::as_stream(stream);
    const int rc = launch_err_scan(work, work_ld_bytes, nrows, P, nullptr, st);
    if (rc != MX_OK) return rc;
    int32_t bad = -1;
    MX_HIP(hipMemcpyAsync(&bad, static_cast<char*>(work) + layout(P).state + offsetof(SelState, scan), sizeof(bad),
                          hipMemcpyDeviceToHost, st));
    MX_HIP(hipStreamSynchronize(st));
    if (bad >= 0) {
        mx::set_error("mx_topk: a row barrier's bounded wait expired (row %d): not every block of the row was "
                      "resident; that call's output is undefined", bad);
        return MX_ERR_HIP;
    }
    return MX_OK;
}

// Stream-ordered and non-blocking: the words are scanned and cleared on `stream` behind the call
// they belong to, and an expired one is forwarded as row + 1 to *flag_dev (mx_host_words: the host
// polls it without a synchronisation, e.g. at the start of its next call).
extern "C" int mx_topk_err_forward(void* work, int64_t work_ld_bytes, int nrows, int64_t P, int32_t* flag_dev,
                                   void* stream) {
    MX_CHECK(work && flag_dev && nrows >= 1 && P >= 1 &&
                 (nrows == 1 || work_ld_bytes >= (int64_t)layout(P).total),
             "mx_topk_err_forward: bad arguments");
    return launch_err_scan(work, work_ld_bytes, nrows, P, flag_dev, mx::as_stream(stream));
}

// The compaction trace (mx_topk_set "compact_trace" 1): n <= 8192 workgroups x {start, floor
// resolved, end} constant-clock stamps of the last traced launch (row 0's blocks).  Synchronises.
extern "C" int mx_topk_trace(uint64_t* out, int64_t nblocks) {
    MX_CHECK(out && nblocks >= 1 && nblocks <= kTraceBlocks, "mx_topk_trace: nblocks %lld", (long long)nblocks);
    MX_HIP(hipDeviceSynchronize());
    MX_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ctrace), (size_t)nblocks * 3 * sizeof(uint64_t)));
    return MX_OK;
}

// Per row: {calls, fallback compactions, current floor-hint margin, the last call's threshold key T,
// its candidate count} (diagnostics of the floor choice).
extern "C" int mx_topk_stats(const void* work, int64_t work_ld_bytes, int nrows, int64_t P, int64_t* out,
                             void* stream) {
    MX_CHECK(work && out && nrows >= 1 && P >= 1 && (nrows == 1 || work_ld_bytes >= (int64_t)layout(P).total),
             "mx_topk_stats: bad arguments");
    MX_HIP(hipStreamSynchronize(mx::as_stream(stream)));
    for (int r = 0; r < nrows; ++r) {
        SelState st;
        MX_HIP(hipMemcpy(&st, static_cast<const char*>(work) + (int64_t)r * work_ld_bytes + layout(P).state, sizeof(st),
                         hipMemcpyDeviceToHost));
        out[5 * r] = st.n_calls;
        out[5 * r + 1] = st.n_fallbacks;
        out[5 * r + 2] = st.margin;
        out[5 * r + 3] = st.T;
        out[5 * r + 4] = st.last_cand;
    }
    return MX_OK;
}

extern "C" int mx_topk_abs_diff(const float* x, const float* x_hat, int64_t P, int64_t k, float* vals,
                                int64_t* idx, void* work, void* stream) {
    MX_CHECK(vals && idx, "mx_topk_abs_diff: null pointer");
    const int64_t idx_off = reinterpret_cast<char*>(idx) - reinterpret_cast<char*>(vals);
    return mx_topk_abs_diff_rows(x, x_hat, P, 1, P, k, vals, 0, idx_off, -1, work, 0, stream);
}

// The tile bounds travel inside the messages; mx_choco_apply needs no scratch (kept in the ABI).
extern "C" size_t mx_choco_apply_work_bytes(int64_t, int) { return 0; }

namespace {
int choco_apply(float* x, float* xhat, float* s, int64_t ld, int64_t P, int64_t k, const void* msgs,
                int64_t msg_ld_bytes, int n_slots, const int32_t* plan_dev, int64_t iter, const int64_t* iter_dev,
                int n_local, int M, float alpha, float gamma, void* work, void* stream, bool slot_table = false);
}

// The pull transport's apply (ChocoWorkerGroup under PullTransport): message `slot` is read from the
// address slot_ptrs_dev[slot] -- the local rows' messages in this GPU's message buffer, the partners'
// in their owners' IPC-mapped snapshot buffers (pointed there by mx_pull_gate on the device).  Same
// pass, same order of updates, same bits as mx_choco_apply.
extern "C" int mx_choco_apply_slots(float* x, float* xhat, float* s, int64_t ld, int64_t P, int64_t k,
                                    const int64_t* slot_ptrs_dev, int n_slots, const int32_t* plan_dev,
                                    int64_t iter, int n_local, int M, float alpha, float gamma, void* stream) {
    MX_CHECK(iter >= 0, "mx_choco_apply_slots: iter < 0");
    MX_CHECK(slot_ptrs_dev, "mx_choco_apply_slots: null slot table");
    return choco_apply(x, xhat, s, ld, P, k, slot_ptrs_dev, 0, n_slots, plan_dev, iter, nullptr, n_local, M,
                       alpha, gamma, nullptr, stream, true);
}

extern "C" int mx_choco_apply(float* x, float* xhat, float* s, int64_t ld, int64_t P, int64_t k,
                              const void* msgs, int64_t msg_ld_bytes, int n_slots, const int32_t* plan_dev,
                              int64_t iter, int n_local, int M, float alpha, float gamma, void* work,
                              void* stream) {
    MX_CHECK(iter >= 0, "mx_choco_apply: iter < 0");
    return choco_apply(x, xhat, s, ld, P, k, msgs, msg_ld_bytes, n_slots, plan_dev, iter, nullptr, n_local, M,
                       alpha, gamma, work, stream);
}

extern "C" int mx_choco_apply_at(float* x, float* xhat, float* s, int64_t ld, int64_t P, int64_t k,
                                 const void* msgs, int64_t msg_ld_bytes, int n_slots, const int32_t* plan_dev,
                                 const int64_t* iter_dev, int64_t n_iters, int n_local, int M, float alpha,
                                 float gamma, void* work, void* stream) {
    MX_CHECK(iter_dev && n_iters >= 0, "mx_choco_apply_at: bad iteration counter");
    return choco_apply(x, xhat, s, ld, P, k, msgs, msg_ld_bytes, n_slots, plan_dev, n_iters, iter_dev, n_local, M,
                       alpha, gamma, work, stream);
}

namespace {
int choco_apply(float* x, float* xhat, float* s, int64_t ld, int64_t P, int64_t k, const void* msgs,
                int64_t msg_ld_bytes, int n_slots, const int32_t* plan_dev, int64_t iter, const int64_t* iter_dev,
                int n_local, int M, float alpha, float gamma, void* work, void* stream, bool slot_table) {
    (void)work;
    MX_CHECK(x && xhat && s && msgs && plan_dev, "mx_choco_apply: null pointer");
    MX_CHECK(P >= 1 && k >= 1 && k <= P && ld >= P && k < (int64_t)1 << 31, "mx_choco_apply: P=%lld k=%lld ld=%lld",
             (long long)P, (long long)k, (long long)ld);
    MX_CHECK(n_local >= 1 && n_local <= 65535 && n_slots >= n_local && n_slots <= 65535 && M >= 1,
             "mx_choco_apply: n_local=%d n_slots=%d M=%d", n_local, n_slots, M);
    const int64_t kpad = (k + 1) / 2 * 2;
    MX_CHECK(slot_table || (msg_ld_bytes >= mx_choco_msg_bytes(P, k) && msg_ld_bytes % 8 == 0),
             "mx_choco_apply: msg_ld %lld", (long long)msg_ld_bytes);
    hipStream_t st = mx::as_stream(stream);
    const int64_t words = mx::plan_words(n_local, M);
    const int32_t* rec = iter_dev ? plan_dev : plan_dev + iter * words;   // with iter_dev: iter = n_iters
    const int64_t nt = n_tiles(P);
    const char* m = static_cast<const char*>(msgs);
    MX_CHECK(nt <= 0x7fffffff, "mx_choco_apply: P too large");
    const bool nt_hint = g_apply_nt < 0 ? n_local > 1 : g_apply_nt > 0;
    // auto: only the slot-table form of ONE row (the direct pull read of config 4's share at N = 8:
    // 66 -> 57 us; with 2-8 rows, and for the strided form, the per-tile grid is faster --
    // tools/choco_slots_ab.py, profiles/r05p2_apply_forms_ab.log)
    const bool persist = n_slots <= kLdsSlots &&
                         (g_apply_persist > 0 || (g_apply_persist < 0 && slot_table && n_local == 1));
    if (persist) {
        auto kern = slot_table ? (nt_hint ? apply_kernel_persist<true, true> : apply_kernel_persist<false, true>)
                               : (nt_hint ? apply_kernel_persist<true, false> : apply_kernel_persist<false, false>);
        // about the co-resident workgroups over the rows, an equal tile count each
        const int64_t cap = persist_capacity(reinterpret_cast<const void*>(kern)) / n_local;
        const int64_t per = (nt + (cap > 0 ? cap : 1) - 1) / (cap > 0 ? cap : 1);
        const int64_t gx = (nt + per - 1) / per;
        hipLaunchKernelGGL(kern, dim3((unsigned)gx, n_local), dim3(kTPB), 0, st, x, xhat, s, ld, P, m, msg_ld_bytes,
                           kpad, k, rec, iter_dev, iter, words, n_local, M, alpha, gamma, n_slots, nt);
        MX_LAUNCH_CHECK();
        return MX_OK;
    }
    auto kern = slot_table ? (g_apply_pf ? (nt_hint ? apply_kernel_pf<true, true> : apply_kernel_pf<false, true>)
                                         : (nt_hint ? apply_kernel<true, 16, true> : apply_kernel<false, 16, true>))
                           : (g_apply_pf ? (nt_hint ? apply_kernel_pf<true, false> : apply_kernel_pf<false, false>)
                                         : (nt_hint ? apply_kernel<true, 16, false> : apply_kernel<false, 16, false>));
    hipLaunchKernelGGL(kern, dim3((unsigned)nt, n_local), dim3(kTPB),
                       0, st, x, xhat, s, ld, P, m,
                       msg_ld_bytes, kpad, k, rec, iter_dev, iter, words, n_local, M, alpha, gamma);
    MX_LAUNCH_CHECK();
    return MX_OK;
}
}  // namespace
