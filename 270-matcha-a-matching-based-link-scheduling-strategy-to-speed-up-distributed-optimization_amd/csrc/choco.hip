// choco.hip -- ChocoSGD compressed gossip on the GPU.
//
// mx_topk_abs_diff  = compressors.get_top_k (compressors.py:3-19) applied to
//                     send = x - x_hat (ChocoCommunicator.prepare_comm_buffer, communicator.py:188-190)
// mx_choco_apply    = ChocoCommunicator.averaging (communicator.py:200-230)
//
// Top-k (k largest |x - x_hat|, ties at the threshold resolved towards the lowest indices,
// output in index order) in THREE streaming passes over x / x_hat:
//   A  hist_kernel     12-bit histogram of the magnitude key's top digit (bits 19..30: the
//                      exponent + 4 mantissa bits) in LDS, non-zero bins flushed with atomics;
//      select_top      one block finds the digit b0 holding the k-th largest key;
//   B  split_kernel    per 4096-element chunk: count keys whose digit is above b0 (certainly
//                      selected) and append the keys in digit b0 (candidates) to a side buffer
//                      with wave-ballot compaction;
//      cand_hist/select_cand (x2, 10 + 9 bits) finish the radix select on the candidates only,
//      giving the exact threshold key T and how many of its ties are needed;
//      cand_mark       per-chunk counts of candidates > T and == T (order-free atomics);
//      scan_kernel     one block: per-chunk output offsets and tie ranks;
//   C  write_kernel    per chunk, wave-ballot stable compaction of every key > T plus the
//                      lowest-index ties, values = x - x_hat, indices int64.
// Everything stays on the device; no host round trip.  All local workers' rows are processed by
// the same launches (blockIdx.y = row), so a round costs ~11 launches, not ~11 per worker.
#include "mx_common.h"

namespace {
constexpr int kTPB = 256;
constexpr int kWaves = kTPB / 64;
constexpr int kChunk = 4096;                 // elements per chunk (4 quads of 4 per lane)
constexpr int kTopBits = 12, kTopShift = 19;
constexpr int kTopBins = 1 << kTopBits;
constexpr int kMidBits = 10, kMidShift = 9;  // bits 9..18
constexpr int kLowBits = 9;                  // bits 0..8
constexpr int kScanTPB = 1024;

struct SelState {
    uint32_t b0;          // top digit of the threshold bin
    uint32_t T;           // exact threshold key (after the candidate passes)
    uint32_t prefix;      // candidate-pass prefix (bits fixed so far, shifted to full key)
    uint32_t mask;
    int64_t need;         // keys still to take at/below the current bin / prefix
    int64_t cand_n;       // unused (candidates live in per-chunk regions)
};

struct WorkLayout {
    size_t hist, state, cnt, off, cidx, ckey, total;
};

__host__ __device__ inline WorkLayout layout(int64_t P) {
    const int64_t nchunks = (P + kChunk - 1) / kChunk;
    WorkLayout w;
    w.hist = 0;
    w.state = w.hist + sizeof(uint32_t) * kTopBins;
    w.cnt = w.state + 64;
    w.off = w.cnt + sizeof(int64_t) * 4 * (size_t)nchunks;
    w.cidx = (w.off + sizeof(int64_t) * 2 * (size_t)nchunks + 255) / 256 * 256;
    w.ckey = w.cidx + sizeof(int64_t) * (size_t)P;
    w.total = (w.ckey + sizeof(uint32_t) * (size_t)P + 255) / 256 * 256;
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
};

struct RowView {
    const float* x;
    const float* xh;
    uint32_t* hist;
    SelState* st;
    int64_t* cnt;
    int64_t* off;
    int64_t* cidx;
    uint32_t* ckey;
    float* vals;
    int64_t* idx;
};

__device__ __forceinline__ RowView row_view(const Rows& R) {
    const int r = blockIdx.y;
    const WorkLayout w = layout(R.P);
    char* wb = R.work + (int64_t)r * R.work_ld;
    RowView v;
    v.x = R.x + (int64_t)r * R.ld;
    v.xh = R.xh ? R.xh + (int64_t)r * R.ld : nullptr;
    v.hist = reinterpret_cast<uint32_t*>(wb + w.hist);
    v.st = reinterpret_cast<SelState*>(wb + w.state);
    v.cnt = reinterpret_cast<int64_t*>(wb + w.cnt);
    v.off = reinterpret_cast<int64_t*>(wb + w.off);
    v.cidx = reinterpret_cast<int64_t*>(wb + w.cidx);
    v.ckey = reinterpret_cast<uint32_t*>(wb + w.ckey);
    v.vals = reinterpret_cast<float*>(R.out + (int64_t)r * R.out_ld);
    v.idx = reinterpret_cast<int64_t*>(R.out + (int64_t)r * R.out_ld + R.idx_off);
    return v;
}

__device__ __forceinline__ uint32_t key_of(float d) { return __float_as_uint(d) & 0x7fffffffu; }

__device__ __forceinline__ float diff_at(const float* x, const float* xh, int64_t i) {
    return xh ? __fsub_rn(x[i], xh[i]) : x[i];
}

typedef float f4 __attribute__((ext_vector_type(4)));

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

// inclusive scan of a per-lane count over the wave
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

// ---- A: top-digit histogram
__global__ __launch_bounds__(kTPB) void hist_kernel(Rows R) {
    const RowView v = row_view(R);
    __shared__ uint32_t h[kTopBins];
    for (int i = threadIdx.x; i < kTopBins; i += kTPB) h[i] = 0;
    __syncthreads();
    const bool vec = (((uintptr_t)v.x | (uintptr_t)v.xh) & 15) == 0;
    const int64_t nq = (R.P + 3) / 4;
    constexpr int U = 4;                       // quads in flight per lane
    const int64_t stride = (int64_t)gridDim.x * kTPB;
    for (int64_t q0 = (int64_t)blockIdx.x * kTPB + threadIdx.x; q0 < nq; q0 += U * stride) {
        float d[U][4];
        int n[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t q = q0 + u * stride;
            n[u] = q < nq ? load_quad(v.x, v.xh, q, R.P, vec, d[u]) : 0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (c < n[u]) atomicAdd(&h[key_of(d[u][c]) >> kTopShift], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kTopBins; i += kTPB)
        if (h[i]) atomicAdd(&v.hist[i], h[i]);
}

// one block: the bin holding the need-th largest count, scanning bins from the top.
// bins/bin_shift describe the histogram; on exit st->need is the rank inside the chosen bin.
template <int NBINS>
__device__ void select_bin(uint32_t* __restrict__ hist, int64_t need, int* bin_out, int64_t* need_out) {
    constexpr int kPer = NBINS / kTPB;
    __shared__ int64_t part[kTPB];
    const int t = threadIdx.x;
    int64_t mine = 0;
    for (int j = 0; j < kPer; ++j) mine += hist[NBINS - 1 - (t * kPer + j)];
    part[t] = mine;
    __syncthreads();
    for (int off = 1; off < kTPB; off <<= 1) {          // inclusive scan from the top bins down
        const int64_t v = t >= off ? part[t - off] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    const int64_t before = part[t] - mine;
    if (before < need && part[t] >= need) {
        int64_t acc = before;
        for (int j = 0; j < kPer; ++j) {
            const int bin = NBINS - 1 - (t * kPer + j);
            const int64_t c = hist[bin];
            if (acc + c >= need) {
                *bin_out = bin;
                *need_out = need - acc;
                break;
            }
            acc += c;
        }
    }
    __syncthreads();
    for (int i = t; i < NBINS; i += kTPB) hist[i] = 0;     // ready for the next use
}

__global__ __launch_bounds__(kTPB) void select_top(Rows R) {
    const RowView v = row_view(R);
    SelState* st = v.st;
    __shared__ int bin;
    __shared__ int64_t need;
    select_bin<kTopBins>(v.hist, R.k, &bin, &need);
    __syncthreads();
    if (threadIdx.x == 0) {
        st->b0 = (uint32_t)bin;
        st->prefix = (uint32_t)bin << kTopShift;
        st->mask = 0xffffffffu << kTopShift;
        st->need = need;
        st->cand_n = 0;
        st->T = 0;
    }
}

// ---- B: per-chunk "certainly selected" counts + candidate compaction.  A chunk is 4 sub-tiles of
// 256 lanes x one 16-byte quad; the 16 keys per lane stay in registers and a wave scan of the
// per-lane candidate counts ranks them inside the chunk's OWN region of the candidate buffer
// (chunk c owns slots [c*4096, c*4096 + ncand)), so no global atomics are needed.
// cnt[4c + 0..3] = {keys above digit b0, candidates > T, candidates == T, candidates}.
constexpr int kQuads = kChunk / (4 * kTPB);   // quads per lane per chunk

__global__ __launch_bounds__(kTPB) void split_kernel(Rows R) {
    const RowView v = row_view(R);
    const int64_t P = R.P;
    __shared__ uint32_t wcand[kWaves], wabove[kWaves];
    const uint32_t b0 = v.st->b0;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const bool vec = (((uintptr_t)v.x | (uintptr_t)v.xh) & 15) == 0;
    const int64_t q0 = (int64_t)blockIdx.x * (kChunk / 4);
    uint32_t keys[kQuads][4];
    uint32_t ccount = 0, above = 0;
#pragma unroll
    for (int j = 0; j < kQuads; ++j) {
        float d[4];
        const int n = load_quad(v.x, v.xh, q0 + (int64_t)j * kTPB + threadIdx.x, P, vec, d);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const bool in = c < n;
            keys[j][c] = in ? key_of(d[c]) : 0xffffffffu;    // sentinel: never a candidate / above
            const uint32_t dg = keys[j][c] >> kTopShift;
            above += in && dg > b0;
            ccount += in && dg == b0;
        }
    }
    const uint32_t incl = wave_incl_scan(ccount);
    uint32_t ab = above;
    for (int o = 32; o > 0; o >>= 1) ab += __shfl_xor(ab, o, 64);
    if (lane == 63) wcand[wave] = incl;
    if (lane == 0) wabove[wave] = ab;
    __syncthreads();
    uint32_t pos = incl - ccount;
    uint32_t tot = 0, a = 0;
    for (int w = 0; w < kWaves; ++w) {
        pos += (w < wave) ? wcand[w] : 0;
        tot += wcand[w];
        a += wabove[w];
    }
    if (threadIdx.x == 0) {
        v.cnt[4 * blockIdx.x + 0] = a;
        v.cnt[4 * blockIdx.x + 3] = tot;
    }
    const int64_t region = (int64_t)blockIdx.x * kChunk;
#pragma unroll
    for (int j = 0; j < kQuads; ++j) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if ((keys[j][c] >> kTopShift) == b0 && keys[j][c] != 0xffffffffu) {
                v.cidx[region + pos] = 4 * (q0 + (int64_t)j * kTPB + threadIdx.x) + c;
                v.ckey[region + pos] = keys[j][c];
                ++pos;
            }
        }
    }
}

// candidate histogram of `bits` bits at `shift`, restricted to keys matching st->prefix/mask
// one wave per chunk region; the block's LDS histogram is flushed once (few global atomics)
template <int BITS>
__global__ __launch_bounds__(kTPB) void cand_hist(Rows R, int shift) {
    const RowView v = row_view(R);
    constexpr int NB = 1 << BITS;
    __shared__ uint32_t h[NB];
    for (int i = threadIdx.x; i < NB; i += kTPB) h[i] = 0;
    __syncthreads();
    const uint32_t prefix = v.st->prefix, mask = v.st->mask;
    const int64_t nchunks = (R.P + kChunk - 1) / kChunk;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int64_t c = (int64_t)blockIdx.x * kWaves + wave; c < nchunks; c += (int64_t)gridDim.x * kWaves) {
        const int64_t nc = v.cnt[4 * c + 3];
        for (int64_t i = lane; i < nc; i += 64) {
            const uint32_t key = v.ckey[c * kChunk + i];
            if ((key & mask) == prefix) atomicAdd(&h[(key >> shift) & (NB - 1)], 1u);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < NB; i += kTPB)
        if (h[i]) atomicAdd(&v.hist[i], h[i]);
}

template <int BITS>
__global__ __launch_bounds__(kTPB) void select_cand(Rows R, int shift) {
    const RowView v = row_view(R);
    uint32_t* hist = v.hist;
    SelState* st = v.st;
    constexpr int NB = 1 << BITS;
    __shared__ int bin;
    __shared__ int64_t need;
    select_bin<NB>(hist, st->need, &bin, &need);
    __syncthreads();
    if (threadIdx.x == 0) {
        st->prefix |= (uint32_t)bin << shift;
        st->mask |= (uint32_t)(NB - 1) << shift;
        st->need = need;
        if (shift == 0) st->T = st->prefix;
    }
}

// per-chunk counts of candidates strictly above T and equal to T
// one wave per chunk region: counts of candidates > T and == T, written without atomics
__global__ __launch_bounds__(kTPB) void cand_mark(Rows R) {
    const RowView v = row_view(R);
    const uint32_t T = v.st->T;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t nchunks = (R.P + kChunk - 1) / kChunk;
    for (int64_t c = (int64_t)blockIdx.x * kWaves + wave; c < nchunks; c += (int64_t)gridDim.x * kWaves) {
        const int64_t nc = v.cnt[4 * c + 3];
        uint32_t g = 0, e = 0;
        for (int64_t i = lane; i < nc; i += 64) {
            const uint32_t key = v.ckey[c * kChunk + i];
            g += key > T;
            e += key == T;
        }
        for (int o = 32; o > 0; o >>= 1) {
            g += __shfl_xor(g, o, 64);
            e += __shfl_xor(e, o, 64);
        }
        if (lane == 0) {
            v.cnt[4 * c + 1] = g;
            v.cnt[4 * c + 2] = e;
        }
    }
}

// one block: per chunk the output offset and the global tie rank of its first tie
__global__ __launch_bounds__(kScanTPB) void scan_kernel(Rows R) {
    const RowView v = row_view(R);
    const int64_t* cnt = v.cnt;
    const int64_t nchunks = (R.P + kChunk - 1) / kChunk;
    const SelState* st = v.st;
    int64_t* off = v.off;
    __shared__ int64_t wsum_g[kScanTPB / 64], wsum_e[kScanTPB / 64];
    __shared__ int64_t carry_g, carry_e;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t need_eq = st->need;
    if (threadIdx.x == 0) carry_g = carry_e = 0;
    __syncthreads();
    for (int64_t b0 = 0; b0 < nchunks; b0 += kScanTPB) {
        const int64_t b = b0 + threadIdx.x;
        const int64_t g = b < nchunks ? cnt[4 * b] + cnt[4 * b + 1] : 0;   // keys > T
        const int64_t e = b < nchunks ? cnt[4 * b + 2] : 0;                // keys == T
        int64_t sg = g, se = e;                                            // wave inclusive scan
        for (int o = 1; o < 64; o <<= 1) {
            const int64_t tg = __shfl_up(sg, o, 64), te = __shfl_up(se, o, 64);
            if (lane >= o) { sg += tg; se += te; }
        }
        if (lane == 63) { wsum_g[wave] = sg; wsum_e[wave] = se; }
        __syncthreads();
        int64_t pg = carry_g, pe = carry_e;
        for (int w = 0; w < wave; ++w) { pg += wsum_g[w]; pe += wsum_e[w]; }
        if (b < nchunks) {
            const int64_t gt_before = pg + sg - g, eq_before = pe + se - e;
            off[2 * b] = gt_before + (eq_before < need_eq ? eq_before : need_eq);
            off[2 * b + 1] = eq_before;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int w = 0; w < kScanTPB / 64; ++w) { carry_g += wsum_g[w]; carry_e += wsum_e[w]; }
        }
        __syncthreads();
    }
}

// ---- C: stable per-chunk compaction in index order.  In sub-tile j lane l holds elements
// 4(q0 + j*256 + l) .. +3, so index order is lane-major: a wave scan of per-lane counts (0..4)
// plus the per-wave totals in LDS rank every tie and every selected element.
__global__ __launch_bounds__(kTPB) void write_kernel(Rows R) {
    const RowView v = row_view(R);
    const int64_t P = R.P;
    __shared__ uint32_t weq[2][kWaves], wsel[2][kWaves];
    const uint32_t T = v.st->T;
    const int64_t need_eq = v.st->need;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const bool vec = (((uintptr_t)v.x | (uintptr_t)v.xh) & 15) == 0;
    const int64_t q0 = (int64_t)blockIdx.x * (kChunk / 4);
    int64_t run_out = v.off[2 * blockIdx.x], run_eq = v.off[2 * blockIdx.x + 1];
    for (int j = 0; j < kQuads; ++j) {
        const int par = j & 1;
        const int64_t q = q0 + (int64_t)j * kTPB + threadIdx.x;
        float d[4];
        const int n = load_quad(v.x, v.xh, q, P, vec, d);
        uint32_t key[4];
        uint32_t ne = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            key[c] = key_of(d[c]);
            ne += (c < n) && key[c] == T;
        }
        const uint32_t einc = wave_incl_scan(ne);
        if (lane == 63) weq[par][wave] = einc;
        __syncthreads();
        uint32_t epre = 0, etot = 0;
        for (int w = 0; w < kWaves; ++w) {
            epre += (w < wave) ? weq[par][w] : 0;
            etot += weq[par][w];
        }
        int64_t er = run_eq + epre + (einc - ne);
        bool sel[4];
        uint32_t ns = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const bool in = c < n;
            const bool eq = in && key[c] == T;
            sel[c] = in && (key[c] > T || (eq && er < need_eq));
            er += eq;
            ns += sel[c];
        }
        const uint32_t sinc = wave_incl_scan(ns);
        if (lane == 63) wsel[par][wave] = sinc;
        __syncthreads();
        uint32_t spre = 0, stot = 0;
        for (int w = 0; w < kWaves; ++w) {
            spre += (w < wave) ? wsel[par][w] : 0;
            stot += wsel[par][w];
        }
        int64_t pos = run_out + spre + (sinc - ns);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (sel[c]) {
                v.vals[pos] = d[c];
                v.idx[pos] = 4 * q + c;
                ++pos;
            }
        }
        run_out += stot;
        run_eq += etot;
    }
}

// ------------------------------------------------------------------------------- apply
// partner position e: s_r[idx_j] = s_r[idx_j] + f32(alpha) * v_j for rows with degree > e
__global__ __launch_bounds__(kTPB) void scatter_partner_kernel(float* __restrict__ s, int64_t ld,
                                                               const char* __restrict__ msgs,
                                                               int64_t msg_ld, int64_t kpad, int64_t k,
                                                               const int32_t* __restrict__ rec,
                                                               int n_local, int M, int e, float alpha) {
    const int r = blockIdx.y;
    const int32_t* deg = rec + mx::kPlanHeader;
    if (deg[r] <= e) return;
    const int slot = deg[2 * n_local + r * M + e];
    const float* v = reinterpret_cast<const float*>(msgs + (int64_t)slot * msg_ld);
    const int64_t* ix = reinterpret_cast<const int64_t*>(msgs + (int64_t)slot * msg_ld + 4 * kpad);
    float* sr = s + (int64_t)r * ld;
    for (int64_t q = (int64_t)blockIdx.x * kTPB + threadIdx.x; q < k; q += (int64_t)gridDim.x * kTPB) {
        const int64_t c = ix[q];
        sr[c] = __fadd_rn(sr[c], __fmul_rn(alpha, v[q]));
    }
}

// own message: s_r[idx_r] += f32(1 - d alpha) v_r ; x_hat_r[idx_r] += v_r
__global__ __launch_bounds__(kTPB) void scatter_self_kernel(float* __restrict__ s, float* __restrict__ xh,
                                                            int64_t ld, const char* __restrict__ msgs,
                                                            int64_t msg_ld, int64_t kpad, int64_t k,
                                                            const int32_t* __restrict__ rec, int n_local) {
    const int r = blockIdx.y;
    const float sw = __int_as_float(rec[mx::kPlanHeader + n_local + r]);
    const float* v = reinterpret_cast<const float*>(msgs + (int64_t)r * msg_ld);
    const int64_t* ix = reinterpret_cast<const int64_t*>(msgs + (int64_t)r * msg_ld + 4 * kpad);
    float* sr = s + (int64_t)r * ld;
    float* hr = xh + (int64_t)r * ld;
    for (int64_t q = (int64_t)blockIdx.x * kTPB + threadIdx.x; q < k; q += (int64_t)gridDim.x * kTPB) {
        const int64_t c = ix[q];
        const float vq = v[q];
        sr[c] = __fadd_rn(sr[c], __fmul_rn(sw, vq));
        hr[c] = __fadd_rn(hr[c], vq);
    }
}

// x = fma(g, s, x); x = fma(-g, x_hat, x)  (communicator.py:225), 16-byte lanes
__global__ __launch_bounds__(kTPB) void dense_kernel(float* __restrict__ x, const float* __restrict__ s,
                                                     const float* __restrict__ xh, int64_t ld, int64_t P,
                                                     float g) {
    const int r = blockIdx.y;
    float* xr = x + (int64_t)r * ld;
    const float* sr = s + (int64_t)r * ld;
    const float* hr = xh + (int64_t)r * ld;
    const bool vec = (((uintptr_t)xr | (uintptr_t)sr | (uintptr_t)hr) & 15) == 0;
    const int64_t nv = vec ? P / 4 : 0;
    typedef float f4 __attribute__((ext_vector_type(4)));
    for (int64_t q = (int64_t)blockIdx.x * kTPB + threadIdx.x; q < nv; q += (int64_t)gridDim.x * kTPB) {
        f4 a = __builtin_nontemporal_load(reinterpret_cast<const f4*>(xr) + q);
        const f4 b = __builtin_nontemporal_load(reinterpret_cast<const f4*>(sr) + q);
        const f4 c = __builtin_nontemporal_load(reinterpret_cast<const f4*>(hr) + q);
#pragma unroll
        for (int j = 0; j < 4; ++j) a[j] = __builtin_fmaf(-g, c[j], __builtin_fmaf(g, b[j], a[j]));
        __builtin_nontemporal_store(a, reinterpret_cast<f4*>(xr) + q);
    }
    for (int64_t i = nv * 4 + (int64_t)blockIdx.x * kTPB + threadIdx.x; i < P; i += (int64_t)gridDim.x * kTPB)
        xr[i] = __builtin_fmaf(-g, hr[i], __builtin_fmaf(g, sr[i], xr[i]));
}

unsigned clamp_grid(int64_t n, int64_t per, int64_t cap) {
    int64_t g = (n + per - 1) / per;
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    return (unsigned)g;
}
}  // namespace

extern "C" size_t mx_topk_work_bytes(int64_t P) { return layout(P < 1 ? 1 : P).total; }

extern "C" int64_t mx_choco_msg_bytes(int64_t k) { return 4 * ((k + 1) / 2 * 2) + 8 * k; }

extern "C" int mx_topk_abs_diff_rows(const float* x, const float* x_hat, int64_t ld, int nrows, int64_t P,
                                     int64_t k, void* out, int64_t out_ld_bytes, int64_t idx_off_bytes,
                                     void* work, int64_t work_ld_bytes, void* stream) {
    MX_CHECK(x && out && work, "mx_topk_abs_diff_rows: null pointer");
    MX_CHECK(P >= 1 && k >= 1 && k <= P && nrows >= 1 && nrows <= 65535 && (nrows == 1 || ld >= P),
             "mx_topk_abs_diff_rows: P=%lld k=%lld nrows=%d ld=%lld", (long long)P, (long long)k, nrows, (long long)ld);
    MX_CHECK(((uintptr_t)(static_cast<char*>(out) + idx_off_bytes)) % 8 == 0 && (nrows == 1 || out_ld_bytes % 8 == 0),
             "mx_topk_abs_diff_rows: int64 index output must be 8-byte aligned");
    MX_CHECK(work_ld_bytes >= (int64_t)layout(P).total || nrows == 1, "mx_topk_abs_diff_rows: work_ld too small");
    hipStream_t st = mx::as_stream(stream);
    Rows R{x, x_hat, ld, static_cast<char*>(out), out_ld_bytes, idx_off_bytes, static_cast<char*>(work),
           work_ld_bytes, P, k};
    const WorkLayout w = layout(P);
    for (int r = 0; r < nrows; ++r)
        MX_HIP(hipMemsetAsync(static_cast<char*>(work) + (int64_t)r * work_ld_bytes + w.hist, 0,
                              sizeof(uint32_t) * kTopBins, st));
    const unsigned nchunks = (unsigned)((P + kChunk - 1) / kChunk);
    const unsigned hgrid = clamp_grid(P, (int64_t)kTPB * 64, (512 + nrows - 1) / nrows);
    const unsigned cgrid = clamp_grid((P + kChunk - 1) / kChunk, kWaves, (1024 + nrows - 1) / nrows);
    const dim3 one(1, nrows);
    hipLaunchKernelGGL(hist_kernel, dim3(hgrid, nrows), dim3(kTPB), 0, st, R);
    MX_LAUNCH_CHECK();
    hipLaunchKernelGGL(select_top, one, dim3(kTPB), 0, st, R);
    MX_LAUNCH_CHECK();
    hipLaunchKernelGGL(split_kernel, dim3(nchunks, nrows), dim3(kTPB), 0, st, R);
    MX_LAUNCH_CHECK();
    hipLaunchKernelGGL(cand_hist<kMidBits>, dim3(cgrid, nrows), dim3(kTPB), 0, st, R, kMidShift);
    MX_LAUNCH_CHECK();
    hipLaunchKernelGGL(select_cand<kMidBits>, one, dim3(kTPB), 0, st, R, kMidShift);
    MX_LAUNCH_CHECK();
    hipLaunchKernelGGL(cand_hist<kLowBits>, dim3(cgrid, nrows), dim3(kTPB), 0, st, R, 0);
    MX_LAUNCH_CHECK();
    hipLaunchKernelGGL(select_cand<kLowBits>, one, dim3(kTPB), 0, st, R, 0);
    MX_LAUNCH_CHECK();
    hipLaunchKernelGGL(cand_mark, dim3(cgrid, nrows), dim3(kTPB), 0, st, R);
    MX_LAUNCH_CHECK();
    hipLaunchKernelGGL(scan_kernel, one, dim3(kScanTPB), 0, st, R);
    MX_LAUNCH_CHECK();
    hipLaunchKernelGGL(write_kernel, dim3(nchunks, nrows), dim3(kTPB), 0, st, R);
    MX_LAUNCH_CHECK();
    return MX_OK;
}

extern "C" int mx_topk_abs_diff(const float* x, const float* x_hat, int64_t P, int64_t k, float* vals,
                                int64_t* idx, void* work, void* stream) {
    MX_CHECK(vals && idx, "mx_topk_abs_diff: null pointer");
    const int64_t idx_off = reinterpret_cast<char*>(idx) - reinterpret_cast<char*>(vals);
    return mx_topk_abs_diff_rows(x, x_hat, P, 1, P, k, vals, 0, idx_off, work, 0, stream);
}

extern "C" int mx_choco_apply(float* x, float* xhat, float* s, int64_t ld, int64_t P, int64_t k,
                              const void* msgs, int64_t msg_ld_bytes, const int32_t* plan_dev,
                              int64_t iter, int n_local, int M, float alpha, float gamma,
                              void* stream) {
    MX_CHECK(x && xhat && s && msgs && plan_dev, "mx_choco_apply: null pointer");
    MX_CHECK(P >= 1 && k >= 1 && k <= P && ld >= P, "mx_choco_apply: P=%lld k=%lld ld=%lld",
             (long long)P, (long long)k, (long long)ld);
    MX_CHECK(n_local >= 1 && n_local <= 65535 && M >= 1, "mx_choco_apply: n_local=%d M=%d", n_local, M);
    const int64_t kpad = (k + 1) / 2 * 2;
    MX_CHECK(msg_ld_bytes >= 4 * kpad + 8 * k && msg_ld_bytes % 8 == 0, "mx_choco_apply: msg_ld %lld",
             (long long)msg_ld_bytes);
    hipStream_t st = mx::as_stream(stream);
    const int32_t* rec = plan_dev + iter * mx::plan_words(n_local, M);
    const unsigned sgrid = clamp_grid(k, kTPB * 4, 1024);
    for (int e = 0; e < M; ++e) {
        hipLaunchKernelGGL(scatter_partner_kernel, dim3(sgrid, n_local), dim3(kTPB), 0, st, s, ld,
                           static_cast<const char*>(msgs), msg_ld_bytes, kpad, k, rec, n_local, M, e, alpha);
        MX_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(scatter_self_kernel, dim3(sgrid, n_local), dim3(kTPB), 0, st, s, xhat, ld,
                       static_cast<const char*>(msgs), msg_ld_bytes, kpad, k, rec, n_local);
    MX_LAUNCH_CHECK();
    const unsigned dgrid = clamp_grid(P, kTPB * 16, 2048);
    hipLaunchKernelGGL(dense_kernel, dim3(dgrid, n_local), dim3(kTPB), 0, st, x, (const float*)s,
                       (const float*)xhat, ld, P, gamma);
    MX_LAUNCH_CHECK();
    return MX_OK;
}
