// choco.hip -- ChocoSGD compressed gossip on the GPU.
//
// mx_topk_abs_diff  = compressors.get_top_k (compressors.py:3-19) applied to
//                     send = x - x_hat (ChocoCommunicator.prepare_comm_buffer, communicator.py:188-190)
// mx_choco_apply    = ChocoCommunicator.averaging (communicator.py:200-230)
//
// Top-k is a 3-digit MSB radix select on the 31-bit magnitude key bits(|x - x_hat|) (non-negative
// floats order like their bit patterns): digits of 11/11/10 bits, one streaming histogram pass
// per digit (LDS histograms, non-zero bins flushed with global atomics), a one-block select
// kernel that walks the histogram from the top to find the digit holding the k-th largest key,
// then a two-pass stable compaction (per-chunk counts -> one-block scan -> per-chunk write) that
// emits every key above the threshold plus the lowest-index keys equal to it, in index order.
// Everything stays on the device; no host round trip between passes.
#include "mx_common.h"

namespace {
constexpr int kTPB = 256;
constexpr int kBins = 2048;
constexpr int kChunk = 4096;                 // elements per compaction chunk (16 per lane)
constexpr int kPerLane = kChunk / kTPB;

struct SelState {
    uint32_t prefix;    // key bits fixed so far
    uint32_t mask;      // which bits of the key are fixed
    int64_t k_rem;      // elements still to take at/below the current prefix
    int64_t n_gt;       // elements strictly above the current prefix's bucket range
};

__device__ __forceinline__ uint32_t key_at(const float* x, const float* xh, int64_t i) {
    const float d = xh ? __fsub_rn(x[i], xh[i]) : x[i];
    return __float_as_uint(d) & 0x7fffffffu;
}

// digit geometry: pass 0 -> bits [21,32), pass 1 -> [10,21), pass 2 -> [0,10)
__device__ __forceinline__ int dshift(int pass) { return pass == 0 ? 21 : (pass == 1 ? 10 : 0); }

__global__ __launch_bounds__(kTPB) void hist_kernel(const float* __restrict__ x,
                                                    const float* __restrict__ xh, int64_t P,
                                                    const SelState* __restrict__ st, int pass,
                                                    uint32_t* __restrict__ ghist) {
    __shared__ uint32_t h[kBins];
    for (int i = threadIdx.x; i < kBins; i += kTPB) h[i] = 0;
    __syncthreads();
    const uint32_t prefix = st->prefix, mask = st->mask;
    const int sh = dshift(pass);
    for (int64_t i = (int64_t)blockIdx.x * kTPB + threadIdx.x; i < P; i += (int64_t)gridDim.x * kTPB) {
        const uint32_t key = key_at(x, xh, i);
        if ((key & mask) == prefix) atomicAdd(&h[(key >> sh) & (kBins - 1)], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kBins; i += kTPB)
        if (h[i]) atomicAdd(&ghist[i], h[i]);
}

// one block: find the digit value holding the k_rem-th largest key among the candidates
__global__ __launch_bounds__(kTPB) void select_kernel(uint32_t* __restrict__ ghist,
                                                      SelState* __restrict__ st, int pass) {
    constexpr int kPer = kBins / kTPB;         // 8 bins per lane, lane 0 holds the TOP bins
    __shared__ int64_t part[kTPB];
    const int t = threadIdx.x;
    int64_t mine = 0;
    for (int j = 0; j < kPer; ++j) mine += ghist[kBins - 1 - (t * kPer + j)];
    part[t] = mine;
    __syncthreads();
    // inclusive scan over lanes (counts from the top)
    for (int off = 1; off < kTPB; off <<= 1) {
        int64_t v = (t >= off) ? part[t - off] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    const int64_t k_rem = st->k_rem;
    const int64_t before = part[t] - mine;     // candidates in higher bins than this lane's
    __syncthreads();
    if (before < k_rem && part[t] >= k_rem) {
        int64_t acc = before;
        for (int j = 0; j < kPer; ++j) {
            const int bin = kBins - 1 - (t * kPer + j);
            const int64_t c = ghist[bin];
            if (acc + c >= k_rem) {
                const int sh = dshift(pass);
                const uint32_t width_mask = (pass == 2) ? 0x3ffu : 0x7ffu;
                st->prefix |= ((uint32_t)bin & width_mask) << sh;
                st->mask |= width_mask << sh;
                st->n_gt += acc;
                st->k_rem = k_rem - acc;
                break;
            }
            acc += c;
        }
    }
    __syncthreads();
    for (int i = t; i < kBins; i += kTPB) ghist[i] = 0;   // ready for the next pass
}

// per-chunk counts of keys > threshold and == threshold
__global__ __launch_bounds__(kTPB) void count_kernel(const float* __restrict__ x,
                                                     const float* __restrict__ xh, int64_t P,
                                                     const SelState* __restrict__ st,
                                                     int64_t* __restrict__ cnt) {
    __shared__ int64_t red[2][kTPB];
    const uint32_t T = st->prefix;
    const int64_t base = (int64_t)blockIdx.x * kChunk;
    int64_t gt = 0, eq = 0;
    for (int j = 0; j < kPerLane; ++j) {
        const int64_t i = base + (int64_t)j * kTPB + threadIdx.x;
        if (i < P) {
            const uint32_t key = key_at(x, xh, i);
            gt += key > T;
            eq += key == T;
        }
    }
    red[0][threadIdx.x] = gt;
    red[1][threadIdx.x] = eq;
    __syncthreads();
    for (int off = kTPB / 2; off > 0; off >>= 1) {
        if (threadIdx.x < off) {
            red[0][threadIdx.x] += red[0][threadIdx.x + off];
            red[1][threadIdx.x] += red[1][threadIdx.x + off];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        cnt[2 * blockIdx.x] = red[0][0];
        cnt[2 * blockIdx.x + 1] = red[1][0];
    }
}

// one block: exclusive scan of chunk counts -> (output offset, equal-rank offset) per chunk
__global__ __launch_bounds__(kTPB) void scan_kernel(const int64_t* __restrict__ cnt, int64_t nchunks,
                                                    const SelState* __restrict__ st,
                                                    int64_t* __restrict__ off) {
    __shared__ int64_t s_gt[kTPB], s_eq[kTPB];
    __shared__ int64_t carry_gt, carry_eq;
    const int64_t need_eq = st->k_rem;
    if (threadIdx.x == 0) { carry_gt = 0; carry_eq = 0; }
    __syncthreads();
    for (int64_t b0 = 0; b0 < nchunks; b0 += kTPB) {
        const int64_t b = b0 + threadIdx.x;
        const int64_t g = b < nchunks ? cnt[2 * b] : 0;
        const int64_t e = b < nchunks ? cnt[2 * b + 1] : 0;
        s_gt[threadIdx.x] = g;
        s_eq[threadIdx.x] = e;
        __syncthreads();
        for (int o = 1; o < kTPB; o <<= 1) {
            int64_t vg = threadIdx.x >= o ? s_gt[threadIdx.x - o] : 0;
            int64_t ve = threadIdx.x >= o ? s_eq[threadIdx.x - o] : 0;
            __syncthreads();
            s_gt[threadIdx.x] += vg;
            s_eq[threadIdx.x] += ve;
            __syncthreads();
        }
        if (b < nchunks) {
            const int64_t eq_before = carry_eq + s_eq[threadIdx.x] - e;
            const int64_t gt_before = carry_gt + s_gt[threadIdx.x] - g;
            int64_t eq_taken_before = eq_before < need_eq ? eq_before : need_eq;
            off[2 * b] = gt_before + eq_taken_before;   // output offset of this chunk
            off[2 * b + 1] = eq_before;                 // global equal-rank of its first tie
        }
        __syncthreads();
        if (threadIdx.x == kTPB - 1) {
            carry_gt += s_gt[kTPB - 1];
            carry_eq += s_eq[kTPB - 1];
        }
        __syncthreads();
    }
}

// per chunk: stable write of the selected (index, value) pairs in index order
__global__ __launch_bounds__(kTPB) void write_kernel(const float* __restrict__ x,
                                                     const float* __restrict__ xh, int64_t P,
                                                     const SelState* __restrict__ st,
                                                     const int64_t* __restrict__ off,
                                                     float* __restrict__ vals, int64_t* __restrict__ idx) {
    __shared__ int s_sel[kTPB], s_eq[kTPB];
    __shared__ int64_t run_out, run_eq;
    const uint32_t T = st->prefix;
    const int64_t need_eq = st->k_rem;
    const int64_t base = (int64_t)blockIdx.x * kChunk;
    if (threadIdx.x == 0) {
        run_out = off[2 * blockIdx.x];
        run_eq = off[2 * blockIdx.x + 1];
    }
    __syncthreads();
    for (int j = 0; j < kPerLane; ++j) {                  // sub-tiles in index order
        const int64_t i = base + (int64_t)j * kTPB + threadIdx.x;
        uint32_t key = 0;
        float d = 0.0f;
        bool in = i < P;
        if (in) {
            d = xh ? __fsub_rn(x[i], xh[i]) : x[i];
            key = __float_as_uint(d) & 0x7fffffffu;
        }
        const int is_eq = in && key == T;
        s_eq[threadIdx.x] = is_eq;
        __syncthreads();
        for (int o = 1; o < kTPB; o <<= 1) {              // inclusive scan of ties
            int v = threadIdx.x >= o ? s_eq[threadIdx.x - o] : 0;
            __syncthreads();
            s_eq[threadIdx.x] += v;
            __syncthreads();
        }
        const int64_t eq_rank = run_eq + s_eq[threadIdx.x] - is_eq;
        const int sel = in && (key > T || (is_eq && eq_rank < need_eq));
        s_sel[threadIdx.x] = sel;
        __syncthreads();
        for (int o = 1; o < kTPB; o <<= 1) {
            int v = threadIdx.x >= o ? s_sel[threadIdx.x - o] : 0;
            __syncthreads();
            s_sel[threadIdx.x] += v;
            __syncthreads();
        }
        if (sel) {
            const int64_t pos = run_out + s_sel[threadIdx.x] - 1;
            vals[pos] = d;
            idx[pos] = i;
        }
        __syncthreads();
        if (threadIdx.x == kTPB - 1) {
            run_out += s_sel[kTPB - 1];
            run_eq += s_eq[kTPB - 1];
        }
        __syncthreads();
    }
}

__global__ void init_state_kernel(SelState* st, int64_t k) {
    st->prefix = 0;
    st->mask = 0x80000000u;   // sign bit is always 0 in the key
    st->k_rem = k;
    st->n_gt = 0;
}

struct WorkLayout {
    size_t hist, state, cnt, off, total;
};

WorkLayout layout(int64_t P) {
    const int64_t nchunks = (P + kChunk - 1) / kChunk;
    WorkLayout w;
    w.hist = 0;
    w.state = w.hist + sizeof(uint32_t) * kBins;
    w.cnt = w.state + 64;
    w.off = w.cnt + sizeof(int64_t) * 2 * (size_t)nchunks;
    w.total = w.off + sizeof(int64_t) * 2 * (size_t)nchunks;
    return w;
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
    for (int64_t q = (int64_t)blockIdx.x * kTPB + threadIdx.x; q < nv; q += (int64_t)gridDim.x * kTPB) {
        float4 a = reinterpret_cast<float4*>(xr)[q];
        const float4 b = reinterpret_cast<const float4*>(sr)[q];
        const float4 c = reinterpret_cast<const float4*>(hr)[q];
        a.x = __builtin_fmaf(-g, c.x, __builtin_fmaf(g, b.x, a.x));
        a.y = __builtin_fmaf(-g, c.y, __builtin_fmaf(g, b.y, a.y));
        a.z = __builtin_fmaf(-g, c.z, __builtin_fmaf(g, b.z, a.z));
        a.w = __builtin_fmaf(-g, c.w, __builtin_fmaf(g, b.w, a.w));
        reinterpret_cast<float4*>(xr)[q] = a;
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

extern "C" int mx_topk_abs_diff(const float* x, const float* x_hat, int64_t P, int64_t k, float* vals,
                                int64_t* idx, void* work, void* stream) {
    MX_CHECK(x && vals && idx && work, "mx_topk_abs_diff: null pointer");
    MX_CHECK(P >= 1 && k >= 1 && k <= P, "mx_topk_abs_diff: P=%lld k=%lld", (long long)P, (long long)k);
    hipStream_t st = mx::as_stream(stream);
    const WorkLayout w = layout(P);
    char* base = static_cast<char*>(work);
    uint32_t* hist = reinterpret_cast<uint32_t*>(base + w.hist);
    SelState* sst = reinterpret_cast<SelState*>(base + w.state);
    int64_t* cnt = reinterpret_cast<int64_t*>(base + w.cnt);
    int64_t* off = reinterpret_cast<int64_t*>(base + w.off);
    const int64_t nchunks = (P + kChunk - 1) / kChunk;
    MX_HIP(hipMemsetAsync(hist, 0, sizeof(uint32_t) * kBins, st));
    hipLaunchKernelGGL(init_state_kernel, dim3(1), dim3(1), 0, st, sst, k);
    MX_LAUNCH_CHECK();
    const unsigned hgrid = clamp_grid(P, kTPB * 16, 2048);
    for (int pass = 0; pass < 3; ++pass) {
        hipLaunchKernelGGL(hist_kernel, dim3(hgrid), dim3(kTPB), 0, st, x, x_hat, P,
                           (const SelState*)sst, pass, hist);
        MX_LAUNCH_CHECK();
        hipLaunchKernelGGL(select_kernel, dim3(1), dim3(kTPB), 0, st, hist, sst, pass);
        MX_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(count_kernel, dim3((unsigned)nchunks), dim3(kTPB), 0, st, x, x_hat, P,
                       (const SelState*)sst, cnt);
    MX_LAUNCH_CHECK();
    hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(kTPB), 0, st, (const int64_t*)cnt, nchunks,
                       (const SelState*)sst, off);
    MX_LAUNCH_CHECK();
    hipLaunchKernelGGL(write_kernel, dim3((unsigned)nchunks), dim3(kTPB), 0, st, x, x_hat, P,
                       (const SelState*)sst, (const int64_t*)off, vals, idx);
    MX_LAUNCH_CHECK();
    return MX_OK;
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
