// flags.hip -- MATCHA activation flags on the GPU, bit-exact with numpy's legacy global RNG.
//
// Replaces MatchaProcessor.set_flags (graph_manager.py:298-309):
//     flags.append(np.random.binomial(1, p[i], iterations))  for each matching i,
// and the discarded np.random.binomial of FixedProcessor.set_flags (graph_manager.py:213).
//
// numpy's RandomState draws binomial(1, p) with legacy_random_binomial_inversion
// (numpy 2.2.6, legacy-distributions.c): one 53-bit double U per draw (two MT19937 words),
// X = 0; px = qn = exp(log(1 - p')); while (U > px) { X++; if (X > 1) { X = 0; px = qn; redraw }
// else { U -= px; px = p' * qn / q } }, with p' = p for p <= 0.5 and 1 - p (result flipped)
// otherwise.  A redraw ("resample") happens only when U > qn + p'qn/q, i.e. in the last ulps
// below 1 -- so the GPU path is:
//   1. mt_stream_kernel  one workgroup regenerates the MT19937 word stream block by block
//                        (624-word twist split in three dependency phases, 624 lanes),
//                        keeping every raw state block so the final state can be handed back;
//   2. draw_kernel       one lane per draw, assuming two words per draw, flags a resample;
//   3. draw_seq_kernel   only if a resample was flagged (or forced): one lane walks the stream
//                        sequentially with the redraw rule.  Same words, same answer.
// qn and p'qn/q are computed on the host with the same libm numpy uses (glibc exp/log).
#include <math.h>
#include <vector>

#include "mx_common.h"

namespace {
constexpr int kN = 624;
constexpr int kM = 397;
constexpr uint32_t kUpper = 0x80000000u, kLower = 0x7fffffffu, kMatrix = 0x9908b0dfu;

__device__ __forceinline__ uint32_t temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

__device__ __forceinline__ uint32_t twist_one(uint32_t cur, uint32_t next, uint32_t far) {
    uint32_t y = (cur & kUpper) | (next & kLower);
    return far ^ (y >> 1) ^ ((y & 1u) ? kMatrix : 0u);
}

// raw[b][624] = state block b (block 0 = key0); words[w] = tempered word at stream position
// pos0 + w, for w in [0, nwords).
__global__ __launch_bounds__(1024) void mt_stream_kernel(const uint32_t* __restrict__ key0, int pos0,
                                                         int64_t nblocks, int64_t nwords,
                                                         uint32_t* __restrict__ raw,
                                                         uint32_t* __restrict__ words) {
    __shared__ uint32_t buf[2][kN];
    const int i = threadIdx.x;
    if (i < kN) buf[0][i] = key0[i];
    __syncthreads();
    int cur = 0;
    for (int64_t b = 0; b < nblocks; ++b) {
        if (b > 0) {
            const uint32_t* o = buf[cur];
            uint32_t* nw = buf[cur ^ 1];
            // in-place sequential twist: index i reads old[i], old[i+1] and, for i >= 227, the
            // NEW value at i-227; i = 623 reads new[0].  Three phases respect those edges.
            if (i < kN - kM) nw[i] = twist_one(o[i], o[i + 1], o[i + kM]);
            __syncthreads();
            if (i >= kN - kM && i < 2 * (kN - kM)) nw[i] = twist_one(o[i], o[i + 1], nw[i - (kN - kM)]);
            __syncthreads();
            if (i >= 2 * (kN - kM) && i < kN - 1) nw[i] = twist_one(o[i], o[i + 1], nw[i - (kN - kM)]);
            if (i == kN - 1) nw[i] = twist_one(o[i], nw[0], nw[kM - 1]);
            __syncthreads();
            cur ^= 1;
        }
        if (i < kN) {
            const uint32_t v = buf[cur][i];
            raw[b * kN + i] = v;
            const int64_t w = b * kN + i - pos0;
            if (w >= 0 && w < nwords) words[w] = temper(v);
        }
        __syncthreads();
    }
}

__device__ __forceinline__ double legacy_double(const uint32_t* w) {
    const int32_t a = (int32_t)(w[0] >> 5), b = (int32_t)(w[1] >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
}

// draw d = m * T + t (matching-major, as set_flags loops), output flags[t][m]
__global__ __launch_bounds__(256) void draw_kernel(const uint32_t* __restrict__ words,
                                                   const mx::BinomParam* __restrict__ prm, int M,
                                                   int64_t T, uint8_t* __restrict__ flags,
                                                   int* __restrict__ resample) {
    const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= (int64_t)M * T) return;
    const int m = (int)(d / T);
    const int64_t t = d - (int64_t)m * T;
    const mx::BinomParam q = prm[m];
    double U = legacy_double(words + 2 * d);
    int X = 0;
    if (U > q.qn) {
        U -= q.qn;
        if (U > q.px1) atomicOr(resample, 1);   // the redraw branch: handled sequentially
        X = 1;
    }
    flags[t * M + m] = (uint8_t)(q.flip ? 1 - X : X);
}

__global__ void draw_seq_kernel(const uint32_t* __restrict__ words, int64_t nwords,
                                const mx::BinomParam* __restrict__ prm, int M, int64_t T,
                                uint8_t* __restrict__ flags, int64_t* __restrict__ consumed,
                                int* __restrict__ overflow) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    int64_t w = 0;
    for (int m = 0; m < M; ++m) {
        const mx::BinomParam q = prm[m];
        for (int64_t t = 0; t < T; ++t) {
            if (w + 2 > nwords) { *overflow = 1; *consumed = w; return; }
            double U = legacy_double(words + w);
            w += 2;
            int X = 0;
            double px = q.qn;
            while (U > px) {
                X++;
                if (X > 1) {
                    X = 0;
                    px = q.qn;
                    if (w + 2 > nwords) { *overflow = 1; *consumed = w; return; }
                    U = legacy_double(words + w);
                    w += 2;
                } else {
                    U -= px;
                    px = q.px1;
                }
            }
            flags[t * M + m] = (uint8_t)(q.flip ? 1 - X : X);
        }
    }
    *consumed = w;
    *overflow = 0;
}

// Host side of legacy_random_binomial_original / _inversion for n = 1 (numpy 2.2.6).
mx::BinomParam binom_param(double p) {
    mx::BinomParam r{};
    double pp = p;
    r.flip = 0;
    if (!(p <= 0.5)) {
        pp = 1.0 - p;
        r.flip = 1;
    }
    const double q = 1.0 - pp;
    volatile double lq = log(q);            // volatile: keep the libm calls, no folding
    const double qn = exp(1.0 * lq);
    r.qn = qn;
    const double num = (1.0 * pp) * qn;
    r.px1 = num / (1.0 * q);
    return r;
}

struct DevBuf {
    void* p = nullptr;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

int flags_impl(const uint32_t* key_in, int pos_in, const double* p, int M, int64_t T,
               uint8_t* flags_dev, uint32_t* key_out, int* pos_out, void* stream_v, bool force_seq) {
    MX_CHECK(key_in && key_out && pos_out && p, "mx_flags_binomial: null pointer");
    MX_CHECK(M >= 1 && T >= 0, "mx_flags_binomial: M=%d T=%lld", M, (long long)T);
    MX_CHECK(pos_in >= 0 && pos_in <= kN, "mx_flags_binomial: pos %d out of [0, 624]", pos_in);
    MX_CHECK(T == 0 || flags_dev, "mx_flags_binomial: null flags");
    hipStream_t st = mx::as_stream(stream_v);
    std::vector<mx::BinomParam> prm(M);
    for (int m = 0; m < M; ++m) {
        double pm = p[m];
        if (isnan(pm) || pm < 0) pm = 0;      // graph_manager.py:305-306
        MX_CHECK(pm <= 1.0, "mx_flags_binomial: p[%d] = %g > 1", m, pm);
        prm[m] = binom_param(pm);
    }
    const int64_t D = (int64_t)M * T;
    if (D == 0) {
        memcpy(key_out, key_in, sizeof(uint32_t) * kN);
        *pos_out = pos_in;
        return MX_OK;
    }
    const int64_t nwords = 2 * D + 2 * kN;               // margin: 624 redraws
    const int64_t nblocks = (pos_in + nwords - 1) / kN + 1;
    DevBuf raw, words, dprm, dkey, dint;
    MX_HIP(hipMalloc(&raw.p, sizeof(uint32_t) * nblocks * kN));
    MX_HIP(hipMalloc(&words.p, sizeof(uint32_t) * nwords));
    MX_HIP(hipMalloc(&dprm.p, sizeof(mx::BinomParam) * M));
    MX_HIP(hipMalloc(&dkey.p, sizeof(uint32_t) * kN));
    MX_HIP(hipMalloc(&dint.p, 4 * sizeof(int64_t)));
    MX_HIP(hipMemcpyAsync(dkey.p, key_in, sizeof(uint32_t) * kN, hipMemcpyHostToDevice, st));
    MX_HIP(hipMemcpyAsync(dprm.p, prm.data(), sizeof(mx::BinomParam) * M, hipMemcpyHostToDevice, st));
    MX_HIP(hipMemsetAsync(dint.p, 0, 4 * sizeof(int64_t), st));
    int64_t* consumed_d = (int64_t*)dint.p;
    int* resample_d = (int*)((int64_t*)dint.p + 1);
    int* overflow_d = (int*)((int64_t*)dint.p + 2);

    hipLaunchKernelGGL(mt_stream_kernel, dim3(1), dim3(1024), 0, st, (const uint32_t*)dkey.p,
                       pos_in, nblocks, nwords, (uint32_t*)raw.p, (uint32_t*)words.p);
    MX_LAUNCH_CHECK();
    int resample = 0;
    if (!force_seq) {
        const int64_t grid = (D + 255) / 256;
        hipLaunchKernelGGL(draw_kernel, dim3((unsigned)grid), dim3(256), 0, st,
                           (const uint32_t*)words.p, (const mx::BinomParam*)dprm.p, M, T,
                           flags_dev, resample_d);
        MX_LAUNCH_CHECK();
        MX_HIP(hipMemcpyAsync(&resample, resample_d, sizeof(int), hipMemcpyDeviceToHost, st));
        MX_HIP(hipStreamSynchronize(st));
    }
    int64_t consumed = 2 * D;
    if (resample || force_seq) {
        hipLaunchKernelGGL(draw_seq_kernel, dim3(1), dim3(64), 0, st, (const uint32_t*)words.p,
                           nwords, (const mx::BinomParam*)dprm.p, M, T, flags_dev, consumed_d,
                           overflow_d);
        MX_LAUNCH_CHECK();
        int overflow = 0;
        MX_HIP(hipMemcpyAsync(&consumed, consumed_d, sizeof(int64_t), hipMemcpyDeviceToHost, st));
        MX_HIP(hipMemcpyAsync(&overflow, overflow_d, sizeof(int), hipMemcpyDeviceToHost, st));
        MX_HIP(hipStreamSynchronize(st));
        if (overflow) {
            mx::set_error("mx_flags_binomial: MT19937 stream margin exhausted by redraws");
            return MX_ERR_RNG;
        }
    }
    // final state: the raw block holding the last consumed word, pos just past it
    const int64_t last = pos_in + consumed - 1;
    const int64_t b = last / kN;
    MX_HIP(hipMemcpyAsync(key_out, (uint32_t*)raw.p + b * kN, sizeof(uint32_t) * kN,
                          hipMemcpyDeviceToHost, st));
    MX_HIP(hipStreamSynchronize(st));
    *pos_out = (int)(last % kN) + 1;
    return MX_OK;
}
}  // namespace

extern "C" int mx_flags_binomial(const uint32_t* key_in, int pos_in, const double* p, int M,
                                 int64_t T, uint8_t* flags_dev, uint32_t* key_out, int* pos_out,
                                 void* stream) {
    return flags_impl(key_in, pos_in, p, M, T, flags_dev, key_out, pos_out, stream, false);
}

extern "C" int mx_flags_binomial_sequential(const uint32_t* key_in, int pos_in, const double* p,
                                            int M, int64_t T, uint8_t* flags_dev,
                                            uint32_t* key_out, int* pos_out, void* stream) {
    return flags_impl(key_in, pos_in, p, M, T, flags_dev, key_out, pos_out, stream, true);
}
