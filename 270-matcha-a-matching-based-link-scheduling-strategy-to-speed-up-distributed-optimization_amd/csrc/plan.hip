// plan.hip -- per-iteration round plans, built on the GPU from the device-resident flag table.
//
// Restates the neighbour walk of decenCommunicator.averaging (communicator.py:99-117) once per
// iteration, for all iterations in parallel (one lane per iteration):
//     for graph_id, flag in enumerate(active_flags):              # ascending matchings
//         if flag and neighbors_info[graph_id][rank] != -1: degree += 1; use that partner
//     selfweight = 1 - degree * alpha
// For each local row the record lists its partners' slots in matching order, so the mixing
// kernel reproduces the reference's FMA order exactly.  Partners owned by another rank get one
// receive-slab slot per distinct worker, numbered by first appearance in (matching asc, sender
// id asc) order -- the order in which mx_exchange_round (exchange.cpp) posts its RCCL receives.
// A remote worker that partners several local rows in one round (different matchings) is
// received ONCE and its slot is shared: its row crosses the link once per round, not once per
// edge.
#include "mx_common.h"

namespace {
constexpr int kMaxRemote = 156;                // the mixing kernels take at most 156 slots

__global__ __launch_bounds__(256) void plan_kernel(const uint8_t* __restrict__ flags, int64_t T,
                                                   int M, const int32_t* __restrict__ partner,
                                                   int n, int row_base, int n_local, double alpha,
                                                   int32_t* __restrict__ plan, int32_t* __restrict__ any_overflow) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    const int64_t W = mx::plan_words(n_local, M);
    int32_t* rec = plan + t * W;
    const uint8_t* f = flags + t * M;
    int32_t* deg = rec + mx::kPlanHeader;
    int32_t* sw = deg + n_local;
    int32_t* src = sw + n_local;
    for (int r = 0; r < n_local; ++r) deg[r] = 0;
    int any = 0, remote = 0, overflow = 0;
    int32_t who[kMaxRemote];                   // slab slot -> remote worker (first appearance)
    for (int g = 0; g < M; ++g) {
        if (!f[g]) continue;
        any = 1;
        for (int p = 0; p < n; ++p) {          // p = sender, ascending
            const int q = partner[g * n + p];  // receiver
            if (q < row_base || q >= row_base + n_local) continue;
            const int r = q - row_base;
            const bool p_local = (p >= row_base && p < row_base + n_local);
            int slot;
            if (p_local) {
                slot = p - row_base;
            } else {
                int k = 0;
                while (k < remote && who[k] != p) ++k;
                if (k == remote) {
                    if (remote == kMaxRemote) {    // more distinct remote partners than any kernel
                        overflow = 1;              // takes: flagged in word [3], row left out
                        continue;
                    }
                    who[remote++] = p;
                }
                slot = n_local + k;
            }
            src[r * M + deg[r]] = slot;
            deg[r] += 1;
        }
    }
    rec[0] = any;
    rec[1] = remote;
    rec[2] = 0;                                // idle rows skipped, local receive slots (mode bits)
    rec[3] = overflow;
    if (overflow) atomicOr(any_overflow, 1);   // read back by mx_plan_build
    for (int r = 0; r < n_local; ++r) {
        const double s = 1.0 - (double)deg[r] * alpha;  // Python float arithmetic, then f32
        const float s32 = (float)s;
        sw[r] = __float_as_int(s32);
    }
}
}  // namespace

namespace {
// word [2] of a record: bit 0 = idle-row mode (mx_plan_set_idle), bit 1 = receive slots are peer
// GPUs' IPC-mapped memory (mx_plan_set_peer_reads); `bit` selects which one is set to `on`
__global__ void mode_kernel(int32_t* __restrict__ plan, int64_t T, int64_t W, int32_t bit, int32_t on) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < T) plan[t * W + 2] = (plan[t * W + 2] & ~bit) | (on ? bit : 0);
}

int set_mode_bit(int32_t* plan_dev, int64_t T, int n_local, int M, int32_t bit, int on, void* stream) {
    if (T == 0) return MX_OK;
    hipLaunchKernelGGL(mode_kernel, dim3((unsigned)((T + 255) / 256)), dim3(256), 0, mx::as_stream(stream),
                       plan_dev, T, mx::plan_words(n_local, M), bit, (int32_t)on);
    MX_LAUNCH_CHECK();
    return MX_OK;
}
}  // namespace

extern "C" int64_t mx_plan_words(int n_local, int M) { return mx::plan_words(n_local, M); }

extern "C" int mx_plan_set_idle(int32_t* plan_dev, int64_t T, int n_local, int M, int mode, void* stream) {
    MX_CHECK(plan_dev && T >= 0 && n_local >= 1 && M >= 1, "mx_plan_set_idle: bad arguments");
    MX_CHECK(mode == 0 || mode == 1, "mx_plan_set_idle: mode %d", mode);
    return set_mode_bit(plan_dev, T, n_local, M, 1, mode, stream);
}

extern "C" int mx_plan_set_peer_reads(int32_t* plan_dev, int64_t T, int n_local, int M, int on, void* stream) {
    MX_CHECK(plan_dev && T >= 0 && n_local >= 1 && M >= 1, "mx_plan_set_peer_reads: bad arguments");
    MX_CHECK(on == 0 || on == 1, "mx_plan_set_peer_reads: on %d", on);
    return set_mode_bit(plan_dev, T, n_local, M, 2, on, stream);
}

extern "C" int mx_plan_build(const uint8_t* flags_dev, int64_t T, int M, const int32_t* partner_dev,
                             int n_global, const int32_t* owner_dev, int my_rank, int row_base,
                             int n_local, double alpha, int32_t* plan_dev, void* stream) {
    (void)owner_dev;  // local rows are the contiguous block [row_base, row_base + n_local)
    (void)my_rank;
    MX_CHECK(flags_dev && partner_dev && plan_dev, "mx_plan_build: null pointer");
    MX_CHECK(M >= 1 && T >= 0 && n_global >= 1, "mx_plan_build: M=%d T=%lld n=%d", M, (long long)T, n_global);
    MX_CHECK(n_local >= 1 && row_base >= 0 && row_base + n_local <= n_global,
             "mx_plan_build: local block [%d, %d) outside [0, %d)", row_base, row_base + n_local, n_global);
    if (T == 0) return MX_OK;
    const int64_t grid = (T + 255) / 256;
    hipStream_t st = mx::as_stream(stream);
    int32_t* ovf = nullptr;                    // one word: did any iteration overflow kMaxRemote?
    MX_HIP(hipMalloc(&ovf, sizeof(int32_t)));
    int32_t host_ovf = 0;
    hipError_t e = hipMemsetAsync(ovf, 0, sizeof(int32_t), st);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(plan_kernel, dim3((unsigned)grid), dim3(256), 0, st, flags_dev, T, M, partner_dev,
                           n_global, row_base, n_local, alpha, plan_dev, ovf);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(&host_ovf, ovf, sizeof(int32_t), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFree(ovf);
    if (e != hipSuccess) {
        mx::set_error("mx_plan_build: %s", hipGetErrorString(e));
        return MX_ERR_HIP;
    }
    MX_CHECK(!host_ovf, "mx_plan_build: a round has more than %d distinct remote partners for the block "
             "[%d, %d) -- more than any mixing kernel takes; spread the workers over more GPUs",
             kMaxRemote, row_base, row_base + n_local);
    return MX_OK;
}
