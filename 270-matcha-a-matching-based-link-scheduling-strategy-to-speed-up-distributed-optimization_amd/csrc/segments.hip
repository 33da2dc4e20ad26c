// segments.hip -- multi-tensor flatten / unflatten and the synthetic-input generator.
//
// mx_gather  = comm_helpers.flatten_tensors (comm_helpers.py:12-30): torch.cat of T tensors.
// mx_scatter = reset_model's `t.copy_(f)` over unflatten_tensors views
//              (communicator.py:124-131, comm_helpers.py:33-56).
// One launch moves every tensor: 1024-element tiles of the flat index space, the owning tensor
// found once per tile by binary search over the offset table and then walked forward, so small
// tensors (biases) share tiles.  Not on the per-round path when the mixing kernel reads tensors
// in place; used by flatten_tensors on device tensors and by host-staged models.
#include "mx_common.h"

namespace {
constexpr int kTPB = 256;
constexpr int kPer = 4;  // elements per lane per tile
constexpr int64_t kTile = (int64_t)kTPB * kPer;

__device__ __forceinline__ int find_seg(const int64_t* off, int nseg, int64_t i) {
    int lo = 0, hi = nseg;  // largest s with off[s] <= i
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (off[mid] <= i) lo = mid; else hi = mid;
    }
    return lo;
}

template <bool kGather>
__global__ __launch_bounds__(kTPB) void seg_copy_kernel(float* const* __restrict__ ptrs,
                                                        const int64_t* __restrict__ off, int nseg,
                                                        int64_t total, float* __restrict__ flat) {
    __shared__ int s_first;
    for (int64_t t0 = (int64_t)blockIdx.x * kTile; t0 < total; t0 += (int64_t)gridDim.x * kTile) {
        if (threadIdx.x == 0) s_first = find_seg(off, nseg, t0);
        __syncthreads();
        int s = s_first;
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const int64_t i = t0 + (int64_t)j * kTPB + threadIdx.x;  // coalesced across lanes
            if (i < total) {
                while (off[s + 1] <= i) ++s;
                const int64_t k = i - off[s];
                // tensor pointers come from a table: address them as global memory (global_* not
                // flat_* instructions)
                typedef __attribute__((address_space(1))) float gfloat;
                gfloat* p = (gfloat*)(ptrs[s]);
                if (kGather) flat[i] = p[k];
                else p[k] = flat[i];
            }
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(kTPB) void synth_kernel(float* __restrict__ dst, int64_t n, uint64_t seed) {
    for (int64_t i = (int64_t)blockIdx.x * kTPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * kTPB) {
        uint64_t z = seed + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        dst[i] = (float)(z >> 40) * (1.0f / 8388608.0f) - 1.0f;
    }
}

// PullTransport snapshot (engine._step_pull): dst[i] = src[i], 16-byte accesses, then every
// workgroup makes its stores visible to OTHER GPUs before the kernel ends.  A peer reads the
// snapshot over xGMI from this GPU's HBM; plain stores may still sit dirty in this XCD's L2
// (write-back), and nothing in the round protocol (kernel end, synchronize, host barrier) is
// documented to write them back at system scope.  So, per workgroup (MI355X_MICROARCH.md, "Valid
// forms", producer): every wave waits for its stores (vmcnt(0)), a workgroup barrier, then one
// lane's system-scope release fence (buffer_wbl2 sc0 sc1 + wait: the XCD L2's dirty lines reach
// HBM) -- the release half of the protocol whose acquire half is the mixing kernels'
// peer_acquire (mix.hip).
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(kTPB) void publish_kernel(const f4* __restrict__ src, f4* __restrict__ dst,
                                                        int64_t n4) {
    for (int64_t i = (int64_t)blockIdx.x * kTPB + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kTPB)
        __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");        // system scope: buffer_wbl2 sc0 sc1
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

// The same copy restricted to the rows a peer reads this round (mx_snapshot_publish_rows): workgroup
// (x, r) first decides, for local row r, whether an active matching pairs worker row_base + r with
// a worker of another block -- the rows mx_pull_gate's peers point their receive slots at -- and a
// workgroup of an unread row leaves before its first store (so it owes no release either).
__global__ __launch_bounds__(kTPB) void publish_rows_kernel(const f4* __restrict__ src, int64_t src_ld4,
                                                            f4* __restrict__ dst, int64_t dst_ld4, int64_t n4,
                                                            const uint8_t* __restrict__ flags, int M,
                                                            const int32_t* __restrict__ partner, int n, int row_base,
                                                            int n_local) {
    const int r = blockIdx.y;
    const int w = row_base + r;
    int read = 0;
    for (int g = threadIdx.x; g < M; g += kTPB) {
        if (flags[g]) {
            const int q = partner[(int64_t)g * n + w];
            read |= q >= 0 && (q < row_base || q >= row_base + n_local);
        }
    }
    if (!__syncthreads_or(read)) return;                      // workgroup-uniform
    const f4* s = src + (int64_t)r * src_ld4;
    f4* d = dst + (int64_t)r * dst_ld4;
    for (int64_t i = (int64_t)blockIdx.x * kTPB + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kTPB)
        __builtin_nontemporal_store(__builtin_nontemporal_load(s + i), d + i);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");        // system scope: buffer_wbl2 sc0 sc1
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

unsigned grid_for(int64_t total) {
    int64_t g = (total + kTile - 1) / kTile;
    if (g > 4096) g = 4096;
    if (g < 1) g = 1;
    return (unsigned)g;
}
}  // namespace

extern "C" int mx_gather(const float* const* ptrs_dev, const int64_t* off_dev, int nseg,
                         int64_t total, float* flat, void* stream) {
    MX_CHECK(nseg >= 1 && total >= 0, "mx_gather: nseg=%d total=%lld", nseg, (long long)total);
    if (total == 0) return MX_OK;
    MX_CHECK(ptrs_dev && off_dev && flat, "mx_gather: null pointer");
    hipLaunchKernelGGL(seg_copy_kernel<true>, dim3(grid_for(total)), dim3(kTPB), 0,
                       mx::as_stream(stream), const_cast<float* const*>(ptrs_dev), off_dev, nseg,
                       total, flat);
    MX_LAUNCH_CHECK();
    return MX_OK;
}

extern "C" int mx_scatter(float* const* ptrs_dev, const int64_t* off_dev, int nseg, int64_t total,
                          const float* flat, void* stream) {
    MX_CHECK(nseg >= 1 && total >= 0, "mx_scatter: nseg=%d total=%lld", nseg, (long long)total);
    if (total == 0) return MX_OK;
    MX_CHECK(ptrs_dev && off_dev && flat, "mx_scatter: null pointer");
    hipLaunchKernelGGL(seg_copy_kernel<false>, dim3(grid_for(total)), dim3(kTPB), 0,
                       mx::as_stream(stream), ptrs_dev, off_dev, nseg, total,
                       const_cast<float*>(flat));
    MX_LAUNCH_CHECK();
    return MX_OK;
}

extern "C" int mx_synth_fill(float* dst, int64_t n, uint64_t seed, void* stream) {
    MX_CHECK(n >= 0, "mx_synth_fill: n < 0");
    if (n == 0) return MX_OK;
    MX_CHECK(dst, "mx_synth_fill: null pointer");
    int64_t g = (n + kTPB - 1) / kTPB;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(synth_kernel, dim3((unsigned)g), dim3(kTPB), 0, mx::as_stream(stream), dst, n, seed);
    MX_LAUNCH_CHECK();
    return MX_OK;
}

extern "C" int mx_snapshot_publish(const float* src, float* dst, int64_t n, void* stream) {
    MX_CHECK(n >= 0, "mx_snapshot_publish: n < 0");
    if (n == 0) return MX_OK;
    MX_CHECK(src && dst, "mx_snapshot_publish: null pointer");
    MX_CHECK(n % 4 == 0 && ((uintptr_t)src | (uintptr_t)dst) % 16 == 0,
             "mx_snapshot_publish: n (%lld) must be a multiple of 4 and both buffers 16-byte aligned", (long long)n);
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) cus = v;
    }
    const int64_t n4 = n / 4;
    int64_t g = (n4 + kTPB - 1) / kTPB;
    if (g > 4 * (int64_t)cus) g = 4 * (int64_t)cus;    // persistent: one release per workgroup at its end
    hipLaunchKernelGGL(publish_kernel, dim3((unsigned)g), dim3(kTPB), 0, mx::as_stream(stream),
                       reinterpret_cast<const f4*>(src), reinterpret_cast<f4*>(dst), n4);
    MX_LAUNCH_CHECK();
    return MX_OK;
}

extern "C" int mx_snapshot_publish_rows(const float* src, int64_t src_ld, float* dst, int64_t dst_ld, int64_t n,
                                        int n_local, const uint8_t* flags_row_dev, int M, const int32_t* partner_dev,
                                        int n_global, int row_base, void* stream) {
    MX_CHECK(n >= 0 && n_local >= 0, "mx_snapshot_publish_rows: n %lld, n_local %d", (long long)n, n_local);
    if (n == 0 || n_local == 0) return MX_OK;
    MX_CHECK(src && dst && flags_row_dev && partner_dev, "mx_snapshot_publish_rows: null pointer");
    MX_CHECK(n_local <= 65535 && M >= 1 && row_base >= 0 && row_base + n_local <= n_global,
             "mx_snapshot_publish_rows: block [%d, %d) of %d workers, M %d", row_base, row_base + n_local, n_global, M);
    MX_CHECK(n % 4 == 0 && src_ld % 4 == 0 && dst_ld % 4 == 0 && src_ld >= n && dst_ld >= n &&
                 ((uintptr_t)src | (uintptr_t)dst) % 16 == 0,
             "mx_snapshot_publish_rows: n %lld, src_ld %lld, dst_ld %lld must be multiples of 4 (ld >= n), buffers "
             "16-byte aligned", (long long)n, (long long)src_ld, (long long)dst_ld);
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) cus = v;
    }
    const int64_t n4 = n / 4;
    int64_t gx = (n4 + kTPB - 1) / kTPB;
    const int64_t cap = (4 * (int64_t)cus + n_local - 1) / n_local;   // ~4 workgroups per CU over all rows
    if (gx > cap) gx = cap;
    if (gx < 1) gx = 1;
    hipLaunchKernelGGL(publish_rows_kernel, dim3((unsigned)gx, (unsigned)n_local), dim3(kTPB), 0,
                       mx::as_stream(stream), reinterpret_cast<const f4*>(src), src_ld / 4, reinterpret_cast<f4*>(dst),
                       dst_ld / 4, n4, flags_row_dev, M, partner_dev, n_global, row_base, n_local);
    MX_LAUNCH_CHECK();
    return MX_OK;
}
