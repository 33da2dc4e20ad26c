// pull.hip -- the pull transport's per-round handshake on the GPU (engine._step_pull).
//
// The reference's round is a blocking comm.sendrecv per active edge, bracketed by barriers
// (communicator.py:94-119).  Under PullTransport a partner's row is read by the mixing kernel
// straight from the peer GPU's IPC-mapped snapshot buffer, so all a round needs from its peers is
// "your snapshot of this round is in your HBM" and "you have finished reading mine of two rounds
// ago".  Both are epochs in the snapshot buffers' headers, published and awaited by one
// single-wave kernel enqueued between mx_snapshot_publish and the mixing launch -- no host
// synchronisation, barrier or copy per round:
//
//   publish(k)  -> gate(k) -> mix(k) -> publish(k+1) -> gate(k+1) -> ...     (one stream per rank)
//
// gate(k), epoch e = k + 1:
//   1. store epoch[me] = e with a system-scope release.  It runs after publish(k) has completed
//      (stream order) and every publish workgroup ended with a system-scope release of its
//      stores, so a peer that acquires e also sees the round-k snapshot;
//   2. wait (bounded) until epoch[r] >= e for every rank r that owns an active partner of a local
//      worker in round k or in the previous pull round (system-scope acquire loads):
//        - round k's partners: their round-k snapshots are complete before this rank's mix reads
//          them;
//        - the previous round's partners: they stored e only after their mix of round k-1 -- the
//          last reads of this rank's buffer (k+1) % 2 -- so publish(k+1), which follows this
//          gate, cannot overwrite a snapshot a peer is still reading.  (Matchings are symmetric:
//          the ranks this rank reads are the ranks that read it.)
//   3. point the round's receive slots at the partners' round-k snapshot rows: slot n_local + j
//      is the j-th distinct remote worker in (matching asc, sender id asc) order -- plan_kernel's
//      numbering (plan.hip) -- so the mixing kernel's plan record reads the right rows.
// On expiry the gate writes the sticky error words (host-mapped, read by the host at the end of
// the round: MXError) and returns; the mixing kernels' per-workgroup system-scope acquire
// (mix.hip, peer_acquire) keeps lines of a peer buffer cached here in round k-2 from being served.
#include "mx_common.h"

namespace {
typedef __attribute__((address_space(1))) uint64_t g_u64;
typedef __attribute__((address_space(1))) int32_t g_i32;

__device__ __forceinline__ uint64_t poll_epoch(const uint64_t* p) {
    return __hip_atomic_load((g_u64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

constexpr int kMaxWorkers = 4096;             // LDS bitmap of workers already given a slot

__global__ __launch_bounds__(64) void pull_gate_kernel(const uint8_t* __restrict__ flags, uint8_t* __restrict__ prev,
                                                       int M, const int32_t* __restrict__ partner, int n,
                                                       const int32_t* __restrict__ owner,
                                                       const mx_pull_rank* __restrict__ ranks, int nranks,
                                                       int me, int row_base, int n_local, int64_t ld_bytes,
                                                       int par, uint64_t epoch, int64_t* __restrict__ slots,
                                                       int n_slots, uint64_t spin_ticks, int32_t* err) {
    __shared__ uint64_t seen[kMaxWorkers / 64];
    __shared__ unsigned long long need;
    const int lane = threadIdx.x;
    for (int i = lane; i < (n + 63) / 64; i += 64) seen[i] = 0;
    if (lane == 0) {
        need = 0;
        __hip_atomic_store((g_u64*)ranks[me].base, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __syncthreads();
    // ranks owning an active remote partner of a local worker, this round or the previous one
    for (int g = 0; g < M; ++g) {
        const bool now = flags[g] != 0, before = prev[g] != 0;
        if (!now && !before) continue;
        for (int r = lane; r < n_local; r += 64) {
            const int p = partner[g * n + row_base + r];
            if (p >= 0 && (p < row_base || p >= row_base + n_local)) atomicOr(&need, 1ull << owner[p]);
        }
    }
    // receive slots of this round, in plan_kernel's first-appearance order
    int remote = 0;
    for (int g = 0; g < M; ++g) {
        if (!flags[g]) continue;
        for (int p0 = 0; p0 < n; p0 += 64) {
            const int p = p0 + lane;
            bool fresh = false;
            if (p < n) {
                const int q = partner[g * n + p];
                fresh = q >= row_base && q < row_base + n_local && (p < row_base || p >= row_base + n_local) &&
                        !((seen[p >> 6] >> (p & 63)) & 1);
            }
            const uint64_t b = __ballot(fresh);
            if (fresh) {
                const int slot = remote + __popcll(b & ((1ull << lane) - 1));
                const mx_pull_rank R = ranks[owner[p]];
                if (n_local + slot < n_slots)
                    slots[n_local + slot] = R.base + MX_PULL_HEADER_BYTES + (int64_t)par * R.n_local * ld_bytes +
                                            (int64_t)(p - R.row_base) * ld_bytes;
                else
                    __hip_atomic_store((g_i32*)err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                atomicOr((unsigned long long*)&seen[p >> 6], 1ull << (p & 63));
            }
            remote += __popcll(b);
            __syncthreads();
        }
    }
    __syncthreads();
    for (int g = lane; g < M; g += 64) prev[g] = flags[g];
    // the bounded wait: lane r polls rank r
    const uint64_t want = need;
    if (lane < nranks && lane != me && ((want >> lane) & 1)) {
        const uint64_t* ep = reinterpret_cast<const uint64_t*>(ranks[lane].base);
        const uint64_t t0 = wall_clock64();
        uint64_t got = poll_epoch(ep);
        while (got < epoch) {
            if ((uint64_t)wall_clock64() - t0 > spin_ticks) {
                __hip_atomic_store((g_i32*)(err + 1), lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store((g_i32*)(err + 2), (int32_t)epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store((g_i32*)(err + 3), (int32_t)got, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store((g_i32*)err, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
            __builtin_amdgcn_s_sleep(4);
            got = poll_epoch(ep);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");            // system scope
}
// The fetch of small remote payloads behind the gate (ChocoWorkerGroup under PullTransport: the
// partners' top-k messages, 1.79 MB each at VGG-16 size).  Workgroup (b, j) copies part b of remote
// slot j -- slot_ptrs[n_local + j], a peer's snapshot row pointed there by mx_pull_gate -- into
// dst + j * dst_ld, for j below the round's remote count (plan record word [1]: plan_kernel numbers
// the remote slots in the gate's order).  The bulk copy streams each message over its xGMI link
// with 16-byte loads, 4 in flight per lane, so the apply pass that follows reads only local memory
// (reading the messages in place inside the apply -- mx_choco_apply_slots -- costs every one of its
// thousands of workgroups a system-scope acquire and a dependent table load: one row 45 -> 66 us,
// profiles/r05y_slots_ab2.log).  Each workgroup acquires at system scope before its first load:
// the gate, earlier on this stream, saw the owners' epochs, which they stored after a system-scope
// release of the snapshot (the mixing kernels' protocol, mix.hip peer_acquire).
typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const f4 g_cf4;
typedef __attribute__((address_space(1))) f4 g_f4;

__global__ __launch_bounds__(256) void pull_fetch_kernel(const int64_t* __restrict__ slots, int n_local,
                                                         const int32_t* __restrict__ rec, char* __restrict__ dst,
                                                         int64_t dst_ld, int64_t n16) {
    const int j = blockIdx.y;
    if (j >= rec[1]) return;                                   // block-uniform
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");          // system scope: buffer_inv sc0 sc1
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    g_cf4* src = (g_cf4*)slots[n_local + j];
    g_f4* out = (g_f4*)(dst + (int64_t)j * dst_ld);
    constexpr int U = 4;
    const int64_t step = (int64_t)gridDim.x * 256;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + (U - 1) * step < n16; i += U * step) {
        f4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = src[i + u * step];
#pragma unroll
        for (int u = 0; u < U; ++u) out[i + u * step] = v[u];
    }
    for (; i < n16; i += step) out[i] = src[i];
}
}  // namespace

extern "C" int mx_pull_fetch(const int64_t* slot_ptrs_dev, int n_local, int max_remote, const int32_t* plan_rec_dev,
                             void* dst, int64_t dst_ld, int64_t nbytes, void* stream) {
    MX_CHECK(slot_ptrs_dev && plan_rec_dev && dst, "mx_pull_fetch: null pointer");
    MX_CHECK(n_local >= 1 && max_remote >= 0 && max_remote <= 65535 && nbytes >= 0,
             "mx_pull_fetch: n_local %d max_remote %d nbytes %lld", n_local, max_remote, (long long)nbytes);
    const int64_t n16 = (nbytes + 15) / 16;
    MX_CHECK(dst_ld >= 16 * n16 && dst_ld % 16 == 0 && (uintptr_t)dst % 16 == 0,
             "mx_pull_fetch: dst_ld %lld must hold %lld bytes, 16-byte aligned", (long long)dst_ld,
             (long long)(16 * n16));
    if (max_remote == 0 || n16 == 0) return MX_OK;
    int64_t nb = (n16 + 4 * 256 - 1) / (4 * 256);
    if (nb > 64) nb = 64;
    hipLaunchKernelGGL(pull_fetch_kernel, dim3((unsigned)nb, (unsigned)max_remote), dim3(256), 0,
                       mx::as_stream(stream), slot_ptrs_dev, n_local, plan_rec_dev, static_cast<char*>(dst), dst_ld,
                       n16);
    MX_LAUNCH_CHECK();
    return MX_OK;
}

extern "C" int mx_pull_gate(const uint8_t* flags_row_dev, uint8_t* prev_row_dev, int M, const int32_t* partner_dev,
                            int n_global, const int32_t* owner_dev, const mx_pull_rank* ranks_dev, int nranks,
                            int my_rank, int row_base, int n_local, int64_t ld_bytes, int parity, uint64_t epoch,
                            int64_t* slot_ptrs_dev, int n_slots, double timeout_s, int32_t* err_dev, void* stream) {
    MX_CHECK(flags_row_dev && prev_row_dev && partner_dev && owner_dev && ranks_dev && slot_ptrs_dev && err_dev,
             "mx_pull_gate: null pointer");
    MX_CHECK(M >= 1 && n_global >= 1 && n_global <= kMaxWorkers, "mx_pull_gate: M=%d n=%d (1..%d)", M, n_global,
             kMaxWorkers);
    MX_CHECK(nranks >= 1 && nranks <= 64 && my_rank >= 0 && my_rank < nranks, "mx_pull_gate: rank %d of %d (<= 64)",
             my_rank, nranks);
    MX_CHECK(n_local >= 1 && row_base >= 0 && row_base + n_local <= n_global && n_slots >= n_local,
             "mx_pull_gate: block [%d, %d) of %d, %d slots", row_base, row_base + n_local, n_global, n_slots);
    MX_CHECK(ld_bytes > 0 && ld_bytes % 16 == 0 && (parity == 0 || parity == 1) && epoch >= 1,
             "mx_pull_gate: ld_bytes %lld parity %d epoch %llu", (long long)ld_bytes, parity,
             (unsigned long long)epoch);
    MX_CHECK(timeout_s > 0, "mx_pull_gate: timeout_s %g", timeout_s);
    const uint64_t ticks = (uint64_t)(timeout_s * 1e8);      // s_memrealtime: the 100 MHz constant clock
    hipLaunchKernelGGL(pull_gate_kernel, dim3(1), dim3(64), 0, mx::as_stream(stream), flags_row_dev, prev_row_dev,
                       M, partner_dev, n_global, owner_dev, ranks_dev, nranks, my_rank, row_base, n_local, ld_bytes,
                       parity, epoch, slot_ptrs_dev, n_slots, ticks, err_dev);
    MX_LAUNCH_CHECK();
    return MX_OK;
}

// Host words the GPU writes and the host reads without a copy (coherent, mapped pinned memory).
extern "C" int mx_host_words(int n, int32_t** host_out, int32_t** dev_out) {
    MX_CHECK(n >= 1 && host_out && dev_out, "mx_host_words: bad arguments");
    void* h = nullptr;
    MX_HIP(hipHostMalloc(&h, (size_t)n * sizeof(int32_t), hipHostMallocMapped | hipHostMallocCoherent));
    memset(h, 0, (size_t)n * sizeof(int32_t));
    void* d = nullptr;
    const hipError_t e = hipHostGetDevicePointer(&d, h, 0);
    if (e != hipSuccess) {
        (void)hipHostFree(h);
        mx::set_error("mx_host_words: hipHostGetDevicePointer -> %s", hipGetErrorString(e));
        return MX_ERR_HIP;
    }
    *host_out = static_cast<int32_t*>(h);
    *dev_out = static_cast<int32_t*>(d);
    return MX_OK;
}

extern "C" int mx_host_words_free(int32_t* host) {
    if (!host) return MX_OK;
    MX_HIP(hipHostFree(host));
    return MX_OK;
}
