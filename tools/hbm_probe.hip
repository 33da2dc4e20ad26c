// hbm_probe.hip -- HBM ceilings for the mixing kernel's access pattern on this box (tool, not product).
//
// Every variant moves the same bytes as one headline gossip round (8 rows x 25.6M fp32 read and
// written = 1.6384 GB) so its time is directly comparable with mix_kernel:
//   copy     dst = src, one 819 MB stream in, another out
//   rmw1     x = a*x in place over one 819 MB buffer
//   rmw8     8 rows of 102 MB updated in place, each lane loading the same column of all 8 rows
//            before storing them (the mixing kernel's pattern, without the partner walk)
//   read / write   half the bytes, one direction only (reported as GB/s of their own bytes)
// Knobs per run: blocks per CU, non-temporal on/off, 16-byte accesses per lane per iteration (U).
//   hipcc --offload-arch=gfx950 -O3 -o tools/hbm_probe tools/hbm_probe.hip && tools/hbm_probe
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

template <bool NT>
__device__ __forceinline__ f4 ld(const f4* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(f4* p, f4 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// n4 = number of float4; every lane handles U float4 per iteration, 256-lane tiles strided
template <bool NT, int U>
__global__ __launch_bounds__(256) void k_copy(const f4* __restrict__ s, f4* __restrict__ d, int64_t n4) {
    const int64_t tile = 256 * U;
    for (int64_t b = (int64_t)blockIdx.x * tile; b < n4; b += (int64_t)gridDim.x * tile) {
        f4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = ld<NT>(s + b + u * 256 + threadIdx.x);
#pragma unroll
        for (int u = 0; u < U; ++u) st<NT>(d + b + u * 256 + threadIdx.x, v[u]);
    }
}

template <bool NT, int U>
__global__ __launch_bounds__(256) void k_rmw1(f4* __restrict__ x, int64_t n4, float a) {
    const int64_t tile = 256 * U;
    for (int64_t b = (int64_t)blockIdx.x * tile; b < n4; b += (int64_t)gridDim.x * tile) {
        f4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = ld<NT>(x + b + u * 256 + threadIdx.x);
#pragma unroll
        for (int u = 0; u < U; ++u) st<NT>(x + b + u * 256 + threadIdx.x, v[u] * a);
    }
}

// 8 rows of ld4 float4 each; lane loads its column of every row, then stores every row
template <bool NT>
__global__ __launch_bounds__(256) void k_rmw8(f4* __restrict__ x, int64_t ld4, float a) {
    for (int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x; c < ld4; c += (int64_t)gridDim.x * 256) {
        f4 v[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] = ld<NT>(x + r * ld4 + c);
        f4 sum = v[0];
#pragma unroll
        for (int r = 1; r < 8; ++r) sum += v[r];
#pragma unroll
        for (int r = 0; r < 8; ++r) st<NT>(x + r * ld4 + c, v[r] * a + sum * 1e-30f);
    }
}

// N rows of ldv VEC-float vectors, in place; each lane loads its column of every row, then stores
template <int N, int VEC>
__global__ __launch_bounds__(256) void k_rmwN(float* __restrict__ x, int64_t ldv, float a) {
    typedef float vt __attribute__((ext_vector_type(VEC)));
    vt* X = reinterpret_cast<vt*>(x);
    for (int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x; c < ldv; c += (int64_t)gridDim.x * 256) {
        vt v[N];
#pragma unroll
        for (int r = 0; r < N; ++r) v[r] = __builtin_nontemporal_load(X + r * ldv + c);
#pragma unroll
        for (int r = 0; r < N; ++r) __builtin_nontemporal_store(v[r] * a, X + r * ldv + c);
    }
}

// 8 rows, U quads per lane per row per tile (per-row contiguous chunk of U*4 KB per block); ROT:
// block b visits the rows starting at row b % 8 (staggers which row the chip hits first)
template <int U, bool ROT>
__global__ __launch_bounds__(256) void k_rmw8u(f4* __restrict__ x, int64_t ld4, float a) {
    const int64_t tile = 256 * U;
    const int r0 = ROT ? (int)(blockIdx.x & 7) : 0;
    for (int64_t b = (int64_t)blockIdx.x * tile; b < ld4; b += (int64_t)gridDim.x * tile) {
        f4 v[8][U];
#pragma unroll
        for (int rr = 0; rr < 8; ++rr)
#pragma unroll
            for (int u = 0; u < U; ++u) v[rr][u] = __builtin_nontemporal_load(x + ((rr + r0) & 7) * ld4 + b + u * 256 + threadIdx.x);
#pragma unroll
        for (int rr = 0; rr < 8; ++rr)
#pragma unroll
            for (int u = 0; u < U; ++u)
                __builtin_nontemporal_store(v[rr][u] * a, x + ((rr + r0) & 7) * ld4 + b + u * 256 + threadIdx.x);
    }
}

// Choco compaction read pattern: R rows of x and x_hat (2R streams), 4096-element chunks.
// FLAT = 0: grid (G, R), block (b, r) walks row r's chunks (every row streams concurrently);
// FLAT = 1: 1-D grid walks flat (row, chunk) indices, so the chip works through one row at a time.
template <int FLAT>
__global__ __launch_bounds__(256) void k_read_rows(const f4* __restrict__ x, const f4* __restrict__ xh,
                                                   int64_t ld4, int64_t nc, int rows, float* out) {
    f4 acc = {0, 0, 0, 0};
    const int64_t total = FLAT ? nc * rows : nc;
    const int64_t start = blockIdx.x, step = gridDim.x;
    for (int64_t f = start; f < total; f += step) {
        const int64_t r = FLAT ? f / nc : blockIdx.y;
        const int64_t c = FLAT ? f % nc : f;
        const int64_t q0 = r * ld4 + c * 1024 + threadIdx.x;
        f4 a[4], b[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            a[j] = __builtin_nontemporal_load(x + q0 + j * 256);
            b[j] = __builtin_nontemporal_load(xh + q0 + j * 256);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) acc += a[j] - b[j];
    }
    if (acc.x + acc.y + acc.z + acc.w == 1.2345f) out[0] = 1.0f;
}

template <bool NT, int U>
__global__ __launch_bounds__(256) void k_read(const f4* __restrict__ s, float* out, int64_t n4) {
    const int64_t tile = 256 * U;
    f4 acc = {0, 0, 0, 0};
    for (int64_t b = (int64_t)blockIdx.x * tile; b < n4; b += (int64_t)gridDim.x * tile) {
#pragma unroll
        for (int u = 0; u < U; ++u) acc += ld<NT>(s + b + u * 256 + threadIdx.x);
    }
    if (acc.x + acc.y + acc.z + acc.w == 1.2345f) out[0] = 1.0f;
}

template <bool NT, int U>
__global__ __launch_bounds__(256) void k_write(f4* __restrict__ d, int64_t n4) {
    const int64_t tile = 256 * U;
    const f4 v = {1, 2, 3, 4};
    for (int64_t b = (int64_t)blockIdx.x * tile; b < n4; b += (int64_t)gridDim.x * tile) {
#pragma unroll
        for (int u = 0; u < U; ++u) st<NT>(d + b + u * 256 + threadIdx.x, v);
    }
}

// One-row Choco compaction pattern with its per-chunk work switched on piece by piece (MODE bits:
// 1 LDS histogram atomics of kept keys, 2 the four wave scans, 4 the per-chunk barrier + cross-wave
// offsets, 8 the candidate stores, 16 the stores staged through LDS and written from the first
// lanes instead), same loop / prefetch structure as choco.hip's compact_kernel.
__global__ void k_fill(float* x, int64_t n, uint32_t seed) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t)i * 2654435761u ^ seed;
        h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
        x[i] = (float)(h >> 8) * (2.0f / 16777216.0f) - 1.0f;
    }
}

__device__ __forceinline__ uint32_t p_scan(uint32_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_compact_probe(const f4* __restrict__ x4, const f4* __restrict__ h4, int64_t nc,
                                                       uint32_t b_lo, float* cval, uint16_t* cloc, int64_t* cnt) {
    __shared__ uint32_t wtot[2][4];
    __shared__ uint32_t h[4096];
    __shared__ float sv[4][1024];                  // MODE 16: kept values / locations staged per wave
    __shared__ uint16_t sl[4][1024];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 4096; i += 256) h[i] = 0;
    f4 ax[4], ah[4];
    auto issue = [&](int64_t c) {
        const int64_t q0 = c * 1024 + wave * 256 + lane;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            ax[j] = __builtin_nontemporal_load(x4 + q0 + j * 64);
            ah[j] = __builtin_nontemporal_load(h4 + q0 + j * 64);
        }
    };
    int64_t c = blockIdx.x;
    if (c < nc) issue(c);
    __syncthreads();
    uint32_t sink = 0;
    for (int par = 0; c < nc; c += gridDim.x, par ^= 1) {
        float d[4][4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) d[j][e] = __fsub_rn(ax[j][e], ah[j][e]);
        const int64_t cn = c + gridDim.x;
        if (cn < nc) issue(cn);
        uint32_t keep = 0, incl[4], m[4], tot = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            m[j] = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t dg = (__float_as_uint(d[j][e]) & 0x7fffffffu) >> 19;
                const bool f = dg >= b_lo;
                keep |= (f ? 1u : 0u) << (4 * j + e);
                m[j] += f;
                if ((MODE & 1) && f) atomicAdd(&h[dg], 1u);
            }
            if (MODE & 2) {
                incl[j] = p_scan(m[j]);
                tot += __shfl(incl[j], 63, 64);
            } else {
                incl[j] = m[j];
                tot += m[j];
            }
        }
        uint32_t pos = 0;
        if (MODE & 4) {
            if (lane == 0) wtot[par][wave] = tot;
            __syncthreads();
            for (int w = 0; w < 4; ++w) pos += w < wave ? wtot[par][w] : 0;
        }
        if (MODE & 16) {                           // stage in LDS (wave-local positions), then
            uint32_t q = 0;                        // contiguous stores from the first lanes
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                uint32_t p = q + incl[j] - m[j];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if ((keep >> (4 * j + e)) & 1u) {
                        sv[wave][p] = d[j][e];
                        sl[wave][p] = (uint16_t)(1024 * wave + 4 * (64 * j + lane) + e);
                        ++p;
                    }
                }
                q += __shfl(incl[j], 63, 64);
            }
            float* cv = cval + c * 4096 + pos;
            uint16_t* cl = cloc + c * 4096 + pos;
            for (uint32_t i = lane; i < tot; i += 64) {
                cv[i & 4095] = sv[wave][i];
                cl[i & 4095] = sl[wave][i];
            }
            if (threadIdx.x == 0) cnt[c] = tot;
        } else if (MODE & 8) {
            float* cv = cval + c * 4096;
            uint16_t* cl = cloc + c * 4096;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                uint32_t p = pos + incl[j] - m[j];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if ((keep >> (4 * j + e)) & 1u) {
                        cv[p & 4095] = d[j][e];
                        cl[p & 4095] = (uint16_t)(1024 * wave + 4 * (64 * j + lane) + e);
                        ++p;
                    }
                }
                pos += (MODE & 2) ? __shfl(incl[j], 63, 64) : 0;
            }
            if (threadIdx.x == 0) cnt[c] = tot;
        } else {
            sink += keep + pos;
        }
    }
    __syncthreads();
    if ((MODE & 1) && h[threadIdx.x] == 12345u) cnt[0] = 1;
    if (sink == 0xdeadbeefu) cnt[1] = 1;
}

template <typename F>
static float time_ms(F launch, int reps = 30) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 5; ++i) launch();
    CK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int i = 0; i < reps; ++i) {
        CK(hipEventRecord(a, 0));
        launch();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int64_t P = 25600000, rows = 8;
    const int64_t n4 = rows * P / 4;            // one 819.2 MB buffer in float4
    const double round_bytes = 2.0 * rows * P * 4;
    f4 *A, *B;
    float* out;
    CK(hipMalloc(&A, n4 * 16 + (int64_t)8 * 65536 * 16 * 2));
    CK(hipMalloc(&B, n4 * 16));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(A, 0, n4 * 16 + (int64_t)8 * 65536 * 16 * 2));
    CK(hipMemset(B, 0, n4 * 16));
    auto report = [&](const char* name, int bpc, int nt, int u, double bytes, float ms) {
        printf("{\"kernel\": \"%s\", \"bpc\": %d, \"nt\": %d, \"U\": %d, \"us\": %.1f, \"TBps\": %.3f}\n",
               name, bpc, nt, u, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
        fflush(stdout);
    };
    for (int bpc : {2, 4, 8}) {
        if (getenv("PROBE_QUICK")) break;
        const int grid = cus * bpc;
#define RUN(NAME, NT, U, BYTES, ...) \
    report(NAME, bpc, NT, U, BYTES, time_ms([&] { hipLaunchKernelGGL(__VA_ARGS__); }))
        RUN("copy", 0, 1, round_bytes, (k_copy<false, 1>), dim3(grid), dim3(256), 0, 0, A, B, n4);
        RUN("copy", 1, 1, round_bytes, (k_copy<true, 1>), dim3(grid), dim3(256), 0, 0, A, B, n4);
        RUN("copy", 1, 4, round_bytes, (k_copy<true, 4>), dim3(grid), dim3(256), 0, 0, A, B, n4);
        RUN("copy", 0, 4, round_bytes, (k_copy<false, 4>), dim3(grid), dim3(256), 0, 0, A, B, n4);
        RUN("rmw1", 1, 1, round_bytes, (k_rmw1<true, 1>), dim3(grid), dim3(256), 0, 0, A, n4, 1.0f);
        RUN("rmw1", 1, 4, round_bytes, (k_rmw1<true, 4>), dim3(grid), dim3(256), 0, 0, A, n4, 1.0f);
        RUN("rmw1", 0, 4, round_bytes, (k_rmw1<false, 4>), dim3(grid), dim3(256), 0, 0, A, n4, 1.0f);
        RUN("rmw8", 1, 8, round_bytes, (k_rmw8<true>), dim3(grid), dim3(256), 0, 0, A, P / 4, 1.0f);
        RUN("rmw8", 0, 8, round_bytes, (k_rmw8<false>), dim3(grid), dim3(256), 0, 0, A, P / 4, 1.0f);
        RUN("read", 1, 4, round_bytes / 2, (k_read<true, 4>), dim3(grid), dim3(256), 0, 0, A, out, n4);
        RUN("read", 0, 4, round_bytes / 2, (k_read<false, 4>), dim3(grid), dim3(256), 0, 0, A, out, n4);
        RUN("write", 1, 4, round_bytes / 2, (k_write<true, 4>), dim3(grid), dim3(256), 0, 0, B, n4);
        RUN("write", 0, 4, round_bytes / 2, (k_write<false, 4>), dim3(grid), dim3(256), 0, 0, B, n4);
#undef RUN
    }
    // rmw8 with padded row strides: does the distance between the 8 rows matter (channel mapping)?
    for (int bpc : {3, 4, 5, 6}) {
        if (getenv("PROBE_WIDE")) break;
        const int grid = cus * bpc;
        for (int64_t pad4 : {0, 16, 64, 192, 256, 1024, 4096 + 64, 65536 + 256}) {
            const int64_t ld4 = P / 4 + pad4;
            char name[64];
            snprintf(name, sizeof(name), "rmw8_pad%lldB", (long long)(pad4 * 16));
            report(name, bpc, 1, 8, round_bytes,
                   time_ms([&] { hipLaunchKernelGGL((k_rmw8<true>), dim3(grid), dim3(256), 0, 0, A, ld4, 1.0f); }));
        }
        report("rmw1", bpc, 1, 1, round_bytes,
               time_ms([&] { hipLaunchKernelGGL((k_rmw1<true, 1>), dim3(grid), dim3(256), 0, 0, A, n4, 1.0f); }));
    }
    if (getenv("PROBE_ROWS")) {        // Choco compaction: 8 rows x 14,774,436 of x and x_hat
        const int64_t Pc = 14774436 / 4096 * 4096, rowsc = 8, ld4 = Pc / 4, ncc = Pc / 4096;
        const double bytes = 2.0 * rowsc * Pc * 4;
        f4* Xh = B;                          // x rows in A, x_hat rows in B (both 819 MB buffers)
        for (int g : {256, 512, 1024, 2048}) {
            report("rows_concurrent", g, 1, 0, bytes, time_ms([&] {
                hipLaunchKernelGGL((k_read_rows<0>), dim3(g / 8, 8), dim3(256), 0, 0, A, Xh, ld4, ncc, 8, out);
            }));
            report("rows_flat", g, 1, 0, bytes, time_ms([&] {
                hipLaunchKernelGGL((k_read_rows<1>), dim3(g), dim3(256), 0, 0, A, Xh, ld4, ncc, 8, out);
            }));
        }
        {   // the compaction's per-chunk work, piece by piece, one row (random x, x_hat = 0)
            hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (float*)A, Pc, 1234u);
            CK(hipMemset(B, 0, Pc * 4));
            float* cv;
            uint16_t* cl;
            int64_t* cn;
            CK(hipMalloc(&cv, Pc * 4));
            CK(hipMalloc(&cl, Pc * 2));
            CK(hipMalloc(&cn, ncc * 8));
            union { float f; uint32_t u; } t{0.9875f};
            const uint32_t b_lo = (t.u & 0x7fffffffu) >> 19;
#define CP(M)                                                                                             \
    report("compact_mode" #M, 1024, 1, M, bytes / 8, time_ms([&] {                                    \
        hipLaunchKernelGGL((k_compact_probe<M>), dim3(1024), dim3(256), 0, 0, A, Xh, ncc, b_lo, cv, cl, cn); \
    }))
            CP(0); CP(1); CP(2); CP(4); CP(8); CP(3); CP(7); CP(15); CP(14); CP(13); CP(11); CP(23);
#undef CP
        }
        for (int g : {256, 512, 1024, 2048, 4096}) {   // one row (a VGG-16 worker per GPU): 118 MB
            report("one_row", g, 1, 0, bytes / 8, time_ms([&] {
                hipLaunchKernelGGL((k_read_rows<1>), dim3(g), dim3(256), 0, 0, A, Xh, ld4, ncc, 1, out);
            }));
        }
        (void)rowsc;
        return 0;
    }
    // many rows, small per-row chunks (the wide-slot mixing layouts)
    if (getenv("PROBE_WIDE")) {
        const int64_t total = rows * P;   // same 819.2 MB arena
        for (int bpc : {2, 4, 8}) {
            const int grid = cus * bpc;
#define RW(N, V)                                                                                   \
    report("rmw" #N "_vec" #V, bpc, 1, V, round_bytes, time_ms([&] {                             \
        hipLaunchKernelGGL((k_rmwN<N, V>), dim3(grid), dim3(256), 0, 0, (float*)A, total / N / V, 1.0f); \
    }))
            RW(8, 4); RW(16, 4); RW(16, 2); RW(32, 4); RW(32, 2); RW(32, 1); RW(64, 2); RW(64, 1);
#undef RW
#define RU(U, ROT)                                                                                 \
    report("rmw8_U" #U "_rot" #ROT, bpc, 1, U, round_bytes, time_ms([&] {                        \
        hipLaunchKernelGGL((k_rmw8u<U, ROT>), dim3(grid), dim3(256), 0, 0, A, P / 4, 1.0f);        \
    }))
            RU(1, false); RU(2, false); RU(4, false); RU(1, true); RU(2, true); RU(4, true);
#undef RU
            report("rmw1", bpc, 1, 1, round_bytes,
                   time_ms([&] { hipLaunchKernelGGL((k_rmw1<true, 1>), dim3(grid), dim3(256), 0, 0, A, n4, 1.0f); }));
        }
        return 0;
    }
    report("hipMemcpyDtoD", 0, 0, 0, round_bytes,
           time_ms([&] { CK(hipMemcpyAsync(B, A, n4 * 16, hipMemcpyDeviceToDevice, 0)); }));
    return 0;
}
