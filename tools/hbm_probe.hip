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
