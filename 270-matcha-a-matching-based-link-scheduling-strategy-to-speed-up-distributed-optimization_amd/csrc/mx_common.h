// mx_common.h -- shared helpers for the gfx950 gossip library (error plumbing, launch math).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/matcha_gossip.h"

namespace mx {

// thread-local last-error text, surfaced through mx_last_error()
void set_error(const char* fmt, ...);

#define MX_HIP(call)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (call);                                                             \
        if (e_ != hipSuccess) {                                                             \
            ::mx::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #call, hipGetErrorString(e_)); \
            return MX_ERR_HIP;                                                              \
        }                                                                                   \
    } while (0)

#define MX_CHECK(cond, ...)                                                                 \
    do {                                                                                    \
        if (!(cond)) {                                                                      \
            ::mx::set_error(__VA_ARGS__);                                                   \
            return MX_ERR_INVALID;                                                          \
        }                                                                                   \
    } while (0)

#define MX_LAUNCH_CHECK()                                                                   \
    do {                                                                                    \
        hipError_t e_ = hipGetLastError();                                                  \
        if (e_ != hipSuccess) {                                                             \
            ::mx::set_error("%s:%d launch -> %s", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return MX_ERR_HIP;                                                              \
        }                                                                                   \
    } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Plan record geometry (see include/matcha_gossip.h, mx_plan_build)
constexpr int kPlanHeader = 4;
__host__ __device__ inline int64_t plan_words(int n_local, int M) {
    return (int64_t)kPlanHeader + 2 * (int64_t)n_local + (int64_t)n_local * M;
}

// LDS per CU (device attribute; 160 KB on gfx950) and the dynamic LDS that, on top of a kernel's
// static_bytes, admits exactly wg_per_cu of its workgroups per CU: the per-workgroup total sits in
// the middle of that count's window, so allocation rounding cannot tip it into the next count
// (0 when no padding is needed or wg_per_cu <= 0).  Streaming kernels whose every load is issued
// at once run fastest with few tiles in flight per CU (tools/occ_sweep.py, tools/mean_ab.py).
int lds_per_cu();
size_t lds_cap_pad(int static_bytes, int wg_per_cu);
extern int g_mean_wgpc;   // mean_tile_kernel's workgroups per CU on large rounds (mx_mix_set "mean_wgpc")

// numpy legacy_random_binomial(n=1) parameters, computed on the host with glibc libm exactly
// as numpy's legacy_random_binomial_inversion does (see flags.hip).
struct BinomParam {
    double qn;   // exp(1 * log(q)),   q = 1 - pp
    double px1;  // ((1 * pp) * qn) / (1 * q)
    int flip;    // p > 0.5: result is 1 - X
    int pad;
};

}  // namespace mx
