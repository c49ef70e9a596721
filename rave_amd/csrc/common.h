// Shared helpers for the rave_amd native library (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/rave_amd.h"

namespace rave {

void set_error(const std::string& msg);

#define RAVE_CHECK_ARG(cond, msg)                 \
    do {                                          \
        if (!(cond)) {                            \
            ::rave::set_error(msg);               \
            return RAVE_ERR_ARG;                  \
        }                                         \
    } while (0)

#define RAVE_CHECK_HIP(expr)                                                        \
    do {                                                                            \
        hipError_t e_ = (expr);                                                     \
        if (e_ != hipSuccess) {                                                     \
            ::rave::set_error(std::string(#expr) + ": " + hipGetErrorString(e_));   \
            return RAVE_ERR_HIP;                                                    \
        }                                                                           \
    } while (0)

inline int launch_status(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error(std::string(what) + " launch: " + hipGetErrorString(e));
        return RAVE_ERR_HIP;
    }
    return RAVE_OK;
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Per-op timing hook of the plan executor (rave_plan_profile).  While set, the
// op's launches carry the events inside their own dispatch packets
// (hipExtLaunchKernelGGL): the first launch takes the start event, every launch
// re-records the stop event, so the op's time is first-kernel start to
// last-kernel end with no marker packets between kernels.
struct OpEvents {
    hipEvent_t start = nullptr;
    hipEvent_t stop = nullptr;
};
extern thread_local OpEvents g_op_events;

template <typename K, typename... Args>
inline void launch(K kernel, dim3 grid, dim3 block, uint32_t lds, hipStream_t st, Args... args) {
    OpEvents& e = g_op_events;
    if (e.stop) {
        hipExtLaunchKernelGGL(kernel, grid, block, lds, st, e.start, e.stop, 0, args...);
        e.start = nullptr;
    } else {
        hipLaunchKernelGGL(kernel, grid, block, lds, st, args...);
    }
}

// Logical workgroup id of a 1-D grid, XCD-major: blocks are dealt round-robin
// over the 8 XCDs, so block i runs on XCD i % 8; the remap hands every XCD a
// contiguous run of logical ids (batch-major tile orders: a contiguous run of
// batch items).  Every kernel of the path uses the same batch-major order, so
// an XCD reads the activations of the batch items it wrote in the previous
// launch out of its own L2 instead of another XCD's (via the Infinity Cache).
// A bijection for any grid, so correctness never depends on the placement.
__device__ __forceinline__ int xcd_major(int lin, int grid) {
#ifndef RAVE_LEGACY_MAP
    if ((grid & 7) == 0) return (lin & 7) * (grid >> 3) + (lin >> 3);
#endif
    (void)grid;
    return lin;
}

// Cache-policy bits of the layer-output stores (buffer instruction aux field;
// 16 = sc1, write-through).  Default: plain stores (the line stays in the
// writing XCD's L2 for the next kernel's reads).
#ifndef RAVE_YAUX
#define RAVE_YAUX 0
#endif

constexpr int ceil_div(int a, int b) { return (a + b - 1) / b; }
constexpr int64_t ceil_div64(int64_t a, int64_t b) { return (a + b - 1) / b; }

// sin(x)^2 with a 3-constant Cody-Waite reduction by pi/2 and Cephes' minimax
// polynomials on [-pi/4, pi/4]; |error| <= 1.7e-7 for |x| < 1e3 (host check
// against libm double), branch-free and scratch-free (ocml's sinf carries a
// Payne-Hanek slow path with a private-memory table).
__device__ __forceinline__ float sin_squared(float x) {
    const float q = rintf(x * 0.636619772367581343f);
    float r = fmaf(q, -1.57079637050628662109375f, x);
    r = fmaf(q, 4.371138828673793e-08f, r);
    r = fmaf(q, 1.7151245100058819e-15f, r);
    const float z = r * r;
    const float s = fmaf(fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f), z * r, r);
    const float c = fmaf(fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z,
                              4.166664568298827e-2f),
                         z * z, fmaf(-0.5f, z, 1.0f));
    const float v = (static_cast<int>(q) & 1) ? c : s;
    return v * v;
}

// Input-activation prologue shared by the conv and noise kernels.
// LeakyReLU(slope) (rave/blocks.py:91) and Snake (rave/blocks.py:852-853):
//   x + (alpha + 1e-9)^-1 * sin(alpha * x)^2   -- same operation order as torch.
__device__ __forceinline__ float apply_act(float v, int act, float slope, float alpha) {
    if (act == RAVE_ACT_LEAKY) return v > 0.f ? v : v * slope;
    if (act == RAVE_ACT_SNAKE) {
        const float r = 1.0f / (alpha + 1e-9f);
        return v + r * sin_squared(alpha * v);
    }
    return v;
}

}  // namespace rave
