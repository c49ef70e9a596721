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
// bf16x3 conv weight image (RAVE_BF3_W4, round 5): 0 = three bf16 planes per
// K-step (6 bytes per weight); 1 = the exact-fp32 ring image (4 bytes per
// weight, rave_conv1d_ring_pack_weight's layout), split into hi / mid / lo in
// registers after each fragment load (conv_split.hip, edge_split.hip's tail)
#ifndef RAVE_BF3_W4
#define RAVE_BF3_W4 0
#endif

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

// Split-f16 range guard (RAVE_PREC_SPLIT16).  An operand v is carried as
// hi = f16(v), lo = f16((v - hi) * 2^11), which needs |v| < 2^15.  Kernels
// bf16x3 operand split (every kernel's RAVE_PREC_BF16X3 path): v == hi + mid + lo
// exactly, each a bf16 (RNE: the remainders v - hi and v - hi - mid are exact in
// fp32).  Worked in pairs: one v_cvt_pk_bf16_f32 per part and pair, the parts
// back to fp32 by a shift / mask of the packed word (bf16 -> fp32 is exact), the
// remainders by packed fp32 subtracts -- about half the VALU instructions of the
// element-wise form, bit for bit the same parts.  FV: 4 or 8 floats, BV: as many
// bf16.
template <typename FV, typename BV>
__device__ __forceinline__ void bf3_split_pk(const FV& v, BV& hi, BV& mid, BV& lo) {
    constexpr int N = (int)(sizeof(FV) / 4);
    static_assert((N == 4 || N == 8) && sizeof(BV) == 2 * sizeof(FV) / 4, "bf3_split_pk: 4 or 8 values");
    typedef float f2 __attribute__((ext_vector_type(2)));
    typedef __bf16 b2 __attribute__((ext_vector_type(2)));
    typedef unsigned uw __attribute__((ext_vector_type(N / 2)));
    uw h, m, l;
#pragma unroll
    for (int p = 0; p < N / 2; ++p) {
        const f2 x = {v[2 * p], v[2 * p + 1]};
        const unsigned hw = __builtin_bit_cast(unsigned, __builtin_convertvector(x, b2));
        const f2 hf = {__builtin_bit_cast(float, hw << 16), __builtin_bit_cast(float, hw & 0xFFFF0000u)};
        const f2 r = x - hf;
        const unsigned mw = __builtin_bit_cast(unsigned, __builtin_convertvector(r, b2));
        const f2 mf = {__builtin_bit_cast(float, mw << 16), __builtin_bit_cast(float, mw & 0xFFFF0000u)};
        h[p] = hw;
        m[p] = mw;
        l[p] = __builtin_bit_cast(unsigned, __builtin_convertvector(r - mf, b2));
    }
    hi = __builtin_bit_cast(BV, h);
    mid = __builtin_bit_cast(BV, m);
    lo = __builtin_bit_cast(BV, l);
}

// convert optimistically and vote per wave on max |v| >= kSplitLimit; a staged
// operand block that fails is re-converted as v * 2^-s (s = split_shift of its
// workgroup-wide max, so |v 2^-s| < 2^14) and the GEMM's accumulator (or the
// epilogue scale) takes the exact 2^s back.  NaN / inf pass through unscaled,
// as they do in fp32.
#ifndef RAVE_SPLIT_GUARD
#define RAVE_SPLIT_GUARD 1          // 0: A/B variant builds only (no range guard)
#endif
constexpr float kSplitLimit = 32768.f;
__device__ __forceinline__ int split_shift(float m) {
    if (!(m < 3.0e38f)) return 0;
    int e;
    (void)frexpf(m, &e);                      // m < 2^e
    return e > 14 ? e - 14 : 0;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}
// per-wave votes: wave w's lane 0 writes byte v[w] (0/1) unconditionally after
// its conversion; after a barrier any wave reads the NW bytes (masked dwords)
__device__ __forceinline__ void vote_cast(unsigned char* v, int wave, float m) {
    if (!RAVE_SPLIT_GUARD) return;
    const bool over = __builtin_amdgcn_ballot_w64(m >= kSplitLimit) != 0;
    if ((threadIdx.x & 63) == 0) v[wave] = over ? 1 : 0;
}
// the same byte from a per-lane flag (the unguarded pass's non-finite check)
__device__ __forceinline__ void vote_cast_any(unsigned char* v, int wave, bool bad) {
    const bool any = __builtin_amdgcn_ballot_w64(bad) != 0;
    if ((threadIdx.x & 63) == 0) v[wave] = any ? 1 : 0;
}
template <int NW>
__device__ __forceinline__ bool vote_any(const unsigned char* v) {
    if (!RAVE_SPLIT_GUARD) return false;
    const uint32_t* p = reinterpret_cast<const uint32_t*>(v);
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < (NW + 3) / 4; ++i) {
        uint32_t w = p[i];
        if ((i + 1) * 4 > NW) w &= (1u << (8 * (NW - 4 * i))) - 1u;
        x |= w;
    }
    return __builtin_amdgcn_readfirstlane(x != 0u ? 1 : 0) != 0;
}
// workgroup max of per-thread m through `red` (NW floats); one barrier
template <int NW>
__device__ __forceinline__ float block_max(float m, float* red) {
    m = wave_max(m);
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[wave] = m;
    __syncthreads();
    float mx = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) mx = fmaxf(mx, red[w]);
    return mx;
}
// max |v_i| of an 8-vector (the optimistic conversion's vote input)
template <typename V8>
__device__ __forceinline__ float absmax8(const V8& v) {
    float m = fabsf(v[0]);
#pragma unroll
    for (int i = 1; i < 8; ++i) m = fmaxf(m, fabsf(v[i]));
    return m;
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

// Shape limits of the fused residual stack (rave_residual_stack refuses the
// rest with RAVE_ERR_UNSUPPORTED): units 2..n reach at most 32 margin columns
// per side, and the bf16x3 form keeps a 24-row plane halo, so no unit's taps
// may reach past 24 columns on either side.  The engine checks it before it
// honours a tuned or pinned stack choice (stack_runs), so such a stack falls
// back to its units instead of failing at launch.
constexpr int kStackMargin = 32, kStackBf3Halo = 24;
inline bool stack_shape_fits(bool bf16x3, const int* dilation, const int* pad_left, int units) {
    int reach_l = 0, reach_r = 0;
    for (int u = 0; u < units; ++u) {
        const int d = dilation[u], pl = pad_left[u];
        if (bf16x3 && (pl > kStackBf3Halo || 2 * d - pl > kStackBf3Halo)) return false;
        if (u > 0) {
            reach_l += pl;
            reach_r += 2 * d - pl;
        }
    }
    return reach_l <= kStackMargin && reach_r <= kStackMargin;
}

}  // namespace rave
