// Fused Residual(DilatedUnit) -- rave/blocks.py:32-46 (Residual / AlignBranches
// sum) around rave/blocks.py:84-113 (DilatedUnit):
//
//     y = x + conv1x1(act2(conv3_d(act0(x)) + b1)) + b2
//
// in ONE kernel: the k=3 dilated conv's output never leaves the chip.
//
// A workgroup owns every channel of a BN-column slab of one batch item:
//   prologue  act0(x) window [C][BN + 2d] -> LDS (one coalesced HBM read; the
//             dilated halo is fetched once and shared by the three taps)
//   phase 1   h = W1 (C x 3C) . window        fp32 MFMA, B fragments from LDS
//   seam      h = act2(h + b1) -> LDS (over the dead window)
//   phase 2   y = W2 (C x C) . h              fp32 MFMA, B fragments from LDS
//   epilogue  y + b2 + x (residual re-read, L2-hot) -> HBM
//
// Weights never touch LDS: each wave streams the A fragments of its own row
// blocks straight from L2 into a register ring (host-packed so that one
// 16-byte load per lane feeds four MFMAs and a wave's 64 loads are one
// contiguous kilobyte), prefetched several MFMA groups ahead and running on
// from W1 into W2 across the seam.
//
// Tile shapes: C <= 128 uses v_mfma_f32_32x32x2_f32 with 32-column blocks;
// C >= 256 uses v_mfma_f32_16x16x4_f32 on 16-column slabs so that the small
// time extents of the deep stages (T = 256 / 128 per item) still spread over
// the chip.  Both are exact fp32 (k-ordered fmaf chains).
#include "common.h"

#include <algorithm>
#include <cstring>

namespace rave {

typedef float u_f32x16 __attribute__((ext_vector_type(16)));
typedef float u_f32x4 __attribute__((ext_vector_type(4)));

constexpr int kUnitMaxDil = 24;     // largest dilation the window staging covers
constexpr unsigned kUnitOOB = 0xFFFFFFF0u;   // buffer offset past any extent: load 0 / store dropped

struct UnitKArgs {
    const float* x; float* y; const float* w;
    const float* b1; const float* b2; const float* a0; const float* a2;
    int64_t x_sb, x_sc, y_sb, y_sc;
    int T, d, pad_l, ntiles, W, XWS, HS;
    int XL, rsh;             // valid input columns; residual column shift (cached form)
    int x_bytes, y_bytes, w_bytes, bias_bytes;
    int act;
    float slope;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t unit_rsrc(const void* p, int bytes) {
    const uint64_t v = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    const uint64_t u = ((uint64_t)hi << 32) | lo;
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(u), (short)0,
                                             __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

__device__ __forceinline__ float ld1(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}

template <bool SNAKE>
__device__ __forceinline__ float unit_act(float v, float slope, float alpha) {
    if constexpr (SNAKE) {
        const float r = 1.0f / (alpha + 1e-9f);
        return v + r * sin_squared(alpha * v);
    } else {
        return v > 0.f ? v : v * slope;     // slope 1 == no activation
    }
}

template <int MT> struct Mfma;
template <> struct Mfma<32> {
    static constexpr int KM = 2, ACC = 16;
    typedef u_f32x16 acc_t;
    static __device__ __forceinline__ acc_t mma(float a, float b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
    }
    // accumulator element r of `lane` -> (row, col) of the 32x32 tile
    static __device__ __forceinline__ int row(int lane, int r) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }
    static __device__ __forceinline__ int col(int lane) { return lane & 31; }
};
template <> struct Mfma<16> {
    static constexpr int KM = 4, ACC = 4;
    typedef u_f32x4 acc_t;
    static __device__ __forceinline__ acc_t mma(float a, float b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ int row(int lane, int r) { return 4 * (lane >> 4) + r; }
    static __device__ __forceinline__ int col(int lane) { return lane & 15; }
};

template <int C> struct UnitShape;
template <> struct UnitShape<64> { static constexpr int BN = 128, MT = 32; };
template <> struct UnitShape<128> { static constexpr int BN = 64, MT = 32; };
template <> struct UnitShape<256> { static constexpr int BN = 16, MT = 16; };
template <> struct UnitShape<512> { static constexpr int BN = 16, MT = 16; };

constexpr int kUnitWaves = 8;
constexpr int kUnitThreads = 64 * kUnitWaves;
constexpr int kRing = 4;            // 16-byte A loads in flight per row block

template <int C>
struct UnitGeo {
    static constexpr int BN = UnitShape<C>::BN, MT = UnitShape<C>::MT;
    static constexpr int KM = Mfma<MT>::KM;
    static constexpr int NT_M = C / MT, NT_N = BN / MT;
    static constexpr int WPC = kUnitWaves / NT_N;          // waves sharing a column block
    static constexpr int TPW = NT_M / WPC;                 // row blocks per wave
    static constexpr int G1 = 3 * C / KM / 4;              // 4-MFMA groups, phase 1
    static constexpr int G2 = C / KM / 4;                  // phase 2
    static constexpr int GT = G1 + G2;
    static constexpr int ROWS = C / kUnitWaves;            // window rows staged per wave
    static constexpr int NCH = (BN + 2 * kUnitMaxDil + 63) / 64;
    static_assert(kUnitWaves % NT_N == 0 && NT_M % WPC == 0, "tile split");
    static_assert(G1 % kRing == 0 && G2 % kRing == 0, "ring");
};

template <int C, bool SNAKE>
__global__ __launch_bounds__(kUnitThreads) void residual_unit_kernel(UnitKArgs a) {
    using G = UnitGeo<C>;
    using M = Mfma<G::MT>;
    constexpr int MT = G::MT, KM = G::KM, TPW = G::TPW;
    extern __shared__ __attribute__((aligned(16))) float lds[];

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lg = __builtin_amdgcn_readfirstlane(xcd_major(blockIdx.x, gridDim.x));
    const int b = lg / a.ntiles;
    const int n0 = (lg - b * a.ntiles) * G::BN;
    const float slope = a.act == RAVE_ACT_LEAKY ? a.slope : 1.0f;

    const auto xrs = unit_rsrc(a.x + (int64_t)b * a.x_sb, a.x_bytes);
    const auto wrs = unit_rsrc(a.w, a.w_bytes);

    // ---------------------------------------------------------------- A ring
    // row block mb_i = mg + i*WPC; group g of its stream at ((mb*GT + g)*64 + lane)*16 bytes
    const int nb = wave % G::NT_N;
    const int mg = wave / G::NT_N;
    unsigned abase[TPW];
#pragma unroll
    for (int i = 0; i < TPW; ++i) abase[i] = ((unsigned)((mg + i * G::WPC) * G::GT) * 64u + lane) * 16u;
    u_f32x4 ring[TPW][kRing];
#pragma unroll
    for (int q = 0; q < kRing; ++q)
#pragma unroll
        for (int i = 0; i < TPW; ++i)
            ring[i][q] = __builtin_bit_cast(u_f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                wrs, abase[i] + (unsigned)q * 1024u, 0, 0));

    // ---------------------------------------------------------------- prologue: act0(x) window
    {
        const int t0 = n0 - a.pad_l;
        float v[G::ROWS][G::NCH];
#pragma unroll
        for (int r = 0; r < G::ROWS; ++r)
#pragma unroll
            for (int ch = 0; ch < G::NCH; ++ch) {
                const int c = wave + r * kUnitWaves;
                const int w = ch * 64 + lane;
                const int t = t0 + w;
                const bool ok = w < a.W && t >= 0 && t < a.XL;
                v[r][ch] = ld1(xrs, ok ? (unsigned)(c * a.x_sc + t) * 4u : kUnitOOB);
            }
#pragma unroll
        for (int r = 0; r < G::ROWS; ++r) {
            const int c = wave + r * kUnitWaves;
            const float al = SNAKE ? a.a0[c] : 0.f;
#pragma unroll
            for (int ch = 0; ch < G::NCH; ++ch) {
                const int w = ch * 64 + lane;
                if (w < a.W) lds[c * a.XWS + w] = unit_act<SNAKE>(v[r][ch], slope, al);
            }
        }
    }
    __syncthreads();

    // ---------------------------------------------------------------- phase 1: k=3 dilated conv
    typename M::acc_t acc[TPW];
#pragma unroll
    for (int i = 0; i < TPW; ++i)
#pragma unroll
        for (int r = 0; r < M::ACC; ++r) acc[i][r] = 0.f;

    const int kl = lane / MT;                       // k row of this lane inside an MFMA
    const int ncol = nb * MT + M::col(lane);        // local output column

    for (int g0 = 0; g0 < G::G1; g0 += kRing) {
#pragma unroll
        for (int q = 0; q < kRing; ++q) {
            const int g = g0 + q;
            const int k0 = g * 4 * KM;               // first k of the group (uniform)
            const int j = k0 / C;                    // tap
            const int ci0 = k0 - j * C;
            const float* bp = lds + (ci0 + kl) * a.XWS + ncol + j * a.d;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float bv = bp[e * KM * a.XWS];
#pragma unroll
                for (int i = 0; i < TPW; ++i) acc[i] = M::mma(ring[i][q][e], bv, acc[i]);
            }
            {   // refill the slot with stream group g + kRing (runs on into W2)
                const int gn = g + kRing;
#pragma unroll
                for (int i = 0; i < TPW; ++i)
                    ring[i][q] = __builtin_bit_cast(u_f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                        wrs, gn < G::GT ? abase[i] + (unsigned)gn * 1024u : kUnitOOB, 0, 0));
                // keep the refill here: the scheduler would otherwise sink the
                // loads next to their consumers kRing groups later
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
    __syncthreads();                                 // window dead

    // ---------------------------------------------------------------- seam: h = act2(h + b1) -> LDS
    {
        const auto brs = unit_rsrc(a.b1, a.bias_bytes);
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
            const int m0 = (mg + i * G::WPC) * MT;
#pragma unroll
            for (int r = 0; r < M::ACC; ++r) {
                const int m = m0 + M::row(lane, r);
                float h = acc[i][r] + ld1(brs, (unsigned)m * 4u);
                h = unit_act<SNAKE>(h, slope, SNAKE ? a.a2[m] : 0.f);
                lds[m * a.HS + ncol] = h;
                acc[i][r] = 0.f;
            }
        }
    }
    __syncthreads();

    // ---------------------------------------------------------------- phase 2: 1x1 conv
    for (int g0 = 0; g0 < G::G2; g0 += kRing) {
#pragma unroll
        for (int q = 0; q < kRing; ++q) {
            const int g = g0 + q;
            const float* bp = lds + (g * 4 * KM + kl) * a.HS + ncol;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float bv = bp[e * KM * a.HS];
#pragma unroll
                for (int i = 0; i < TPW; ++i) acc[i] = M::mma(ring[i][q][e], bv, acc[i]);
            }
            {   // refill the slot with stream group g + kRing (runs on into W2)
                const int gn = G::G1 + g + kRing;
#pragma unroll
                for (int i = 0; i < TPW; ++i)
                    ring[i][q] = __builtin_bit_cast(u_f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                        wrs, gn < G::GT ? abase[i] + (unsigned)gn * 1024u : kUnitOOB, 0, 0));
                // keep the refill here: the scheduler would otherwise sink the
                // loads next to their consumers kRing groups later
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }

    // ---------------------------------------------------------------- epilogue: + b2 + x
    {
        const auto brs = unit_rsrc(a.b2, a.bias_bytes);
        const auto yrs = unit_rsrc(a.y + (int64_t)b * a.y_sb, a.y_bytes);
        const int n = n0 + ncol;
        const bool nok = n < a.T;
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
            const int m0 = (mg + i * G::WPC) * MT;
            float res[M::ACC];
#pragma unroll
            for (int r = 0; r < M::ACC; ++r) {
                const int m = m0 + M::row(lane, r);
                res[r] = ld1(xrs, nok ? (unsigned)(m * a.x_sc + n + a.rsh) * 4u : kUnitOOB) +
                         ld1(brs, (unsigned)m * 4u);
            }
#pragma unroll
            for (int r = 0; r < M::ACC; ++r) {
                const int m = m0 + M::row(lane, r);
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, acc[i][r] + res[r]), yrs,
                                                      nok ? (unsigned)(m * a.y_sc + n) * 4u : kUnitOOB, 0, 0);
            }
        }
    }
}

template <int C>
static int unit_launch(UnitKArgs k, int B, bool snake, hipStream_t st) {
    using G = UnitGeo<C>;
    // LDS: the window, then h over it
    const size_t lds = (size_t)std::max(C * k.XWS, C * k.HS) * sizeof(float);
    auto kern = snake ? residual_unit_kernel<C, true> : residual_unit_kernel<C, false>;
    static bool attr_set[2] = {false, false};
    if (lds > 65536 && !attr_set[snake]) {
        RAVE_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        attr_set[snake] = true;
    }
    (void)G::BN;
    launch(kern, dim3(k.ntiles * B), dim3(kUnitThreads), (uint32_t)lds, st, k);
    return launch_status("residual_unit_kernel");
}

static int unit_mt(int C) { return C >= 256 ? 16 : 32; }
static int unit_bn(int C) { return C == 64 ? 128 : (C == 128 ? 64 : 16); }
static bool unit_supported(int C) { return C == 64 || C == 128 || C == 256 || C == 512; }

// LDS row stride >= w, chosen so an MFMA's B-fragment read is bank-conflict
// free: 32x32 reads 2 rows x 32 columns (stride = 32 mod 64), 16x16x4 reads
// 4 rows x 16 columns (stride = 16 mod 32).
static int unit_stride(int w, int mt) {
    int s = w;
    if (mt == 32) while (s % 64 != 32) ++s;
    else while (s % 32 != 16) ++s;
    return s;
}

}  // namespace rave

using namespace rave;

extern "C" int64_t rave_unit_packed_size(int channels) {
    if (!unit_supported(channels)) return -1;
    return (int64_t)4 * channels * channels;
}

extern "C" int rave_unit_pack_weight(const float* w1, const float* w2, int C, float* packed) {
    RAVE_CHECK_ARG(w1 && w2 && packed, "unit_pack_weight: null pointer");
    if (!unit_supported(C)) {
        set_error("unit_pack_weight: fused residual unit supports C in {64, 128, 256, 512}");
        return RAVE_ERR_UNSUPPORTED;
    }
    const int MT = unit_mt(C), KM = MT == 32 ? 2 : 4;
    const int S1 = 3 * C / KM, S2 = C / KM, GT = (S1 + S2) / 4;
    for (int mb = 0; mb < C / MT; ++mb)
        for (int g = 0; g < GT; ++g)
            for (int l = 0; l < 64; ++l)
                for (int e = 0; e < 4; ++e) {
                    const int s = 4 * g + e;
                    const int m = mb * MT + l % MT;
                    float v;
                    if (s < S1) {
                        const int k = s * KM + l / MT, j = k / C, ci = k % C;
                        v = w1[((int64_t)m * C + ci) * 3 + j];
                    } else {
                        const int ci = (s - S1) * KM + l / MT;
                        v = w2[(int64_t)m * C + ci];
                    }
                    packed[(((int64_t)mb * GT + g) * 64 + l) * 4 + e] = v;
                }
    return RAVE_OK;
}

namespace rave {
int residual_unit_split(const rave_unit_args& a, void* stream);   // unit_split.hip
}

extern "C" int rave_residual_unit(const rave_unit_args* p, void* stream) {
    RAVE_CHECK_ARG(p && p->x && p->y && p->weight, "residual_unit: null pointer");
    const rave_unit_args& a = *p;
    RAVE_CHECK_ARG(a.precision == RAVE_PREC_F32 || a.precision == RAVE_PREC_SPLIT16 || a.precision == RAVE_PREC_F32_RING ||
                       a.precision == RAVE_PREC_BF16X3,
                   "residual_unit: unknown precision");
    if (!unit_supported(a.channels)) {
        set_error("residual_unit: fused residual unit supports C in {64, 128, 256, 512}");
        return RAVE_ERR_UNSUPPORTED;
    }
    RAVE_CHECK_ARG(a.batch > 0 && a.t_len > 0, "residual_unit: empty shape");
    RAVE_CHECK_ARG(a.dilation >= 1 && a.dilation <= kUnitMaxDil, "residual_unit: dilation out of range");
    RAVE_CHECK_ARG(a.pad_left >= 0 && a.pad_left <= 2 * a.dilation,
                   "residual_unit: pad_left must be in [0, 2*dilation] (centered d, causal 2d)");
    RAVE_CHECK_ARG(a.act == RAVE_ACT_LEAKY || a.act == RAVE_ACT_SNAKE || a.act == RAVE_ACT_NONE,
                   "residual_unit: bad activation");
    RAVE_CHECK_ARG(a.act != RAVE_ACT_SNAKE || (a.alpha0 && a.alpha2), "residual_unit: snake needs alphas");
    RAVE_CHECK_ARG(a.act != RAVE_ACT_LEAKY || a.leaky_slope <= 1.0f, "residual_unit: leaky slope above 1");
    RAVE_CHECK_ARG(a.x != a.y, "residual_unit: y must not alias x (other slabs still read it)");
    {
        // cached form: the window and the shifted residual stay inside x's valid columns
        const int xl = a.x_len > 0 ? a.x_len : a.t_len;
        RAVE_CHECK_ARG(xl >= a.t_len && a.res_shift >= 0 && a.t_len + a.res_shift <= xl,
                       "residual_unit: x_len / res_shift leave the residual outside x");
        RAVE_CHECK_ARG(a.x_len <= 0 || a.x_sc >= xl, "residual_unit: x_len exceeds the row stride");
    }
    if (a.precision == RAVE_PREC_SPLIT16 || a.precision == RAVE_PREC_F32_RING || a.precision == RAVE_PREC_BF16X3)
        return residual_unit_split(a, stream);
    const int C = a.channels;
    UnitKArgs k{};
    k.x = a.x; k.y = a.y; k.w = a.weight;
    k.b1 = a.bias1; k.b2 = a.bias2; k.a0 = a.alpha0; k.a2 = a.alpha2;
    k.x_sb = a.x_sb; k.x_sc = a.x_sc; k.y_sb = a.y_sb; k.y_sc = a.y_sc;
    k.T = a.t_len; k.d = a.dilation; k.pad_l = a.pad_left;
    k.XL = a.x_len > 0 ? a.x_len : a.t_len;
    k.rsh = a.res_shift;
    const int BN = unit_bn(C), MT = unit_mt(C);
    k.ntiles = ceil_div(a.t_len, BN);
    k.W = BN + 2 * a.dilation;
    k.XWS = unit_stride(k.W, MT);
    k.HS = unit_stride(BN, MT);
    k.act = a.act; k.slope = a.leaky_slope;
    const int64_t xb = ((int64_t)(C - 1) * a.x_sc + k.XL) * 4;
    const int64_t yb = ((int64_t)(C - 1) * a.y_sc + a.t_len) * 4;
    RAVE_CHECK_ARG(xb < (1ll << 31) && yb < (1ll << 31), "residual_unit: tensors beyond 2 GiB per item");
    k.x_bytes = (int)xb; k.y_bytes = (int)yb;
    k.w_bytes = (int)(rave_unit_packed_size(C) * 4);
    k.bias_bytes = C * 4;
    if (!a.bias1) k.bias_bytes = 0;      // both biases present or both absent (conv_bias)
    RAVE_CHECK_ARG((a.bias1 == nullptr) == (a.bias2 == nullptr), "residual_unit: give both biases or none");
    RAVE_CHECK_ARG((size_t)std::max(C * k.XWS, C * k.HS) * 4 <= 160 * 1024,
                   "residual_unit: window exceeds LDS (dilation too large for this width)");
    const bool snake = a.act == RAVE_ACT_SNAKE;
    hipStream_t st = as_stream(stream);
    switch (C) {
        case 64: return unit_launch<64>(k, a.batch, snake, st);
        case 128: return unit_launch<128>(k, a.batch, snake, st);
        case 256: return unit_launch<256>(k, a.batch, snake, st);
        default: return unit_launch<512>(k, a.batch, snake, st);
    }
}
