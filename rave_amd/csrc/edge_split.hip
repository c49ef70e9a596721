// The two edges of the encode -> decode path, each one launch on the f16
// matrix cores (split-f16 arithmetic, RAVE_PREC_SPLIT16; see conv_split.hip):
//
//   rave_encoder_head   CachedPQMF.forward + RAVE.encode's band slice
//                       (rave/pqmf.py:269-273 + reverse_half :13-17,
//                       rave/model.py:613) feeding EncoderV2's first conv
//                       (rave/blocks.py:533-536, no activation before it), and
//                       the speaker concat of RAVE.encode (model.py:618-620)
//   rave_decoder_tail   GeneratorV2's last activation + conv + its
//                       `x * sigmoid(a) (+ noise) -> tanh` epilogue
//                       (rave/blocks.py:691-707) feeding CachedPQMF.inverse
//                       (rave/pqmf.py:275-284)
//
// Separately these are two launches each (PQMF + conv) whose intermediate
// (6 bands / 32 wave+amplitude channels, 1.5-8 MB) makes an HBM round trip,
// and each launch pays its own fill and drain; both GEMMs are small (K = 42
// and 544; K = 448 and 544).  Here a workgroup owns a run of frames and
// computes the intermediate for them plus the halo its consumer needs
// (head: the conv's 6 frames; tail: the synthesis filter's 33), keeping it in
// LDS as (hi, lo) f16 planes.
//
// Head analysis in phase-packed form: 16x16x32 MFMA rows are (phase p, band k)
// = 8p + k with A[8p + k][j'] = h_k[j' - 16p], so one column (frame pair) of the
// window B[j'][n] = x[32 n + j'] yields frames 2n and 2n + 1: the 6 bands fill
// 12 of 16 rows (the unpacked form computes 16 rows for 6 bands and half the
// frames per MFMA).
//
// F32 (rave_edge_args.precision = RAVE_PREC_F32_RING): the same kernels in
// exact fp32 -- every (hi, lo) plane pair becomes one fp32 plane in the same
// bytes, each 3-MFMA split-f16 group becomes eight v_mfma_f32_16x16x4 /
// v_mfma_f32_32x32x2 (lane slot g of a K-group of 8 holds K index 8g + e for
// MFMA e, on both operands), the filter image is fp32 (scale 1) and the conv
// weight the ring image (rave_conv1d_ring_pack_weight); no range guard.
//
// Ranges: every staged operand block is scaled by one power of two from the
// workgroup's maximum (PQMF filters: max |h 2^e| in [8, 16); signals: 2^-s
// with |v 2^-s| < 2^15), so no f16 half overflows; the epilogues undo the
// scales exactly.  The tail's synthesis input is tanh-bounded.
#include "common.h"

#include <algorithm>
#include <cmath>

namespace rave {

typedef _Float16 e_h8 __attribute__((ext_vector_type(8)));
typedef _Float16 e_h4 __attribute__((ext_vector_type(4)));
typedef float e_f32x4 __attribute__((ext_vector_type(4)));
typedef float e_f32x16 __attribute__((ext_vector_type(16)));
typedef float e_f32x8 __attribute__((ext_vector_type(8)));
typedef __bf16 e_b8 __attribute__((ext_vector_type(8)));
typedef __bf16 e_b4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ e_f32x8 e_ld8(const float* p) {    // 8 floats (two b128 LDS reads)
    const e_f32x4 u = *reinterpret_cast<const e_f32x4*>(p), v = *reinterpret_cast<const e_f32x4*>(p + 4);
    return e_f32x8{u[0], u[1], u[2], u[3], v[0], v[1], v[2], v[3]};
}

constexpr int kEdgeWaves = 8;
constexpr int kEdgeNT = 64 * kEdgeWaves;
constexpr int kEdgeK7 = 7;                         // edge conv taps (2 * kernel_size + 1)
constexpr int kEdgeKW = 544;                       // PQMF K extent (17 steps of 32)
constexpr int kEdgeFP = 552;                       // halves per filter row (conflict-free b128)
constexpr int kSynTapsE = 33;
constexpr int kAnaTapsE = 513;

// Host-split PQMF filter image (rave_encoder_head_pack_filter /
// rave_decoder_tail_pack_filter): the kernel's LDS layout verbatim -- hi plane
// [16 rows][kEdgeFP halves] then lo plane -- with the filter scaled by 2^e
// (max |h 2^e| in [8, 16)), followed by one float 2^-(e + 11).  A workgroup
// copies it with 16-byte loads instead of converting the fp32 filter.
constexpr int kEdgeFilterHalves = 2 * 16 * kEdgeFP;
constexpr int kEdgeFilterFloats = kEdgeFilterHalves / 2 + 4;

// launch geometry the host derives from the args
struct EdgeGeo {
    int tiles;                 // frame tiles per batch item
    int w_mb;                  // 32-row blocks of the packed conv weight (Mpad / 32)
    int w_bytes;               // bytes of the packed weight (fragments + row scales)
    int y_vec;                 // head: 16-byte output stores are aligned
    int64_t w_frag_floats;     // floats of fragments before the row scales
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t e_rsrc(const void* p, int64_t bytes) {
    const uint64_t v = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    const uint64_t u = ((uint64_t)hi << 32) | lo;
    const int nb = (int)std::min<int64_t>(bytes, 0x7FFFFFF0);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(u), (short)0,
                                             __builtin_amdgcn_readfirstlane(nb), 0x00020000);
}

__device__ __forceinline__ void e_split(float v, _Float16& hi, _Float16& lo) {
    hi = (_Float16)v;
    lo = (_Float16)((v - (float)hi) * 2048.0f);
}

// split-f16 conv weight image (rave_conv1d_split_pack_weight, 7 taps, stride 1):
// [chunk of 16 in-channels][32-row block mb][tap][hi|lo][64 lanes][8 halves],
// then one float row scale 2^-(e_m + 11) per padded row.  bf16x3
// (rave_conv1d_bf3_pack_weight): three planes per tap, [hi|lo|mid], scales 1.
struct EdgeW {
    __amdgpu_buffer_rsrc_t rs;
    int mb_count;                                   // Mpad / 32
    int np = 2;                                     // planes per tap
    __device__ unsigned off(int chunk, int mb, int tap, int plane, int lane) const {
        return (unsigned)((((chunk * mb_count + mb) * kEdgeK7 + tap) * np + plane) * 1024 + lane * 16);
    }
    __device__ e_h8 frag(int chunk, int mb, int tap, int plane, int lane) const {
        return __builtin_bit_cast(e_h8, __builtin_amdgcn_raw_buffer_load_b128(rs, off(chunk, mb, tap, plane, lane), 0, 0));
    }
    // ring image (F32): the same slots carry floats 0-3 (plane 0) and 4-7 (plane 1)
    __device__ static e_f32x8 f32(const e_h8& p0, const e_h8& p1) {
        const e_f32x4 u = __builtin_bit_cast(e_f32x4, p0), v = __builtin_bit_cast(e_f32x4, p1);
        return e_f32x8{u[0], u[1], u[2], u[3], v[0], v[1], v[2], v[3]};
    }
};

// Diagnostic stage cut (tools/probes/edge_probe.hip builds with -DRAVE_EDGE_STOP=n;
// off in the product): end the kernel after stage n, sinking one value so the
// work before it stays live.
#ifdef RAVE_EDGE_STOP
#define EDGE_STOP(n, v)                                                   \
    if (RAVE_EDGE_STOP == (n)) {                                          \
        if (threadIdx.x == 0) a.y[(int64_t)blockIdx.x] = (float)(v);      \
        return;                                                           \
    }
#else
#define EDGE_STOP(n, v)
#endif

template <int V> struct EdgeN {
    static constexpr int value = V;
};

// =================================================================== encoder head
// A workgroup owns kHF conv output frames [n0, n0 + kHF) of one batch item:
// bands for frames [g0, g0 + 32 kHAB) with g0 = n0 - conv pad (the conv's
// 6-frame halo included), analysis block i = frames g0 + 32 i + (0..31).
constexpr int kHF = 256;
constexpr int kHAB = kHF / 32 + 1;                  // analysis blocks (288 frames >= kHF + 6)
constexpr int kHBR = 32 * kHAB;                     // band-plane rows
constexpr int kHBP = 24;                            // halves per band-plane row (16 channels + 8)
constexpr int kHXS = 512 * (kHAB - 1) + 32 * 15 + kEdgeKW;   // window samples (5120 + 32)
__host__ __device__ constexpr int e_xi(int i) { return i + 8 * (i >> 7); }   // 8 halves of pad per 128
constexpr int kHXP = e_xi(kHXS) + 8;                // halves per window plane
constexpr int kHeadLds = (2 * 16 * kEdgeFP + 2 * kHXP + 2 * kHBR * kHBP) * 2 + 4 * kEdgeWaves * 4 + 16 +
                         kEdgeWaves * 64 * 4 * 4;        // + the split analysis block's partial sums
// bf16x3 analysis (AR = 2, round 6): three bf16 planes of the filter and of the
// audio window, the fp32 band planes and the exact-fp32 conv after them
constexpr int kHeadBaBand = (3 * 16 * kEdgeFP + 3 * kHXP) * 2;   // bytes before the fp32 band planes
static_assert(kHeadBaBand % 16 == 0, "band planes 16-byte aligned");
constexpr int kHeadLdsBa = kHeadBaBand + kHBR * kHBP * 4 + 4 * kEdgeWaves * 4 + 16 + kEdgeWaves * 64 * 4 * 4;

// AR: 0 split-f16, 1 exact fp32, 2 bf16x3 analysis (fp32 on the bf16 matrix
// cores: exact three-way split of the filter and of the audio, six
// v_mfma_f32_16x16x32_bf16 per 32-deep K-step) with the exact-fp32 conv
template <int AR>
__global__ __launch_bounds__(kEdgeNT) void encoder_head_kernel(rave_edge_args a, EdgeGeo geo) {
    constexpr bool FC = AR != 0;                     // exact-fp32 band planes and conv
    constexpr bool F32 = AR == 1, BA = AR == 2;      // analysis: exact fp32 / bf16x3
    const int tiles = geo.tiles;
    extern __shared__ __attribute__((aligned(16))) char e_smem[];
    _Float16* fh = reinterpret_cast<_Float16*>(e_smem);          // [16][kEdgeFP]
    _Float16* fl = fh + 16 * kEdgeFP;
    _Float16* xh = fl + 16 * kEdgeFP;                              // [kHXP] flat, padded
    _Float16* xl = xh + kHXP;
    _Float16* bh = BA ? reinterpret_cast<_Float16*>(e_smem + kHeadBaBand) : xl + kHXP;   // [kHBR][kHBP]
    _Float16* bl = bh + kHBR * kHBP;
    float* red = reinterpret_cast<float*>(bl + kHBR * kHBP);
    // BA: filter planes (hi, mid, lo) [16][kEdgeFP] and window planes (hi, mid, lo) [kHXP]
    __bf16* gbh = reinterpret_cast<__bf16*>(e_smem);
    __bf16* gbm = gbh + 16 * kEdgeFP;
    __bf16* gbl = gbm + 16 * kEdgeFP;
    __bf16* wbh = gbl + 16 * kEdgeFP;
    __bf16* wbm = wbh + kHXP;
    __bf16* wbl = wbm + kHXP;
    float* part = red + 4 * kEdgeWaves + 4;                        // [waves][64 lanes][4] (after the votes)
    // F32: one fp32 plane in the bytes of each (hi, lo) pair
    float* ff = reinterpret_cast<float*>(fh);                     // [16][kEdgeFP]
    float* xf = reinterpret_cast<float*>(xh);                     // [kHXP] flat, padded
    float* bf = reinterpret_cast<float*>(bh);                     // FC: [kHBR][kHBP]
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nmain = tiles * a.batch;

    const int lg = __builtin_amdgcn_readfirstlane(xcd_major(blockIdx.x, nmain));
    const int b = lg / tiles;
    const int tile = lg - b * tiles;
    const int n0 = tile * kHF;
    if (a.fill_channels > 0) {
        // the speaker concat of RAVE.encode: the batch item's tiles share its rows
        float* z = a.fill_y + (int64_t)b * a.f_sb;
        const int n = a.fill_channels * a.fill_t;
        for (int i = tile * kEdgeNT + tid; i < n; i += tiles * kEdgeNT) {
            const int c = i / a.fill_t, t = i - c * a.fill_t;
            z[(int64_t)c * a.f_sc + t] = a.fill_values[c];
        }
    }
    const int F = a.frames;
    const int T = F * 16;
    const int g0 = n0 - a.conv_pad_left;            // band frame of band-plane row 0
    const int s0 = 16 * g0 - a.pqmf_pad_left;       // audio sample of window sample 0

    unsigned char* vote = reinterpret_cast<unsigned char*>(red + 4 * kEdgeWaves);
    // ---- phase-packed filter image -> LDS (16-byte copies); audio window,
    // split optimistically (no scale) with a per-wave range vote
    {
        const e_h8* src = reinterpret_cast<const e_h8*>(a.filter);
        if constexpr (BA) {      // the exact-fp32 image, split into three bf16 planes on the way in
            for (int i = tid; i < kEdgeFilterHalves / 8; i += kEdgeNT) {
                e_b4 hi, mid, lo;
                bf3_split_pk(__builtin_bit_cast(e_f32x4, src[i]), hi, mid, lo);
                *reinterpret_cast<e_b4*>(gbh + 4 * i) = hi;
                *reinterpret_cast<e_b4*>(gbm + 4 * i) = mid;
                *reinterpret_cast<e_b4*>(gbl + 4 * i) = lo;
            }
        } else {
            e_h8* dst = reinterpret_cast<e_h8*>(fh);
            for (int i = tid; i < kEdgeFilterHalves / 8; i += kEdgeNT) dst[i] = src[i];
        }
    }
    const float f_unscale = a.filter[kEdgeFilterHalves / 2];        // 2^-(e + 11)
    constexpr int XT = (kHXS + kEdgeNT - 1) / kEdgeNT;             // 11
    const float* xb = a.x + (int64_t)b * a.x_sb;
    float xv[XT];
    float xmax = 0.f;
#pragma unroll
    for (int it = 0; it < XT; ++it) {
        const int i = tid + it * kEdgeNT;
        const int t = s0 + i;
        const float v = xb[min(max(t, 0), T - 1)];
        xv[it] = (i < kHXS && t >= 0 && t < T) ? v : 0.f;
        xmax = fmaxf(xmax, fabsf(xv[it]));
    }
#pragma unroll
    for (int it = 0; it < XT; ++it) {
        const int i = tid + it * kEdgeNT;
        if (i < kHXS) {
            if constexpr (BA) {
                const float v = xv[it];
                const __bf16 hi = (__bf16)v;
                const float r = v - (float)hi;
                const __bf16 mid = (__bf16)r;
                wbh[e_xi(i)] = hi;
                wbm[e_xi(i)] = mid;
                wbl[e_xi(i)] = (__bf16)(r - (float)mid);
            } else if constexpr (F32) {
                xf[e_xi(i)] = xv[it];
            } else {
                e_split(xv[it], xh[e_xi(i)], xl[e_xi(i)]);
            }
        }
    }
    if constexpr (AR == 0) vote_cast(vote, wave, xmax);
    // band-plane channels 8..15 stay zero (the conv chunk is 16 channels wide)
    for (int i = tid; i < kHBR; i += kEdgeNT) {
        if constexpr (FC) {
            *reinterpret_cast<e_f32x4*>(bf + i * kHBP + 8) = e_f32x4{0.f, 0.f, 0.f, 0.f};
            *reinterpret_cast<e_f32x4*>(bf + i * kHBP + 12) = e_f32x4{0.f, 0.f, 0.f, 0.f};
        } else {
            *reinterpret_cast<e_h8*>(bh + i * kHBP + 8) = e_h8{0, 0, 0, 0, 0, 0, 0, 0};
            *reinterpret_cast<e_h8*>(bl + i * kHBP + 8) = e_h8{0, 0, 0, 0, 0, 0, 0, 0};
        }
    }
    __syncthreads();
    float xs = 1.f;
    if (AR == 0 && __builtin_expect(vote_any<kEdgeWaves>(vote), 0)) {
        // rare: audio at 2^15 or beyond -- the window again as x 2^-s
        xs = ldexpf(1.f, -__builtin_amdgcn_readfirstlane(split_shift(block_max<kEdgeWaves>(xmax, red))));
#pragma unroll
        for (int it = 0; it < XT; ++it) {
            const int i = tid + it * kEdgeNT;
            if (i < kHXS) e_split(xv[it] * xs, xh[e_xi(i)], xl[e_xi(i)]);
        }
        __syncthreads();
    }
    EDGE_STOP(1, xh[tid] + fh[tid])

    // ---- analysis: block blk, column n = frame pair (frames 32 blk + 2n + p)
    const int g = lane >> 4, col = lane & 15;
    // three independent accumulator chains (one per product), summed at the end
    // BA: the six bf16 products of one 32-deep K-step, smallest first (A = filter
    // part, B = audio part): lo*hi, hi*lo, mid*mid, mid*hi, hi*mid, hi*hi
    auto ba_step = [&](int blk, int s, e_f32x4& c) __attribute__((always_inline)) {
        const int ka = col * kEdgeFP + 32 * s + 8 * g;
        const int xi = e_xi(512 * blk + 32 * col + 32 * s + 8 * g);
        const e_b8 fh8 = *reinterpret_cast<const e_b8*>(gbh + ka), fm8 = *reinterpret_cast<const e_b8*>(gbm + ka),
                   fl8 = *reinterpret_cast<const e_b8*>(gbl + ka);
        const e_b8 xh8 = *reinterpret_cast<const e_b8*>(wbh + xi), xm8 = *reinterpret_cast<const e_b8*>(wbm + xi),
                   xl8 = *reinterpret_cast<const e_b8*>(wbl + xi);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fl8, xh8, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh8, xl8, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fm8, xm8, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fm8, xh8, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh8, xm8, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh8, xh8, c, 0, 0, 0);
    };
    auto analysis_block = [&](int blk, e_f32x4& acc) __attribute__((always_inline)) {
        e_f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0;
        if constexpr (BA) {
            // two chains (even / odd K-steps), summed at the end
#pragma unroll
            for (int s = 0; s < kEdgeKW / 32; ++s) ba_step(blk, s, (s & 1) ? c1 : c0);
            acc = c0 + c1;
            return;
        }
        if constexpr (F32) {
#pragma unroll
            for (int s = 0; s < kEdgeKW / 32; ++s) {
                const e_f32x8 af = e_ld8(ff + col * kEdgeFP + 32 * s + 8 * g);
                const e_f32x8 xf8 = e_ld8(xf + e_xi(512 * blk + 32 * col + 32 * s + 8 * g));
#pragma unroll
                for (int e = 0; e < 8; e += 2) {
                    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(af[e], xf8[e], c0, 0, 0, 0);
                    c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(af[e + 1], xf8[e + 1], c1, 0, 0, 0);
                }
            }
            acc = c0 + c1;
            return;
        }
#pragma unroll
        for (int s = 0; s < kEdgeKW / 32; ++s) {
            const int ka = col * kEdgeFP + 32 * s + 8 * g;
            const e_h8 ah = *reinterpret_cast<const e_h8*>(fh + ka);
            const e_h8 al = *reinterpret_cast<const e_h8*>(fl + ka);
            const e_h8 a2 = ah * (_Float16)2048.0f;
            const int xi = e_xi(512 * blk + 32 * col + 32 * s + 8 * g);
            const e_h8 xh8 = *reinterpret_cast<const e_h8*>(xh + xi);
            const e_h8 xl8 = *reinterpret_cast<const e_h8*>(xl + xi);
            c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2, xh8, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, xl8, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, xh8, c2, 0, 0, 0);
        }
        acc = (c0 + c1) + c2;
    };
    // K-steps s0, s0 + waves, s0 + 2 waves of block blk (the block the waves share)
    auto analysis_steps = [&](int blk, e_f32x4& acc, int s0) __attribute__((always_inline)) {
        e_f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0;
#pragma unroll
        for (int j = 0; j < (kEdgeKW / 32 + kEdgeWaves - 1) / kEdgeWaves; ++j) {
            const int s = s0 + kEdgeWaves * j;
            if (s >= kEdgeKW / 32) break;               // (wave-uniform)
            if constexpr (BA) {
                ba_step(blk, s, c0);
            } else if constexpr (F32) {
                const e_f32x8 af = e_ld8(ff + col * kEdgeFP + 32 * s + 8 * g);
                const e_f32x8 xf8 = e_ld8(xf + e_xi(512 * blk + 32 * col + 32 * s + 8 * g));
#pragma unroll
                for (int e = 0; e < 8; e += 2) {
                    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(af[e], xf8[e], c0, 0, 0, 0);
                    c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(af[e + 1], xf8[e + 1], c1, 0, 0, 0);
                }
            } else {
                const int ka = col * kEdgeFP + 32 * s + 8 * g;
                const e_h8 ah = *reinterpret_cast<const e_h8*>(fh + ka);
                const e_h8 al = *reinterpret_cast<const e_h8*>(fl + ka);
                const e_h8 a2 = ah * (_Float16)2048.0f;
                const int xi = e_xi(512 * blk + 32 * col + 32 * s + 8 * g);
                const e_h8 xh8 = *reinterpret_cast<const e_h8*>(xh + xi);
                const e_h8 xl8 = *reinterpret_cast<const e_h8*>(xl + xi);
                c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2, xh8, c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, xl8, c1, 0, 0, 0);
                c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, xh8, c2, 0, 0, 0);
            }
        }
        acc = (c0 + c1) + c2;
    };
    // acc rows 4g + r = (p = g >> 1, k = 4 (g & 1) + r); value = band k of frame
    // g0 + 32 blk + 2 col + p (reverse_half, zero outside [0, F))
    const float unscale = f_unscale / xs;
    auto band_values = [&](int blk, const e_f32x4& acc, e_f32x4& v, float& m) __attribute__((always_inline)) {
        const int p = g >> 1;
        const int f = g0 + 32 * blk + 2 * col + p;
        const bool fok = f >= 0 && f < F;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int k = 4 * (g & 1) + r;
            float x = acc[r] * unscale;
            if ((k & 1) && !(f & 1)) x = -x;
            v[r] = fok ? x : 0.f;
            m = fmaxf(m, fabsf(v[r]));
        }
    };
    e_f32x4 acc0, acc1, v0, v1;
    float bmax = 0.f;
    analysis_block(wave, acc0);
    band_values(wave, acc0, v0, bmax);
    // the ninth block (kHAB = waves + 1): its K-steps split over every wave, the
    // partial sums added in wave order (fixed: reproducible) by wave 0, so that
    // no wave computes two whole blocks
    static_assert(kHAB == kEdgeWaves + 1, "one shared analysis block");
    {
        e_f32x4 pacc;
        analysis_steps(kEdgeWaves, pacc, wave);
        *reinterpret_cast<e_f32x4*>(part + (wave * 64 + lane) * 4) = pacc;
    }
    __syncthreads();
    const bool extra = wave == 0;
    if (extra) {
        acc1 = *reinterpret_cast<const e_f32x4*>(part + lane * 4);
#pragma unroll
        for (int w2 = 1; w2 < kEdgeWaves; ++w2) acc1 += *reinterpret_cast<const e_f32x4*>(part + (w2 * 64 + lane) * 4);
        band_values(kEdgeWaves, acc1, v1, bmax);
    }
    auto put_bands = [&](int blk, const e_f32x4& v, float bs) __attribute__((always_inline)) {
        const int row = 32 * blk + 2 * col + (g >> 1);
        if constexpr (FC) {
            *reinterpret_cast<e_f32x4*>(bf + row * kHBP + 4 * (g & 1)) = v;
            return;
        }
        e_h4 hv4, lv4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float u = v[r] * bs;
            const _Float16 hi = (_Float16)u;
            hv4[r] = hi;
            lv4[r] = (_Float16)((u - (float)hi) * 2048.0f);
        }
        *reinterpret_cast<e_h4*>(bh + row * kHBP + 4 * (g & 1)) = hv4;
        *reinterpret_cast<e_h4*>(bl + row * kHBP + 4 * (g & 1)) = lv4;
    };
    // the conv's weight fragments (no data dependence): in flight across the band barrier
    const EdgeW W{e_rsrc(a.weight, (int64_t)geo.w_bytes), geo.w_mb};
    const int MB = (a.conv_c_out + 31) / 32;        // 1 or 2 row blocks
    e_h8 wr[kEdgeK7][2][2];
#pragma unroll
    for (int q = 0; q < kEdgeK7; ++q)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int pl = 0; pl < 2; ++pl) wr[q][j][pl] = j < MB ? W.frag(0, j, q, pl, lane) : e_h8{};
    // band planes split optimistically, with a range vote (rare: a rescale by 2^-s)
    put_bands(wave, v0, 1.f);
    if (extra) put_bands(wave + kEdgeWaves, v1, 1.f);
    if constexpr (AR == 0) vote_cast(vote + 8, wave, bmax);
    __syncthreads();
    float bs = 1.f;
    if (AR == 0 && __builtin_expect(vote_any<kEdgeWaves>(vote + 8), 0)) {
        bs = ldexpf(1.f, -__builtin_amdgcn_readfirstlane(split_shift(block_max<kEdgeWaves>(bmax, red))));
        put_bands(wave, v0, bs);
        if (extra) put_bands(wave + kEdgeWaves, v1, bs);
        __syncthreads();
    }
    EDGE_STOP(2, bh[tid] + bl[tid])

    // ---- conv (7 taps, 16-channel chunk, rows 0..63): wave = 32 output columns
    const int h = lane >> 5, l32 = lane & 31;
    e_f32x16 acc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
#pragma unroll
    for (int q = 0; q < kEdgeK7; ++q) {
        const int row = 32 * wave + l32 + q;
        if constexpr (FC) {
            // K pairs of input channels (2e, 2e + 1) on the two lane halves: ceil(c_in / 2)
            // MFMAs per tap instead of 8 (the image's lane half 1 holds channels 8-15, all
            // zero for the <= 8 bands here; lane half 0 holds channels 0-7)
            const e_f32x8 x8 = e_ld8(bf + row * kHBP);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                if (j >= MB) break;
                const e_f32x8 w8 = EdgeW::f32(wr[q][j][0], wr[q][j][1]);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (2 * e >= a.conv_c_in) break;                    // (wave-uniform)
                    const float w_odd = __shfl(w8[2 * e + 1], l32);    // lane half 0's channel 2e + 1
                    const float wv = h ? w_odd : w8[2 * e];
                    const float xv = h ? x8[2 * e + 1] : x8[2 * e];
                    acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(xv, wv, acc[j], 0, 0, 0);
                }
            }
            continue;
        }
        const e_h8 xh8 = *reinterpret_cast<const e_h8*>(bh + row * kHBP + 8 * h);
        const e_h8 xl8 = *reinterpret_cast<const e_h8*>(bl + row * kHBP + 8 * h);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if (j >= MB) break;
            const e_h8 b2 = wr[q][j][0] * (_Float16)2048.0f;
            acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh8, b2, acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl8, wr[q][j][0], acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh8, wr[q][j][1], acc[j], 0, 0, 0);
        }
    }
    EDGE_STOP(3, acc[0][0] + acc[1][7])
    // epilogue: lane = output channel m, registers 4c..4c+3 = 4 consecutive frames
    const float* rsc = a.weight + geo.w_frag_floats;
    const float inv_bs = 1.0f / bs;
    float* yb = a.y + (int64_t)b * a.y_sb;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        if (j >= MB) break;
        const int m = 32 * j + l32;
        if (m >= a.conv_c_out) continue;
        const float rs = rsc[m] * inv_bs;
        const float bias = a.bias ? a.bias[m] : 0.f;
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) {
            const int t = n0 + 32 * wave + 8 * c4 + 4 * h;
            e_f32x4 v;
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = acc[j][4 * c4 + e] * rs + bias;
            float* dst = yb + (int64_t)m * a.y_sc + t;
            if (t + 3 < F && geo.y_vec) {
                *reinterpret_cast<e_f32x4*>(dst) = v;
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (t + e < F) dst[e] = v[e];
            }
        }
    }
}

// =================================================================== decoder tail
// A workgroup owns kTF synthesis frames [n0, n0 + kTF) of one batch item.
// The synthesis reads its input at frames [f0, f0 + kTF + 33) with f0 = n0 -
// synthesis pad: the conv computes kTB x 32 output frames from f0, from an
// act(x) window of kTB x 32 + 6 frames (channels-last planes, 64 channels).
constexpr int kTF = 256;
constexpr int kTB = (kTF + kSynTapsE + 31) / 32;    // conv column blocks (10)
constexpr int kTC = 64;                             // conv input channels
constexpr int kTXR = 32 * kTB + kEdgeK7 - 1;        // act(x) rows (326)
constexpr int kTXP = kTC + 8;                       // halves per act(x) row
constexpr int kTSW = kTF + kSynTapsE + 1;           // synthesis window rows (290)
constexpr int kTSP = 24;                            // halves per synthesis row
constexpr int kTPlane = 2 * kTXR * kTXP;            // halves of the two act(x) planes
static_assert(2 * kTSW * kTSP <= kTPlane, "synthesis planes reuse the act(x) planes");
constexpr int kTailLds = (2 * 16 * kEdgeFP + kTPlane) * 2 + 2 * kEdgeWaves * 4 + 16;
// bf16x3 (AR = 2): three act(x) planes from byte 0, no filter in LDS during
// the conv; after it (planes dead) the fp32 synthesis planes at 0, the K-split
// partial tiles after them, and the fp32 filter at kTailBfFilt
constexpr int kTailBfX = 3 * kTXR * kTXP * 2;                  // bytes of the three act(x) planes
constexpr int kTailBfFilt = 61440;
constexpr int kTailLdsBf = kTailBfX + 2 * kEdgeWaves * 4 + 16;
static_assert(kTailBfFilt >= 2 * kTSW * kTSP * 2 + kEdgeWaves * 16 * 64 * 4 &&
              kTailBfFilt + 16 * kEdgeFP * 4 <= kTailBfX, "bf16x3 tail LDS reuse");
// bf16x3 synthesis (RAVE_TAIL_BF3_SYN, round 6): the synthesis on the bf16
// matrix cores too -- three bf16 planes of the synthesis input at 0, the K-split
// partial tiles after them, the filter's three bf16 planes at kTailBsFilt (split
// in-kernel from the exact fp32 image); six v_mfma_f32_16x16x32_bf16 per 32-deep
// K-step instead of eight v_mfma_f32_16x16x4_f32 per 4-deep one
#ifndef RAVE_TAIL_BF3_SYN
#define RAVE_TAIL_BF3_SYN 1
#endif
constexpr int kTailBsFilt = 75776;
static_assert(kTailBsFilt >= 3 * kTSW * kTSP * 2 + kEdgeWaves * 16 * 64 * 4 &&
              kTailBsFilt + 3 * 16 * kEdgeFP * 2 <= kTailBfX, "bf16x3 synthesis LDS reuse");

// AR: 0 split-f16, 1 exact fp32, 2 bf16x3 conv (fp32 on the bf16 matrix cores,
// exact three-way operand split, six bf16 MFMAs per 16-deep K-step) with the
// exact-fp32 synthesis
template <bool SNAKE, bool AM, int AR>
__global__ __launch_bounds__(kEdgeNT) void decoder_tail_kernel(rave_edge_args a, EdgeGeo geo) {
    constexpr bool F32 = AR == 1, BF = AR == 2;
    constexpr bool BS = BF && RAVE_TAIL_BF3_SYN != 0;            // BS: bf16x3 synthesis stage
    constexpr bool FS = AR != 0 && !BS;                          // FS: exact-fp32 synthesis stage
    const int tiles = geo.tiles;
    extern __shared__ __attribute__((aligned(16))) char e_smem[];
    _Float16* fh = reinterpret_cast<_Float16*>(e_smem);          // [16][kEdgeFP] synthesis filter
    _Float16* fl = fh + 16 * kEdgeFP;
    _Float16* xh = BF ? fh : fl + 16 * kEdgeFP;                    // [kTXR][kTXP] act(x)
    _Float16* xl = xh + kTXR * kTXP;
    _Float16* xm = xl + kTXR * kTXP;                               // BF: the mid plane
    _Float16* sh = xh;                                             // [kTSW][kTSP] (after the conv)
    _Float16* sl = xh + kTSW * kTSP;
    float* red = reinterpret_cast<float*>(BF ? reinterpret_cast<char*>(e_smem) + kTailBfX
                                             : reinterpret_cast<char*>(xh + kTPlane));
    float* ff = reinterpret_cast<float*>(BF ? e_smem + kTailBfFilt : e_smem);   // FS: [16][kEdgeFP]
    float* xf = reinterpret_cast<float*>(xh);                     // F32: [kTXR][kTXP] act(x)
    float* sf = xf;                                                // FS: [kTSW][kTSP] (after the conv)
    // BS: synthesis input planes [kTSW][kTSP] (hi, lo, mid) and filter planes [16][kEdgeFP] (hi, mid, lo)
    __bf16* sbh = reinterpret_cast<__bf16*>(xh);
    __bf16* sbl = sbh + kTSW * kTSP;
    __bf16* sbm = sbl + kTSW * kTSP;
    __bf16* fbh = reinterpret_cast<__bf16*>(e_smem + kTailBsFilt);
    __bf16* fbm = fbh + 16 * kEdgeFP;
    __bf16* fbl = fbm + 16 * kEdgeFP;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nmain = tiles * a.batch;
    const int lg = __builtin_amdgcn_readfirstlane(xcd_major(blockIdx.x, nmain));
    const int b = lg / tiles;
    const int n0 = (lg - b * tiles) * kTF;
    const int F = a.frames;
    const int f0 = n0 - a.pqmf_pad_left;             // conv output frame of synthesis row 0
    const int x0 = f0 - a.conv_pad_left;             // input frame of act(x) row 0
    const float slope = a.leaky_slope;

    unsigned char* vote = reinterpret_cast<unsigned char*>(red + 2 * kEdgeWaves);
    // ---- the conv's first weight fragments (no data dependence): issued first
    constexpr int NPW = BF && !RAVE_BF3_W4 ? 3 : 2;   // weight fragments per tap (W4: fp32 image)
    const EdgeW W{e_rsrc(a.weight, (int64_t)geo.w_bytes), geo.w_mb, NPW};
    constexpr int KS = (kTC / 16) * kEdgeK7;          // 28 K-steps
    constexpr int RING = 4;
    e_h8 wr[RING][NPW];
#pragma unroll
    for (int s = 0; s < RING; ++s)
#pragma unroll
        for (int pl = 0; pl < NPW; ++pl) wr[s][pl] = W.frag(s / kEdgeK7, 0, s % kEdgeK7, pl, lane);
    // ---- synthesis filter image -> LDS (16-byte copies); act(x) in 4-channel
    // groups (coalesced along time), split optimistically with a range vote.
    // BF: the fp32 filter is held in registers through the conv (its LDS is
    // the act(x) planes' until then) and stored after it
    constexpr int FQ = (kEdgeFilterHalves / 8 + kEdgeNT - 1) / kEdgeNT;   // 16-byte pieces per thread
    e_h8 fq[BF ? FQ : 1];
    if constexpr (BF) {
        const e_h8* src = reinterpret_cast<const e_h8*>(a.filter);
#pragma unroll
        for (int i = 0; i < FQ; ++i) {
            const int k = tid + i * kEdgeNT;
            if (k < kEdgeFilterHalves / 8) fq[i] = src[k];
        }
    } else {
        const e_h8* src = reinterpret_cast<const e_h8*>(a.filter);
        e_h8* dst = reinterpret_cast<e_h8*>(fh);
        for (int i = tid; i < kEdgeFilterHalves / 8; i += kEdgeNT) dst[i] = src[i];
    }
    const float f_unscale = a.filter[kEdgeFilterHalves / 2];        // 2^-(e + 11)
    constexpr int NG = kTC / 4;                                      // 4-channel groups
    constexpr int XT = (NG * kTXR + kEdgeNT - 1) / kEdgeNT;          // 11
    const float* xb = a.x + (int64_t)b * a.x_sb;
    e_f32x4 xv[XT];
    float xmax = 0.f;
#pragma unroll
    for (int it = 0; it < XT; ++it) {
        const int i = tid + it * kEdgeNT;
        const int cg = i / kTXR, w = i - cg * kTXR;
        const int t = x0 + w;
        const bool ok = i < NG * kTXR && t >= 0 && t < F;
        const int tt = min(max(t, 0), F - 1);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int cc = min(4 * cg + e, kTC - 1);
            const float v = xb[(int64_t)cc * a.x_sc + tt];
            float r;
            if constexpr (SNAKE) {
                const float al = a.alpha[cc];
                r = v + (1.0f / (al + 1e-9f)) * sin_squared(al * v);
            } else {
                r = v > 0.f ? v : v * slope;
            }
            xv[it][e] = ok ? r : 0.f;
            xmax = fmaxf(xmax, fabsf(xv[it][e]));
        }
    }
    auto put_x = [&](float xs) __attribute__((always_inline)) {
#pragma unroll
        for (int it = 0; it < XT; ++it) {
            const int i = tid + it * kEdgeNT;
            if (i < NG * kTXR) {
                const int cg = i / kTXR, w = i - cg * kTXR;
                const e_f32x4 v = xv[it] * xs;
                if constexpr (F32) {
                    *reinterpret_cast<e_f32x4*>(xf + w * kTXP + 4 * cg) = v;
                    continue;
                }
                if constexpr (BF) {
                    e_b4 hi, mid, lo;
                    bf3_split_pk(v, hi, mid, lo);
                    *reinterpret_cast<e_b4*>(xh + w * kTXP + 4 * cg) = hi;
                    *reinterpret_cast<e_b4*>(xl + w * kTXP + 4 * cg) = lo;
                    *reinterpret_cast<e_b4*>(xm + w * kTXP + 4 * cg) = mid;
                    continue;
                }
                const e_h4 hi = __builtin_convertvector(v, e_h4);
                const e_h4 lo = __builtin_convertvector((v - __builtin_convertvector(hi, e_f32x4)) * 2048.0f, e_h4);
                *reinterpret_cast<e_h4*>(xh + w * kTXP + 4 * cg) = hi;
                *reinterpret_cast<e_h4*>(xl + w * kTXP + 4 * cg) = lo;
            }
        }
    };
    put_x(1.f);
    if constexpr (AR == 0) vote_cast(vote, wave, xmax);
    __syncthreads();
    float xs = 1.f;
    if (AR == 0 && __builtin_expect(vote_any<kEdgeWaves>(vote), 0)) {
        // rare: act(x) at 2^15 or beyond -- the window again as act(x) 2^-s
        xs = ldexpf(1.f, -__builtin_amdgcn_readfirstlane(split_shift(block_max<kEdgeWaves>(xmax, red))));
        put_x(xs);
        __syncthreads();
    }
    EDGE_STOP(1, xh[tid] + fh[tid])

    // ---- conv: 32 rows (16 wave + 16 amplitude channels, or 16 + padding),
    // K = 4 chunks x 7 taps.  Wave w owns column block w; the last two blocks
    // (8, 9) are split by K: wave w also takes block 8 + (w >> 2) over chunk w & 3
    // (its 7 K-steps share the main block's weight fragments), and the four
    // partial tiles of each meet in LDS in chunk order.
    static_assert(kTB == kEdgeWaves + 2 && KS == 4 * kEdgeK7, "tail conv balance");
    const int h = lane >> 5, l32 = lane & 31;
    e_f32x16 acc, acl, acc_x, acl_x;                  // main block, K-split block; hi x hi / lo-term chains
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = acl[r] = acc_x[r] = acl_x[r] = 0.f;
    const int xblk = kEdgeWaves + (wave >> 2), xchunk = wave & 3;
    auto mfma3 = [&](int row, int ch, const e_h8& b2, const e_h8& bh8, const e_h8& bl8, const e_h8& bm8,
                     e_f32x16& c0, e_f32x16& c1) __attribute__((always_inline)) {
        if constexpr (BF) {
            // smallest products first (A = act(x) part, B = weight part): lo*hi, hi*lo,
            // mid*mid, mid*hi, hi*mid, hi*hi -- all cross products but mid*lo, lo*mid, lo*lo
            const int xo = row * kTXP + 16 * ch + 8 * h;
            const e_b8 xh8 = *reinterpret_cast<const e_b8*>(xh + xo), xl8 = *reinterpret_cast<const e_b8*>(xl + xo),
                       xm8 = *reinterpret_cast<const e_b8*>(xm + xo);
            e_b8 wh, wl, wm;
            if constexpr (RAVE_BF3_W4) {     // the fp32 image's 8 values -> hi / mid / lo
                const e_f32x8 w8 = EdgeW::f32(bh8, bl8);
                wh = __builtin_convertvector(w8, e_b8);
                const e_f32x8 r = w8 - __builtin_convertvector(wh, e_f32x8);
                wm = __builtin_convertvector(r, e_b8);
                wl = __builtin_convertvector(r - __builtin_convertvector(wm, e_f32x8), e_b8);
            } else {
                wh = __builtin_bit_cast(e_b8, bh8);
                wl = __builtin_bit_cast(e_b8, bl8);
                wm = __builtin_bit_cast(e_b8, bm8);
            }
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xl8, wh, c0, 0, 0, 0);
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh8, wl, c0, 0, 0, 0);
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xm8, wm, c0, 0, 0, 0);
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xm8, wh, c0, 0, 0, 0);
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh8, wm, c0, 0, 0, 0);
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh8, wh, c0, 0, 0, 0);
            return;
        }
        if constexpr (F32) {
            const e_f32x8 x8 = e_ld8(xf + row * kTXP + 16 * ch + 8 * h);
            const e_f32x8 w8 = EdgeW::f32(bh8, bl8);
#pragma unroll
            for (int e = 0; e < 8; e += 2) {
                c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(x8[e], w8[e], c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(x8[e + 1], w8[e + 1], c1, 0, 0, 0);
            }
            return;
        }
        const e_h8 xh8 = *reinterpret_cast<const e_h8*>(xh + row * kTXP + 16 * ch + 8 * h);
        const e_h8 xl8 = *reinterpret_cast<const e_h8*>(xl + row * kTXP + 16 * ch + 8 * h);
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh8, b2, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl8, bh8, c1, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh8, bl8, c1, 0, 0, 0);
    };
#pragma unroll
    for (int s = 0; s < KS; ++s) {
        const int ch = s / kEdgeK7, q = s - ch * kEdgeK7;
        const e_h8 bh8 = wr[s % RING][0], bl8 = wr[s % RING][1], bm8 = wr[s % RING][NPW - 1];
        if (s + RING < KS) {
            const int s2 = s + RING;
#pragma unroll
            for (int pl = 0; pl < NPW; ++pl) wr[s % RING][pl] = W.frag(s2 / kEdgeK7, 0, s2 % kEdgeK7, pl, lane);
        }
        const e_h8 b2 = bh8 * (_Float16)2048.0f;
        mfma3(32 * wave + l32 + q, ch, b2, bh8, bl8, bm8, acc, acl);
        if (ch == xchunk) mfma3(32 * xblk + l32 + q, ch, b2, bh8, bl8, bm8, acc_x, acl_x);
    }
    acc += acl;
    acc_x += acl_x;
    __syncthreads();                                 // act(x) planes dead
    if constexpr (BS) {                              // the filter as three bf16 planes (read after the epilogue's barrier)
#pragma unroll
        for (int i = 0; i < FQ; ++i) {
            const int k = tid + i * kEdgeNT;
            if (k < kEdgeFilterHalves / 8) {
                e_b4 hi, mid, lo;
                bf3_split_pk(__builtin_bit_cast(e_f32x4, fq[i]), hi, mid, lo);
                *reinterpret_cast<e_b4*>(fbh + 4 * k) = hi;
                *reinterpret_cast<e_b4*>(fbm + 4 * k) = mid;
                *reinterpret_cast<e_b4*>(fbl + 4 * k) = lo;
            }
        }
    } else if constexpr (BF) {                       // the fp32 filter into its place (read after the epilogue's barrier)
        e_h8* dst = reinterpret_cast<e_h8*>(ff);
#pragma unroll
        for (int i = 0; i < FQ; ++i) {
            const int k = tid + i * kEdgeNT;
            if (k < kEdgeFilterHalves / 8) dst[k] = fq[i];
        }
    }
    // the K-split blocks' partial tiles -> LDS (past the synthesis planes), summed
    // in chunk order by waves 0 (block 8) and 4 (block 9)
    float* part = reinterpret_cast<float*>(xh + (BS ? 3 : 2) * kTSW * kTSP);
#pragma unroll
    for (int r = 0; r < 16; ++r) part[(wave * 16 + r) * 64 + lane] = acc_x[r];
    __syncthreads();
    const bool has_x = (wave & 3) == 0;
    if (has_x) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            float v = part[((wave + 0) * 16 + r) * 64 + lane];
#pragma unroll
            for (int c = 1; c < 4; ++c) v += part[((wave + c) * 16 + r) * 64 + lane];
            acc_x[r] = v;
        }
    }
    EDGE_STOP(2, acc[0] + acc_x[5])
    // ---- epilogue: wave/amplitude pairs -> x * sigmoid(a) (+ noise) -> tanh ->
    // reverse_half -> synthesis planes (zero outside [0, F))
    const float* rsc = a.weight + geo.w_frag_floats;
    const float rs = rsc[l32] / xs;                   // the conv's row scale and the act(x) range scale
    const float bias = (a.bias && l32 < a.conv_c_out) ? a.bias[l32] : 0.f;
    const float* nz = a.noise ? a.noise + (int64_t)b * a.n_sb : nullptr;
    // Lanes pair up across the 16-row halves (l32 and l32 ^ 16 hold the same
    // frames): the low lane finishes positions r < 8 of channel c = l32 & 15, the
    // high lane positions r >= 8, each taking the other half of the (wave,
    // amplitude) pair by one xor-shuffle -- every lane works, 8 outputs each.
    const int c_out = l32 & 15;
    const bool lo_half = l32 < 16;
    const float* nzc = nz ? nz + (int64_t)c_out * a.n_sc : nullptr;
    auto put_block = [&](int blk, const e_f32x16& c) __attribute__((always_inline)) {
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = c[r] * rs + bias;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const float recv = __shfl_xor(lo_half ? v[k + 8] : v[k], 16);
            const int r = lo_half ? k : k + 8;
            float out = lo_half ? v[k] : recv;              // the wave channel's value
            if constexpr (AM) {
                const float amp = lo_half ? recv : v[k + 8];  // its amplitude channel (+16)
                out = out * __builtin_amdgcn_rcpf(1.0f + __expf(-amp));
            }
            const int w = 32 * blk + 8 * (r >> 2) + 4 * h + (r & 3);
            const int f = f0 + w;
            const bool ok = f >= 0 && f < F;
            if (nzc && ok) out = out + nzc[f];
            // tanh(x) = 1 - 2 / (e^2x + 1): saturates to +-1 through inf / 0
            out = 1.0f - 2.0f * __builtin_amdgcn_rcpf(__expf(2.0f * out) + 1.0f);
            if ((c_out & 1) && !(f & 1)) out = -out;
            if (w < kTSW) {
                if constexpr (BS) {
                    const float v = ok ? out : 0.f;
                    const __bf16 hi = (__bf16)v;
                    const float r = v - (float)hi;
                    const __bf16 mid = (__bf16)r;
                    sbh[w * kTSP + c_out] = hi;
                    sbm[w * kTSP + c_out] = mid;
                    sbl[w * kTSP + c_out] = (__bf16)(r - (float)mid);
                } else if constexpr (FS) {
                    sf[w * kTSP + c_out] = ok ? out : 0.f;
                } else {
                    e_split(ok ? out : 0.f, sh[w * kTSP + c_out], sl[w * kTSP + c_out]);
                }
            }
        }
    };
    put_block(wave, acc);
    if (has_x) put_block(xblk, acc_x);
    __syncthreads();
    EDGE_STOP(3, sh[tid] + fl[tid])

    // ---- synthesis (as pqmf_synthesis_split_kernel): wave = 2 blocks of 16 frames
    const int g = lane >> 4, col = lane & 15;
    constexpr int BLK = kTF / (16 * kEdgeWaves);     // 2
    const int fb = wave * BLK * 16;
    e_f32x4 sacc[BLK], sac1[BLK], sac2[BLK];
#pragma unroll
    for (int q = 0; q < BLK; ++q) sacc[q] = sac1[q] = sac2[q] = e_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < kEdgeKW / 32; ++s) {
        const int ka = col * kEdgeFP + 32 * s + 8 * g;
        const int tap = 2 * s + (g >> 1);
        if constexpr (BS) {
            // smallest products first (A = filter part, B = signal part): lo*hi, hi*lo,
            // mid*mid, mid*hi, hi*mid, hi*hi
            const e_b8 fh8 = *reinterpret_cast<const e_b8*>(fbh + ka), fm8 = *reinterpret_cast<const e_b8*>(fbm + ka),
                       fl8 = *reinterpret_cast<const e_b8*>(fbl + ka);
#pragma unroll
            for (int q = 0; q < BLK; ++q) {
                const int xi = (fb + 16 * q + col + tap) * kTSP + 8 * (g & 1);
                const e_b8 bh8 = *reinterpret_cast<const e_b8*>(sbh + xi), bm8 = *reinterpret_cast<const e_b8*>(sbm + xi),
                           bl8 = *reinterpret_cast<const e_b8*>(sbl + xi);
                e_f32x4 c = sacc[q];
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fl8, bh8, c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh8, bl8, c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fm8, bm8, c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fm8, bh8, c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh8, bm8, c, 0, 0, 0);
                sacc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh8, bh8, c, 0, 0, 0);
            }
            continue;
        }
        if constexpr (FS) {
            const e_f32x8 af = e_ld8(ff + ka);
#pragma unroll
            for (int q = 0; q < BLK; ++q) {
                const e_f32x8 b8 = e_ld8(sf + (fb + 16 * q + col + tap) * kTSP + 8 * (g & 1));
#pragma unroll
                for (int e = 0; e < 8; e += 2) {
                    sacc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[e], b8[e], sacc[q], 0, 0, 0);
                    sac1[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[e + 1], b8[e + 1], sac1[q], 0, 0, 0);
                }
            }
            continue;
        }
        const e_h8 ah = *reinterpret_cast<const e_h8*>(fh + ka);
        const e_h8 al = *reinterpret_cast<const e_h8*>(fl + ka);
        const e_h8 a2 = ah * (_Float16)2048.0f;
#pragma unroll
        for (int q = 0; q < BLK; ++q) {
            const int xi = (fb + 16 * q + col + tap) * kTSP + 8 * (g & 1);
            const e_h8 b_h = *reinterpret_cast<const e_h8*>(sh + xi);
            const e_h8 b_l = *reinterpret_cast<const e_h8*>(sl + xi);
            sacc[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2, b_h, sacc[q], 0, 0, 0);
            sac1[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, b_l, sac1[q], 0, 0, 0);
            sac2[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, b_h, sac2[q], 0, 0, 0);
        }
    }
#pragma unroll
    for (int q = 0; q < BLK; ++q) sacc[q] = (sacc[q] + sac1[q]) + sac2[q];
    const float o = 16.f * f_unscale;
    float* yb = a.y + (int64_t)b * a.y_sb;
#pragma unroll
    for (int q = 0; q < BLK; ++q) {
        const int t = n0 + fb + q * 16 + col;
        if (t >= F) continue;
        const e_f32x4 v = {o * sacc[q][3], o * sacc[q][2], o * sacc[q][1], o * sacc[q][0]};
        *reinterpret_cast<e_f32x4*>(yb + (int64_t)t * 16 + 12 - 4 * g) = v;
    }
}

}  // namespace rave

using namespace rave;

// rave_conv1d_split_pack_weight of a 7-tap stride-1 conv: chunks of 16
// in-channels, Mpad = c_out rounded up to 128, fragments then row scales
// (np: weight planes per tap -- 2, or 3 for the bf16x3 image)
static EdgeGeo edge_geometry(const rave_edge_args& a, int frames_per_tile, int np = 2) {
    EdgeGeo g{};
    g.tiles = ceil_div(a.frames, frames_per_tile);
    const int nchunks = (a.conv_c_in + 15) / 16;
    const int mpad = ceil_div(a.conv_c_out, 128) * 128;
    g.w_mb = mpad / 32;
    g.w_frag_floats = (int64_t)nchunks * g.w_mb * kEdgeK7 * np * 256;
    g.w_bytes = (int)((g.w_frag_floats + mpad) * 4);
    g.y_vec = (reinterpret_cast<uintptr_t>(a.y) % 16 == 0) && a.y_sb % 4 == 0 && a.y_sc % 4 == 0;
    return g;
}

template <typename K>
static int edge_lds_attr(K kern, int lds, bool& done) {
    if (!done) {
        RAVE_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        done = true;
    }
    return RAVE_OK;
}

// ------------------------------------------------------------ filter images
static int edge_row_exponent(double amax) {   // max |h 2^e| in [8, 16)
    if (!(amax > 0.0)) return 0;
    int e = (int)std::floor(std::log2(16.0 / amax));
    while (std::ldexp(amax, e) >= 16.0) --e;
    while (std::ldexp(amax, e) < 8.0) ++e;
    return e;
}

// A[r][k] (16 rows x kEdgeKW, zero beyond) -> hi / lo planes + 2^-(e + 11);
// f32: one fp32 plane [16][kEdgeFP] in the same bytes, then 1
template <typename Fn>
static void edge_filter_image(Fn&& A, float* image, bool f32) {
    if (f32) {
        for (int r = 0; r < 16; ++r)
            for (int k = 0; k < kEdgeFP; ++k) image[r * kEdgeFP + k] = k < kEdgeKW ? A(r, k) : 0.f;
        image[kEdgeFilterHalves / 2] = 1.f;
        for (int i = kEdgeFilterHalves / 2 + 1; i < kEdgeFilterFloats; ++i) image[i] = 0.f;
        return;
    }
    double amax = 0.0;
    for (int r = 0; r < 16; ++r)
        for (int k = 0; k < kEdgeKW; ++k) amax = std::max(amax, std::fabs((double)A(r, k)));
    const int e = edge_row_exponent(amax);
    _Float16* hi = reinterpret_cast<_Float16*>(image);
    _Float16* lo = hi + 16 * kEdgeFP;
    for (int r = 0; r < 16; ++r)
        for (int k = 0; k < kEdgeFP; ++k) {
            const float v = k < kEdgeKW ? (float)std::ldexp((double)A(r, k), e) : 0.f;
            const _Float16 vh = (_Float16)v;
            hi[r * kEdgeFP + k] = vh;
            lo[r * kEdgeFP + k] = (_Float16)((v - (float)vh) * 2048.0f);
        }
    image[kEdgeFilterHalves / 2] = (float)std::ldexp(1.0, -(e + 11));
    for (int i = kEdgeFilterHalves / 2 + 1; i < kEdgeFilterFloats; ++i) image[i] = 0.f;
}

static int head_pack(const float* hkf, int n_band, int taps, int n_out_bands, float* image, bool f32) {
    RAVE_CHECK_ARG(hkf && image, "encoder_head_pack_filter: null pointer");
    if (n_band != 16 || taps != kAnaTapsE || n_out_bands < 1 || n_out_bands > 8) {
        set_error("encoder_head_pack_filter: built for 16 bands, 513 taps, <= 8 output bands");
        return RAVE_ERR_UNSUPPORTED;
    }
    // row 8p + k, K index j: h_k[j - 16 p] (phase p = 0, 1)
    edge_filter_image([&](int r, int j) -> float {
        const int p = r >> 3, k = r & 7, jj = j - 16 * p;
        return (k < n_out_bands && jj >= 0 && jj < taps) ? hkf[(int64_t)k * taps + jj] : 0.f;
    }, image, f32);
    return RAVE_OK;
}
extern "C" int rave_encoder_head_pack_filter(const float* hkf, int n_band, int taps, int n_out_bands, float* image) {
    return head_pack(hkf, n_band, taps, n_out_bands, image, false);
}
extern "C" int rave_encoder_head_pack_filter_f32(const float* hkf, int n_band, int taps, int n_out_bands,
                                                 float* image) {
    return head_pack(hkf, n_band, taps, n_out_bands, image, true);
}

static int tail_pack(const float* hki, int n_band, int taps, float* image, bool f32) {
    RAVE_CHECK_ARG(hki && image, "decoder_tail_pack_filter: null pointer");
    if (n_band != 16 || taps != kSynTapsE) {
        set_error("decoder_tail_pack_filter: built for 16 bands, 33 taps");
        return RAVE_ERR_UNSUPPORTED;
    }
    // row m, K index tap * 16 + c: hki[m][c][tap]
    edge_filter_image([&](int m, int k) -> float {
        const int tap = k >> 4, c = k & 15;
        return tap < taps ? hki[((int64_t)m * n_band + c) * taps + tap] : 0.f;
    }, image, f32);
    return RAVE_OK;
}
extern "C" int rave_decoder_tail_pack_filter(const float* hki, int n_band, int taps, float* image) {
    return tail_pack(hki, n_band, taps, image, false);
}
extern "C" int rave_decoder_tail_pack_filter_f32(const float* hki, int n_band, int taps, float* image) {
    return tail_pack(hki, n_band, taps, image, true);
}

// rave_edge_args.precision: 0 / RAVE_PREC_SPLIT16 (split-f16) or RAVE_PREC_F32_RING (exact fp32);
// the tail also RAVE_PREC_BF16X3 (bf16x3 conv, exact-fp32 synthesis)
static int edge_prec(const rave_edge_args& a, bool& f32, bool allow_bf3 = false) {
    f32 = a.precision == RAVE_PREC_F32_RING;
    if (a.precision != 0 && a.precision != RAVE_PREC_SPLIT16 && !f32 &&
        !(allow_bf3 && a.precision == RAVE_PREC_BF16X3)) {
        set_error(allow_bf3 ? "edge: precision must be RAVE_PREC_SPLIT16, RAVE_PREC_F32_RING or RAVE_PREC_BF16X3"
                            : "edge: precision must be RAVE_PREC_SPLIT16 or RAVE_PREC_F32_RING");
        return RAVE_ERR_ARG;
    }
    return RAVE_OK;
}

extern "C" int rave_encoder_head(const rave_edge_args* p, void* stream) {
    RAVE_CHECK_ARG(p && p->x && p->y && p->weight && p->filter, "encoder_head: null pointer");
    const rave_edge_args& a = *p;
    RAVE_CHECK_ARG(a.batch > 0 && a.frames > 0, "encoder_head: empty shape");
    if (a.conv_kernel != kEdgeK7 || a.conv_c_in < 1 || a.conv_c_in > 8 || a.conv_c_out < 1 || a.conv_c_out > 64 ||
        a.conv_pad_left < 0 || a.conv_pad_left > kEdgeK7 - 1 || a.pqmf_taps != kAnaTapsE) {
        set_error("encoder_head: built for RAVE's 513-tap analysis, <= 8 bands and a 7-tap conv to <= 64 channels");
        return RAVE_ERR_UNSUPPORTED;
    }
    RAVE_CHECK_ARG(a.fill_channels == 0 || (a.fill_y && a.fill_values && a.fill_t > 0),
                   "encoder_head: fill needs fill_y, fill_values and fill_t");
    if (a.act != RAVE_ACT_NONE) {   // EncoderV2's first conv has no input activation (rave/blocks.py:533-536)
        set_error("encoder_head: the fused analysis + first conv applies no input activation (act must be RAVE_ACT_NONE)");
        return RAVE_ERR_UNSUPPORTED;
    }
    // RAVE_PREC_BF16X3: the analysis in bf16x3, the conv in exact fp32 (the
    // exact-fp32 filter image and the ring weight image, as RAVE_PREC_F32_RING)
    bool f32;
    int rc = edge_prec(a, f32, true);
    if (rc != RAVE_OK) return rc;
    const int ar = a.precision == RAVE_PREC_BF16X3 ? 2 : f32 ? 1 : 0;
    const EdgeGeo g = edge_geometry(a, kHF);
    static bool attr[3] = {false, false, false};
    auto kern = ar == 2 ? encoder_head_kernel<2> : ar == 1 ? encoder_head_kernel<1> : encoder_head_kernel<0>;
    const int lds = ar == 2 ? kHeadLdsBa : kHeadLds;
    rc = edge_lds_attr(kern, lds, attr[ar]);
    if (rc != RAVE_OK) return rc;
    const int grid = g.tiles * a.batch;
    launch(kern, dim3(grid), dim3(kEdgeNT), (uint32_t)lds, as_stream(stream), a, g);
    return launch_status("encoder_head_kernel");
}

extern "C" int rave_decoder_tail(const rave_edge_args* p, void* stream) {
    RAVE_CHECK_ARG(p && p->x && p->y && p->weight && p->filter, "decoder_tail: null pointer");
    const rave_edge_args& a = *p;
    RAVE_CHECK_ARG(a.batch > 0 && a.frames > 0, "decoder_tail: empty shape");
    if (a.conv_kernel != kEdgeK7 || a.conv_c_in != kTC || (a.conv_c_out != 16 && a.conv_c_out != 32) ||
        a.conv_pad_left < 0 || a.conv_pad_left > kEdgeK7 - 1 || a.pqmf_taps != kSynTapsE ||
        (a.mode != 1 && a.mode != 2) || (a.mode == 1) != (a.conv_c_out == 32)) {
        set_error("decoder_tail: built for a 7-tap conv 64 -> 32 (amplitude modulation) or 64 -> 16 "
                  "into RAVE's 33-tap synthesis");
        return RAVE_ERR_UNSUPPORTED;
    }
    RAVE_CHECK_ARG(a.act == RAVE_ACT_LEAKY || (a.act == RAVE_ACT_SNAKE && a.alpha),
                   "decoder_tail: act must be RAVE_ACT_LEAKY or RAVE_ACT_SNAKE (with alpha)");
    RAVE_CHECK_ARG(reinterpret_cast<uintptr_t>(a.y) % 16 == 0 && a.y_sb % 4 == 0,
                   "decoder_tail: output must be 16-byte aligned");
    bool f32;
    int rc = edge_prec(a, f32, true);
    if (rc != RAVE_OK) return rc;
    const bool bf = a.precision == RAVE_PREC_BF16X3;
    const int ar = bf ? 2 : f32 ? 1 : 0;
    const EdgeGeo g = edge_geometry(a, kTF, bf && !RAVE_BF3_W4 ? 3 : 2);
    const dim3 grid(g.tiles * a.batch);
    const bool snake = a.act == RAVE_ACT_SNAKE, am = a.mode == 1;
    auto pick = [&](auto art) {
        constexpr int AR = decltype(art)::value;
        return snake ? (am ? decoder_tail_kernel<true, true, AR> : decoder_tail_kernel<true, false, AR>)
                     : (am ? decoder_tail_kernel<false, true, AR> : decoder_tail_kernel<false, false, AR>);
    };
    auto kern = ar == 2 ? pick(EdgeN<2>{}) : ar == 1 ? pick(EdgeN<1>{}) : pick(EdgeN<0>{});
    const int lds = bf ? kTailLdsBf : kTailLds;
    static bool attr[12] = {false, false, false, false, false, false, false, false, false, false, false, false};
    rc = edge_lds_attr(kern, lds, attr[4 * ar + 2 * snake + am]);
    if (rc != RAVE_OK) return rc;
    launch(kern, grid, dim3(kEdgeNT), (uint32_t)lds, as_stream(stream), a, g);
    return launch_status("decoder_tail_kernel");
}
