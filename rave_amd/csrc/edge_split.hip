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
// Ranges: every staged operand block is scaled by one power of two from the
// workgroup's maximum (PQMF filters: max |h 2^e| in [8, 16); signals: 2^-s
// with |v 2^-s| < 2^15), so no f16 half overflows; the epilogues undo the
// scales exactly.  The tail's synthesis input is tanh-bounded.
#include "common.h"

#include <algorithm>

namespace rave {

typedef _Float16 e_h8 __attribute__((ext_vector_type(8)));
typedef _Float16 e_h4 __attribute__((ext_vector_type(4)));
typedef float e_f32x4 __attribute__((ext_vector_type(4)));
typedef float e_f32x16 __attribute__((ext_vector_type(16)));

constexpr int kEdgeWaves = 8;
constexpr int kEdgeNT = 64 * kEdgeWaves;
constexpr int kEdgeK7 = 7;                         // edge conv taps (2 * kernel_size + 1)
constexpr int kEdgeKW = 544;                       // PQMF K extent (17 steps of 32)
constexpr int kEdgeFP = 552;                       // halves per filter row (conflict-free b128)
constexpr int kSynTapsE = 33;
constexpr int kAnaTapsE = 513;

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

// 2^e with max |h 2^e| in [8, 16) for a filter maximum m (1 if m == 0)
__device__ __forceinline__ float e_filter_scale(float m) {
    if (!(m > 0.f)) return 1.f;
    int e;
    (void)frexpf(m, &e);
    return ldexpf(1.f, 4 - e);
}

// workgroup maxima of two per-thread values through `red` (2 * kEdgeWaves floats)
__device__ __forceinline__ void e_block_max2(float& a, float& b, float* red) {
    a = wave_max(a);
    b = wave_max(b);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) {
        red[wave] = a;
        red[kEdgeWaves + wave] = b;
    }
    __syncthreads();
    float ma = red[0], mb = red[kEdgeWaves];
#pragma unroll
    for (int w = 1; w < kEdgeWaves; ++w) {
        ma = fmaxf(ma, red[w]);
        mb = fmaxf(mb, red[kEdgeWaves + w]);
    }
    a = ma;
    b = mb;
}

// split-f16 conv weight image (rave_conv1d_split_pack_weight, 7 taps, stride 1):
// [chunk of 16 in-channels][32-row block mb][tap][hi|lo][64 lanes][8 halves],
// then one float row scale 2^-(e_m + 11) per padded row
struct EdgeW {
    __amdgpu_buffer_rsrc_t rs;
    int mb_count;                                   // Mpad / 32
    __device__ unsigned off(int chunk, int mb, int tap, int plane, int lane) const {
        return (unsigned)((((chunk * mb_count + mb) * kEdgeK7 + tap) * 2 + plane) * 1024 + lane * 16);
    }
    __device__ e_h8 frag(int chunk, int mb, int tap, int plane, int lane) const {
        return __builtin_bit_cast(e_h8, __builtin_amdgcn_raw_buffer_load_b128(rs, off(chunk, mb, tap, plane, lane), 0, 0));
    }
};

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
constexpr int kHeadLds = (2 * 16 * kEdgeFP + 2 * kHXP + 2 * kHBR * kHBP) * 2 + 4 * kEdgeWaves * 4;

__global__ __launch_bounds__(kEdgeNT) void encoder_head_kernel(rave_edge_args a, EdgeGeo geo) {
    const int tiles = geo.tiles;
    extern __shared__ __attribute__((aligned(16))) char e_smem[];
    _Float16* fh = reinterpret_cast<_Float16*>(e_smem);          // [16][kEdgeFP]
    _Float16* fl = fh + 16 * kEdgeFP;
    _Float16* xh = fl + 16 * kEdgeFP;                              // [kHXP] flat, padded
    _Float16* xl = xh + kHXP;
    _Float16* bh = xl + kHXP;                                      // [kHBR][kHBP]
    _Float16* bl = bh + kHBR * kHBP;
    float* red = reinterpret_cast<float*>(bl + kHBR * kHBP);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nmain = tiles * a.batch;

    if ((int)blockIdx.x >= nmain) {
        // the speaker concat of RAVE.encode: one workgroup per batch item
        const int b = blockIdx.x - nmain;
        float* z = a.fill_y + (int64_t)b * a.f_sb;
        const int n = a.fill_channels * a.fill_t;
        for (int i = tid; i < n; i += kEdgeNT) {
            const int c = i / a.fill_t, t = i - c * a.fill_t;
            z[(int64_t)c * a.f_sc + t] = a.fill_values[c];
        }
        return;
    }
    const int lg = __builtin_amdgcn_readfirstlane(xcd_major(blockIdx.x, nmain));
    const int b = lg / tiles;
    const int n0 = (lg - b * tiles) * kHF;
    const int F = a.frames;
    const int T = F * 16;
    const int NB = a.conv_c_in;                     // bands the encoder reads (<= 8)
    const int g0 = n0 - a.conv_pad_left;            // band frame of band-plane row 0
    const int s0 = 16 * g0 - a.pqmf_pad_left;       // audio sample of window sample 0

    // ---- operands into registers: phase-packed filter rows, audio window
    // filter row 8p + k, K index j: h_k[j - 16 p] (zero outside [0, 513), k >= NB)
    constexpr int HT = (16 * kEdgeKW + kEdgeNT - 1) / kEdgeNT;    // 17
    float hv[HT];
    float amax = 0.f;
#pragma unroll
    for (int it = 0; it < HT; ++it) {
        const int i = tid + it * kEdgeNT;
        const int r = i / kEdgeKW, j = i - r * kEdgeKW;
        const int p = r >> 3, k = r & 7, jj = j - 16 * p;
        const bool ok = k < NB && jj >= 0 && jj < kAnaTapsE;
        const float v = a.filter[(int64_t)min(k, NB - 1) * kAnaTapsE + min(max(jj, 0), kAnaTapsE - 1)];
        hv[it] = ok ? v : 0.f;
        amax = fmaxf(amax, fabsf(hv[it]));
    }
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
    e_block_max2(amax, xmax, red);
    const float sc = e_filter_scale(amax);
    const float xs = ldexpf(1.f, -split_shift(xmax));
#pragma unroll
    for (int it = 0; it < HT; ++it) {
        const int i = tid + it * kEdgeNT;
        const int r = i / kEdgeKW, j = i - r * kEdgeKW;
        e_split(hv[it] * sc, fh[r * kEdgeFP + j], fl[r * kEdgeFP + j]);
    }
#pragma unroll
    for (int it = 0; it < XT; ++it) {
        const int i = tid + it * kEdgeNT;
        if (i < kHXS) e_split(xv[it] * xs, xh[e_xi(i)], xl[e_xi(i)]);
    }
    // band-plane channels 8..15 stay zero (the conv chunk is 16 channels wide)
    for (int i = tid; i < kHBR; i += kEdgeNT) {
        *reinterpret_cast<e_h8*>(bh + i * kHBP + 8) = e_h8{0, 0, 0, 0, 0, 0, 0, 0};
        *reinterpret_cast<e_h8*>(bl + i * kHBP + 8) = e_h8{0, 0, 0, 0, 0, 0, 0, 0};
    }
    __syncthreads();

    // ---- analysis: block blk, column n = frame pair (frames 32 blk + 2n + p)
    const int g = lane >> 4, col = lane & 15;
    auto analysis_block = [&](int blk, e_f32x4& acc) __attribute__((always_inline)) {
        acc = e_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < kEdgeKW / 32; ++s) {
            const int ka = col * kEdgeFP + 32 * s + 8 * g;
            const e_h8 ah = *reinterpret_cast<const e_h8*>(fh + ka);
            const e_h8 al = *reinterpret_cast<const e_h8*>(fl + ka);
            const e_h8 a2 = ah * (_Float16)2048.0f;
            const int xi = e_xi(512 * blk + 32 * col + 32 * s + 8 * g);
            const e_h8 xh8 = *reinterpret_cast<const e_h8*>(xh + xi);
            const e_h8 xl8 = *reinterpret_cast<const e_h8*>(xl + xi);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2, xh8, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, xl8, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, xh8, acc, 0, 0, 0);
        }
    };
    // acc rows 4g + r = (p = g >> 1, k = 4 (g & 1) + r); value = band k of frame
    // g0 + 32 blk + 2 col + p (reverse_half, zero outside [0, F))
    const float unscale = 1.0f / (sc * 2048.0f * xs);
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
    const bool extra = wave + kEdgeWaves < kHAB;
    if (extra) {
        analysis_block(wave + kEdgeWaves, acc1);
        band_values(wave + kEdgeWaves, acc1, v1, bmax);
    }
    float dummy = 0.f;
    e_block_max2(bmax, dummy, red + 2 * kEdgeWaves);
    const float bs = ldexpf(1.f, -split_shift(bmax));             // band planes' range scale
    auto put_bands = [&](int blk, const e_f32x4& v) __attribute__((always_inline)) {
        const int row = 32 * blk + 2 * col + (g >> 1);
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
    put_bands(wave, v0);
    if (extra) put_bands(wave + kEdgeWaves, v1);
    __syncthreads();

    // ---- conv (7 taps, 16-channel chunk, rows 0..63): wave = 32 output columns
    const EdgeW W{e_rsrc(a.weight, (int64_t)geo.w_bytes), geo.w_mb};
    const int h = lane >> 5, l32 = lane & 31;
    const int MB = (a.conv_c_out + 31) / 32;        // 1 or 2 row blocks
    e_f32x16 acc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    e_h8 wr[kEdgeK7][2][2];
#pragma unroll
    for (int q = 0; q < kEdgeK7; ++q)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int pl = 0; pl < 2; ++pl) wr[q][j][pl] = j < MB ? W.frag(0, j, q, pl, lane) : e_h8{};
#pragma unroll
    for (int q = 0; q < kEdgeK7; ++q) {
        const int row = 32 * wave + l32 + q;
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
constexpr int kTailLds = (2 * 16 * kEdgeFP + kTPlane) * 2 + 2 * kEdgeWaves * 4;

template <bool SNAKE, bool AM>
__global__ __launch_bounds__(kEdgeNT) void decoder_tail_kernel(rave_edge_args a, EdgeGeo geo) {
    const int tiles = geo.tiles;
    extern __shared__ __attribute__((aligned(16))) char e_smem[];
    _Float16* fh = reinterpret_cast<_Float16*>(e_smem);          // [16][kEdgeFP] synthesis filter
    _Float16* fl = fh + 16 * kEdgeFP;
    _Float16* xh = fl + 16 * kEdgeFP;                              // [kTXR][kTXP] act(x)
    _Float16* xl = xh + kTXR * kTXP;
    _Float16* sh = xh;                                             // [kTSW][kTSP] (after the conv)
    _Float16* sl = xh + kTSW * kTSP;
    float* red = reinterpret_cast<float*>(xh + kTPlane);
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

    // ---- operands into registers: synthesis filter (K = tap * 16 + c), act(x)
    constexpr int KD = 16 * kSynTapsE;               // 528
    constexpr int HT = (16 * KD + kEdgeNT - 1) / kEdgeNT;   // 17 (coalesced reads of hki rows)
    float hv[HT];
    float amax = 0.f;
#pragma unroll
    for (int it = 0; it < HT; ++it) {
        const int i = min(tid + it * kEdgeNT, 16 * KD - 1);
        hv[it] = a.filter[i];                        // hki[m][c][tap], i = m*528 + c*33 + tap
        amax = fmaxf(amax, fabsf(hv[it]));
    }
    constexpr int XT = (kTC * kTXR + kEdgeNT - 1) / kEdgeNT;   // 41
    const float* xb = a.x + (int64_t)b * a.x_sb;
    float xv[XT];
    float xmax = 0.f;
#pragma unroll
    for (int it = 0; it < XT; ++it) {
        const int i = tid + it * kEdgeNT;
        const int c = i / kTXR, w = i - c * kTXR;
        const int t = x0 + w;
        const bool ok = i < kTC * kTXR && t >= 0 && t < F;
        const int cc = min(c, kTC - 1);
        const float v = xb[(int64_t)cc * a.x_sc + min(max(t, 0), F - 1)];
        float r = v;
        if constexpr (SNAKE) {
            const float al = a.alpha[cc];
            r = v + (1.0f / (al + 1e-9f)) * sin_squared(al * v);
        } else {
            r = v > 0.f ? v : v * slope;
        }
        xv[it] = ok ? r : 0.f;
        xmax = fmaxf(xmax, fabsf(xv[it]));
    }
    e_block_max2(amax, xmax, red);
    const float sc = e_filter_scale(amax);
    const float xs = ldexpf(1.f, -split_shift(xmax));
#pragma unroll
    for (int it = 0; it < HT; ++it) {
        const int i = tid + it * kEdgeNT;
        if (i < 16 * KD) {
            const int m = i / KD, rem = i - m * KD;
            const int c = rem / kSynTapsE, tap = rem - c * kSynTapsE;
            const int k = tap * 16 + c;
            e_split(hv[it] * sc, fh[m * kEdgeFP + k], fl[m * kEdgeFP + k]);
        }
    }
    for (int i = tid; i < 16 * (kEdgeKW - KD); i += kEdgeNT) {     // K rows 528..543
        const int m = i / (kEdgeKW - KD), k = KD + i % (kEdgeKW - KD);
        fh[m * kEdgeFP + k] = (_Float16)0.f;
        fl[m * kEdgeFP + k] = (_Float16)0.f;
    }
#pragma unroll
    for (int it = 0; it < XT; ++it) {
        const int i = tid + it * kEdgeNT;
        if (i < kTC * kTXR) {
            const int c = i / kTXR, w = i - c * kTXR;
            e_split(xv[it] * xs, xh[w * kTXP + c], xl[w * kTXP + c]);
        }
    }
    __syncthreads();

    // ---- conv: 32 rows (16 wave + 16 amplitude channels, or 16 + padding),
    // K = 4 chunks x 7 taps; wave w owns column blocks w (and w + 8)
    const EdgeW W{e_rsrc(a.weight, (int64_t)geo.w_bytes), geo.w_mb};
    const int h = lane >> 5, l32 = lane & 31;
    e_f32x16 acc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    const bool two = wave + kEdgeWaves < kTB;
    constexpr int KS = (kTC / 16) * kEdgeK7;          // 28 K-steps
    constexpr int RING = 4;
    e_h8 wr[RING][2];
#pragma unroll
    for (int s = 0; s < RING; ++s)
#pragma unroll
        for (int pl = 0; pl < 2; ++pl) wr[s][pl] = W.frag(s / kEdgeK7, 0, s % kEdgeK7, pl, lane);
    auto kstep = [&](int s, auto nblk) __attribute__((always_inline)) {
        constexpr int NBK = decltype(nblk)::value;
        const int ch = s / kEdgeK7, q = s - ch * kEdgeK7;
        const e_h8 bh8 = wr[s % RING][0], bl8 = wr[s % RING][1];
        if (s + RING < KS) {
            const int s2 = s + RING;
#pragma unroll
            for (int pl = 0; pl < 2; ++pl) wr[s % RING][pl] = W.frag(s2 / kEdgeK7, 0, s2 % kEdgeK7, pl, lane);
        }
        const e_h8 b2 = bh8 * (_Float16)2048.0f;
#pragma unroll
        for (int j = 0; j < NBK; ++j) {
            const int row = 32 * (wave + kEdgeWaves * j) + l32 + q;
            const e_h8 xh8 = *reinterpret_cast<const e_h8*>(xh + row * kTXP + 16 * ch + 8 * h);
            const e_h8 xl8 = *reinterpret_cast<const e_h8*>(xl + row * kTXP + 16 * ch + 8 * h);
            acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh8, b2, acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl8, bh8, acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh8, bl8, acc[j], 0, 0, 0);
        }
    };
    if (two) {
#pragma unroll
        for (int s = 0; s < KS; ++s) kstep(s, EdgeN<2>{});
    } else {
#pragma unroll
        for (int s = 0; s < KS; ++s) kstep(s, EdgeN<1>{});
    }
    // ---- epilogue: wave/amplitude pairs -> x * sigmoid(a) (+ noise) -> tanh ->
    // reverse_half -> synthesis planes (zero outside [0, F))
    const float* rsc = a.weight + geo.w_frag_floats;
    const float rs = rsc[l32] / xs;
    const float bias = (a.bias && l32 < a.conv_c_out) ? a.bias[l32] : 0.f;
    const float* nz = a.noise ? a.noise + (int64_t)b * a.n_sb : nullptr;
    float sv[2][16];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        if (j == 1 && !two) break;
        const int blk = wave + kEdgeWaves * j;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float v = acc[j][r] * rs + bias;
            float out = v;
            if constexpr (AM) {
                const float amp = __shfl(v, (lane + 16) & 63);   // lane l32 + 16: channel + 16, same frames
                out = v * (1.0f / (1.0f + __expf(-amp)));
            }
            const int w = 32 * blk + 8 * (r >> 2) + 4 * h + (r & 3);
            const int f = f0 + w;
            const bool ok = f >= 0 && f < F && l32 < 16;
            if (nz && ok) out = out + nz[(int64_t)l32 * a.n_sc + f];
            out = tanhf(out);
            if ((l32 & 1) && !(f & 1)) out = -out;
            sv[j][r] = ok ? out : 0.f;
        }
    }
    __syncthreads();                                 // act(x) planes dead: the synthesis planes reuse them
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        if (j == 1 && !two) break;
        const int blk = wave + kEdgeWaves * j;
        if (l32 < 16) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int w = 32 * blk + 8 * (r >> 2) + 4 * h + (r & 3);
                if (w < kTSW) e_split(sv[j][r], sh[w * kTSP + l32], sl[w * kTSP + l32]);
            }
        }
    }
    __syncthreads();

    // ---- synthesis (as pqmf_synthesis_split_kernel): wave = 2 blocks of 16 frames
    const int g = lane >> 4, col = lane & 15;
    constexpr int BLK = kTF / (16 * kEdgeWaves);     // 2
    const int fb = wave * BLK * 16;
    e_f32x4 sacc[BLK];
#pragma unroll
    for (int q = 0; q < BLK; ++q) sacc[q] = e_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < kEdgeKW / 32; ++s) {
        const int ka = col * kEdgeFP + 32 * s + 8 * g;
        const e_h8 ah = *reinterpret_cast<const e_h8*>(fh + ka);
        const e_h8 al = *reinterpret_cast<const e_h8*>(fl + ka);
        const e_h8 a2 = ah * (_Float16)2048.0f;
        const int tap = 2 * s + (g >> 1);
#pragma unroll
        for (int q = 0; q < BLK; ++q) {
            const int xi = (fb + 16 * q + col + tap) * kTSP + 8 * (g & 1);
            const e_h8 b_h = *reinterpret_cast<const e_h8*>(sh + xi);
            const e_h8 b_l = *reinterpret_cast<const e_h8*>(sl + xi);
            sacc[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2, b_h, sacc[q], 0, 0, 0);
            sacc[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, b_l, sacc[q], 0, 0, 0);
            sacc[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, b_h, sacc[q], 0, 0, 0);
        }
    }
    const float o = 16.f / (sc * 2048.0f);
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
static EdgeGeo edge_geometry(const rave_edge_args& a, int frames_per_tile) {
    EdgeGeo g{};
    g.tiles = ceil_div(a.frames, frames_per_tile);
    const int nchunks = (a.conv_c_in + 15) / 16;
    const int mpad = ceil_div(a.conv_c_out, 128) * 128;
    g.w_mb = mpad / 32;
    g.w_frag_floats = (int64_t)nchunks * g.w_mb * kEdgeK7 * 2 * 256;
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
    const EdgeGeo g = edge_geometry(a, kHF);
    static bool attr = false;
    const int rc = edge_lds_attr(encoder_head_kernel, kHeadLds, attr);
    if (rc != RAVE_OK) return rc;
    const int grid = g.tiles * a.batch + (a.fill_channels > 0 ? a.batch : 0);
    launch(encoder_head_kernel, dim3(grid), dim3(kEdgeNT), (uint32_t)kHeadLds, as_stream(stream), a, g);
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
    const EdgeGeo g = edge_geometry(a, kTF);
    const dim3 grid(g.tiles * a.batch);
    const bool snake = a.act == RAVE_ACT_SNAKE, am = a.mode == 1;
    auto kern = snake ? (am ? decoder_tail_kernel<true, true> : decoder_tail_kernel<true, false>)
                      : (am ? decoder_tail_kernel<false, true> : decoder_tail_kernel<false, false>);
    static bool attr[4] = {false, false, false, false};
    const int rc = edge_lds_attr(kern, kTailLds, attr[2 * snake + am]);
    if (rc != RAVE_OK) return rc;
    launch(kern, grid, dim3(kEdgeNT), (uint32_t)kTailLds, as_stream(stream), a, g);
    return launch_status("decoder_tail_kernel");
}
