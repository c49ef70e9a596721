/*
 * rave_amd.h -- C-ABI of the MI355X-native RAVE encode->decode path.
 *
 * Plain C, plain pointers and sizes; no torch or HIP types in any signature
 * (streams are passed as `void*` holding a hipStream_t, NULL = default stream).
 * Every entry point returns RAVE_OK (0) or a negative status; the last error
 * text is available through rave_last_error().  Kernels never allocate:
 * callers own every buffer (weights, activations, workspace, streaming state).
 * Calls are asynchronous on the given stream and never synchronise the host.
 *
 * What each entry point replaces in the reference (abargum/RAVE @ 2024-10-16):
 *
 *   rave_conv1d          cc.Conv1d / cc.ConvTranspose1d forward (third-party
 *                        cached_conv, non-cached mode: F.pad + conv), fused with
 *                        the preceding activation module (nn.LeakyReLU(.2),
 *                        rave/blocks.py:91 / Snake rave/blocks.py:845-853) and
 *                        the Residual add (rave/blocks.py:44-46).  Call sites:
 *                        DilatedUnit rave/blocks.py:96-106, EncoderV2
 *                        :533-584, GeneratorV2 :631-677, NoiseGeneratorV2
 *                        :257-266.
 *   rave_pqmf_analysis   CachedPQMF.forward rave/pqmf.py:269-273 (+ reverse_half
 *                        :13-17, + the band slice of RAVE.encode model.py:613).
 *   rave_pqmf_synthesis  CachedPQMF.inverse rave/pqmf.py:275-284, optionally fused
 *                        with GeneratorV2's `x*sigmoid(a) (+noise) -> tanh`
 *                        epilogue rave/blocks.py:699-707.
 *   rave_fill_channels   the speaker-embedding concat of RAVE.encode
 *                        rave/model.py:618-620.
 *   rave_rvq_encode /    ResidualVectorQuantization.encode / decode
 *   rave_rvq_decode      rave/quantization.py:302-318.
 *   rave_encoder_head    rave_pqmf_analysis + EncoderV2's first conv (+ the speaker
 *                        concat) in one launch (split-f16): RAVE.encode's head.
 *   rave_decoder_tail    GeneratorV2's last act + conv + epilogue +
 *                        rave_pqmf_synthesis in one launch (split-f16).
 *   rave_plan_*          RAVE.encode / decode / forward rave/model.py:594-634 as
 *                        one pre-built launch sequence (the module graph).
 */
#ifndef RAVE_AMD_H
#define RAVE_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RAVE_ABI_VERSION 18
/* int32 arrival counters at the head of every split-K workspace (rave_conv1d_args.partial) */
#define RAVE_SPLITK_TICKETS 4096
/* The last of those words is reserved: no conv ticket uses it.  A cooperative
 * fused unit (rave_unit_workspace) whose in-launch hand-off gave up sets it to
 * nonzero and leaves it set (sticky); a direct caller that owns the workspace
 * reads it and zeroes it.  The model engine does not use this word: it reads
 * (and clears) the per-op host-mapped words it passes as rave_unit_args.status,
 * so in its plans the workspace word may stay set after a reported give-up
 * (harmless: no conv ticket uses it). */
#define RAVE_SPLITK_STATUS_WORD (RAVE_SPLITK_TICKETS - 1)

/* ---------------------------------------------------------------- status */
enum {
    RAVE_OK = 0,
    RAVE_ERR_ARG = -1,          /* invalid argument (ValueError in Python)      */
    RAVE_ERR_HIP = -2,          /* HIP runtime error (RuntimeError)             */
    RAVE_ERR_UNSUPPORTED = -3,  /* shape/config the kernels do not implement    */
    RAVE_ERR_STATE = -4,        /* bad handle / plan                            */
    RAVE_ERR_COOP = -5          /* a cooperative unit's in-launch hand-off gave up:
                                   that call's outputs are NaN (RuntimeError)   */
};

/* activation applied to a conv INPUT (fused prologue) */
enum { RAVE_ACT_NONE = 0, RAVE_ACT_LEAKY = 1, RAVE_ACT_SNAKE = 2 };

/* arithmetic of the conv / unit GEMMs (the `precision` field of their args):
 *   RAVE_PREC_F32      v_mfma_f32_32x32x2_f32: exact fp32 (k-ordered fmaf chain).
 *   RAVE_PREC_SPLIT16  every fp32 operand split exactly-ish into an f16 pair
 *                      (hi = f16(v), lo = f16((v - hi) * 2^11); weights pre-scaled
 *                      per output row by a power of two), three
 *                      v_mfma_f32_32x32x16_f16 products hi*hi*2^11 + hi*lo + lo*hi
 *                      into one fp32 accumulator, exact power-of-two unscale in the
 *                      epilogue.  Operand representation error <= ~2^-23 relative,
 *                      products exact in fp32; measured layer error within 1.5x of
 *                      the fp32 path.  Requires |act(x)| < 65504 (f16 range);
 *                      5.3x the fp32 MFMA rate.  Weights must be packed with the
 *                      *_split_* packers. */
enum { RAVE_PREC_F32 = 0, RAVE_PREC_SPLIT16 = 1 };
/*   RAVE_PREC_F32_RING exact fp32 (v_mfma_f32_32x32x2_f32) on the split16 kernels'
 *                      staging machinery (LDS-DMA window ring, register weight ring,
 *                      K-groups, the same tiles and launch configurations); weights
 *                      packed with rave_conv1d_ring_pack_weight (sizes as the split
 *                      image).  Value 4: 2 and 3 are model-level modes below. */
#define RAVE_PREC_F32_RING 4
/*   RAVE_PREC_BF16X3   fp32 on the bf16 matrix cores (fused units, C in {64, 128, 256}, and
 *                      512 at dilations <= 4; rave_conv1d on the split kernels' machinery,
 *                      16-byte aligned input rows):
 *                      every operand split exactly into three bf16 parts
 *                      (v = hi + mid + lo, 24 significand bits, the fp32 exponent
 *                      range: no row scales, no range guard; hi rounds to nearest, so
 *                      a finite |v| above ~3.39e38 rounds hi to inf and the output is
 *                      non-finite -- the only ceiling below FLT_MAX); six
 *                      v_mfma_f32_32x32x16_bf16 products per K-step (all cross
 *                      products but mid*lo, lo*mid, lo*lo: each < 2^-25 |a b|) into one
 *                      fp32 accumulator.  Weights packed with rave_unit_bf3_pack_weight /
 *                      rave_conv1d_bf3_pack_weight. */
#define RAVE_PREC_BF16X3 5

const char* rave_last_error(void);
int rave_abi_version(void);
/* sizeof of every public struct, in declaration order (ABI self-check) */
int rave_struct_sizes(int64_t* out, int n);

/* ---------------------------------------------------------------- conv1d
 * y[b, m, n] = bias[m] + sum_{ci,j} W[m, ci, j] * act(x)[b, ci, n*stride + j*dil - pad_left]
 *              (+ residual[b, m, n])
 * with zero padding outside [0, t_in).  Time is contiguous (stride 1) in every
 * tensor; batch and channel strides are free, so views into larger buffers
 * (concatenations, streaming history) need no copies.
 *
 * transposed = 1: nn.ConvTranspose1d(c_in, c_out, 2r, stride=r) in polyphase
 * form.  Output t = u*r + q (u in [0, t_in - pad_left)) for every phase q is a
 * 2-tap conv of the input: with P = out_shift, phases q < r-P read (x[u-1],
 * x[u]) and phases q >= r-P read (x[u], x[u+1]); the two phase groups are
 * separate row blocks of one GEMM, so no output column is wasted.
 *   offline (torch padding r//2): pad_left = 0, out_shift = r/2, t_out = t_in*r
 *   cached streaming (overlap-add cache): the input view starts with one history
 *   column, pad_left = 1, out_shift = 0, t_out = (t_in - 1)*r
 * pad_right is ignored; the weight must be packed with the same out_shift.
 */
typedef struct rave_conv1d_args {
    int32_t c_in, c_out, kernel, stride, dilation;
    int32_t pad_left, pad_right;
    int32_t transposed;     /* 0/1; kernel == 2*stride when set                  */
    int32_t out_shift;      /* transposed only                                   */
    int32_t act;            /* RAVE_ACT_*                                        */
    float   leaky_slope;    /* 0.2 (<= 1 for the split16 / fp32-ring / bf16x3 kernels) */
    int32_t batch;
    int32_t t_in;           /* input length (columns of x)                       */
    int32_t t_out;          /* output length (columns of y)                      */
    int32_t precision;      /* RAVE_PREC_*                                       */
    const float* x;       int64_t x_sb, x_sc;
    float* y;             int64_t y_sb, y_sc;
    const float* residual; int64_t r_sb, r_sc;   /* NULL = none                  */
    const float* weight;  /* packed by rave_conv1d_pack_weight                   */
    const float* bias;    /* c_out floats or NULL                                */
    const float* alpha;   /* c_in Snake alphas (act == RAVE_ACT_SNAKE)           */
    float* partial;       /* split-K workspace of rave_conv1d_workspace() floats, or
                             NULL (then the layer runs unsplit).  Its first
                             RAVE_SPLITK_TICKETS 4-byte words are arrival
                             counters: zero them once before the first call;
                             every call leaves them zero again.  The slabs
                             after them need no initialisation.              */
    unsigned long long* stamps;   /* diagnostic builds only (-DRAVE_STAMPS): 8 clock
                                     stamps per workgroup; ignored otherwise      */
    int32_t config;       /* launch configuration: 0 = the launcher's own choice,
                             else one of rave_conv1d_configs() for these args  */
    int32_t _pad1;
} rave_conv1d_args;

/* Supported layer families (every RAVE conv): kernel 1/3/7 stride 1, kernel 4
 * stride 2, kernel 8 stride 4, dilation <= 16 on 3-tap convs, and transposed
 * kernel 2r stride r.  Others return RAVE_ERR_UNSUPPORTED.
 * input channels per K-chunk the kernels use for a layer shape */
int rave_conv1d_chunk(int c_in, int kernel, int stride, int dilation, int transposed);
/* floats of the packed weight of a layer */
int64_t rave_conv1d_packed_size(int c_in, int c_out, int kernel, int stride, int dilation,
                                int transposed);
/* Host-side repack of a folded torch-layout weight (Conv1d: (c_out, c_in, k);
 * ConvTranspose1d: (c_in, c_out, k)) into the kernel's K-chunked layout. */
int rave_conv1d_pack_weight(const float* w, int c_in, int c_out, int kernel, int stride,
                            int dilation, int transposed, int out_shift, float* packed);
/* Launch configurations (tile shape, K-splits, split-K combine) valid for
 * these args and precision, for plan-time autotuning (cf. cuDNN's Find API):
 * writes up to max_cfgs values for rave_conv1d_args.config into cfgs and
 * returns how many exist (0 is always valid and is not listed), or an error. */
int rave_conv1d_configs(const rave_conv1d_args* a, int32_t* cfgs, int max_cfgs);
/* floats of split-K workspace the launcher would use for these args (0 = none);
 * RAVE_SPLITK_TICKETS counter words + the fp32 slabs */
int64_t rave_conv1d_workspace(const rave_conv1d_args* a);
/* RAVE_PREC_SPLIT16 weight image: per K-chunk, per 32-row block, per K-step of
 * 16, the (hi, lo) f16 MFMA A-fragments in lane order, then one float row scale
 * per padded GEMM row.  Sizes in floats (4-byte units). */
int64_t rave_conv1d_split_packed_size(int c_in, int c_out, int kernel, int stride, int dilation,
                                      int transposed);
int rave_conv1d_split_pack_weight(const float* w, int c_in, int c_out, int kernel, int stride,
                                  int dilation, int transposed, int out_shift, float* packed);
/* RAVE_PREC_F32_RING weight image: the split image's layout with 8 fp32 values
 * per lane and K-step (4 in each 1 KB slot) and row scales 1 */
int rave_conv1d_ring_pack_weight(const float* w, int c_in, int c_out, int kernel, int stride,
                                 int dilation, int transposed, int out_shift, float* packed);
/* RAVE_PREC_BF16X3 weight image: the split image's layout with three bf16 fragments
 * (hi, lo, mid) per 32-row block and K-step, row scales 1. */
int64_t rave_conv1d_bf3_packed_size(int c_in, int c_out, int kernel, int stride, int dilation, int transposed);
int rave_conv1d_bf3_pack_weight(const float* w, int c_in, int c_out, int kernel, int stride, int dilation,
                                int transposed, int out_shift, float* packed);
int rave_conv1d(const rave_conv1d_args* a, void* stream);

/* ---------------------------------------------------------------- PQMF
 * analysis: y[b, band, t] = rh(band, t) * sum_j hkf[band, j] * x[b, t*n_band + j - pad_left]
 * for band < n_out_bands, rh = -1 on odd bands at even t (reverse_half).
 * hkf: (n_band, taps) analysis filter (taps = 513 for 16 bands).
 */
typedef struct rave_pqmf_analysis_args {
    int32_t n_band, taps, n_out_bands, batch;
    int32_t t_in, pad_left;     /* t_out = t_in / n_band                          */
    int32_t t_out, precision;   /* RAVE_PREC_F32 (exact fp32 MFMA) or RAVE_PREC_SPLIT16 */
    const float* x; int64_t x_sb;
    float* y;       int64_t y_sb, y_sc;
    const float* hkf;
} rave_pqmf_analysis_args;
int rave_pqmf_analysis(const rave_pqmf_analysis_args* a, void* stream);

/* synthesis: in = reverse_half(mode 0: x
 *                                mode 1: tanh(x[:n]*sigmoid(x[n:2n]) + noise)   (amplitude modulation)
 *                                mode 2: tanh(x[:n] + noise))
 * (modes 1/2 are GeneratorV2's epilogue, rave/blocks.py:699-707; noise may be NULL)
 * c[m, t] = n_band * sum_{c,k} hki[m, c, k] * in[c, t + k - pad_left]   for t in [0, t_in)
 * y[b, t*n_band + i] = c[n_band-1-i, t]
 * x columns [0, x_len) are valid input frames (x_len = 0 means t_in; columns
 * outside read as zero padding); `frame0` is the global frame index of
 * column 0 (reverse_half parity).  noise: (B, n_band, x_len) or NULL.
 * Streaming: point x at the cached history, pad_left = 0, x_len = hist + t_in.
 */
typedef struct rave_pqmf_synthesis_args {
    int32_t n_band, taps, batch, t_in;
    int32_t pad_left, mode, frame0, x_len;
    const float* x;     int64_t x_sb, x_sc;
    const float* noise; int64_t n_sb, n_sc;
    float* y;           int64_t y_sb;
    const float* hki;   /* (n_band, n_band, taps) */
    int32_t precision;  /* RAVE_PREC_F32 (exact fp32 MFMA) or RAVE_PREC_SPLIT16 */
    int32_t _pad0;
} rave_pqmf_synthesis_args;
int rave_pqmf_synthesis(const rave_pqmf_synthesis_args* a, void* stream);

/* ---------------------------------------------------------------- misc */
/* y[b, c, t] = values[c] for c < channels, t < t_len (speaker concat) */
typedef struct rave_fill_args {
    int32_t batch, channels, t_len, _pad0;
    float* y; int64_t y_sb, y_sc;
    const float* values;
} rave_fill_args;
int rave_fill_channels(const rave_fill_args* a, void* stream);

/* y[b, c, t] = x[b, c, t] for c < channels, t < t_len (streaming input staging) */
typedef struct rave_copy_args {
    int32_t batch, channels, t_len, _pad0;
    const float* x; int64_t x_sb, x_sc;
    float* y;       int64_t y_sb, y_sc;
} rave_copy_args;
int rave_copy(const rave_copy_args* a, void* stream);

/* ---------------------------------------------------------------- RVQ
 * encode: for q in [0, n_q): idx[b, q, t] = argmax_k -(|r|^2 - 2 r.E_q[k] + |E_q[k]|^2),
 *         r -= E_q[idx];   r starts as z[b, :, t]   (first index on ties)
 * decode: y[b, :, t] = sum_q E_q[idx[b, q, t]]
 * codebooks: (n_q, codebook_size, dim) fp32; idx int64.
 * encode runs one launch per quantizer layer (frames x code splits, so the chip
 * fills at any batch) plus a final index reduction; `work` is caller-owned
 * device scratch of rave_rvq_workspace(a) floats (residual double buffer and
 * per-split best candidates), unused by decode.
 */
typedef struct rave_rvq_args {
    int32_t n_q, codebook_size, dim, batch;
    int32_t t_len, _pad0;
    const float* codebooks;
    const float* z;  int64_t z_sb, z_sc;      /* encode input                     */
    int64_t* idx;    int64_t i_sb, i_sq;      /* (B, n_q, T) int64                */
    float* y;        int64_t y_sb, y_sc;      /* decode output                    */
    float* work;                              /* encode scratch                   */
} rave_rvq_args;
/* floats of encode scratch for these shapes (>= 0), or a negative status */
int64_t rave_rvq_workspace(const rave_rvq_args* a);
int rave_rvq_encode(const rave_rvq_args* a, void* stream);
int rave_rvq_decode(const rave_rvq_args* a, void* stream);

/* SHIFT_HISTORY payload (streaming state update): for each (b, c) row of a
 * buffer with `hist` history columns and `t_new` fresh ones, move the last
 * `hist` columns to the front.  Rows are independent. */
typedef struct rave_shift_args {
    int32_t batch, channels, hist, t_new;
    float* buf; int64_t sb, sc;
} rave_shift_args;
int rave_shift_history(const rave_shift_args* a, void* stream);

/* ---------------------------------------------------------------- noise synthesizer
 * NoiseGeneratorV2's filter stage (rave/blocks.py:281-291, rave/core.py:66-67,95-129),
 * after its conv stack:  for every (b, frame f, band j)
 *   A[k]  = 2 * sigmoid(amp[b, j*noise_bands + k, f] - 5)^2.3 + 1e-7     k < noise_bands
 *   ir    = irfft(A) (fs = 2*(noise_bands-1) taps), Hann-windowed and centred by the
 *           roll/pad/roll of amp_to_impulse_response, length `target`
 *   y[b, j, f*target + i] = sum_{m<=i} (2*u[b, f, j, m] - 1) * ir[i - m]   i < target
 *           (the second half of fft_convolve's zero-padded circular product)
 * u: (B, frames, n_band, target) U[0,1) samples (torch.rand_like(ir)); u_sb its
 * batch stride, inner dims contiguous.  Requires target >= fs, target <= 32.
 */
typedef struct rave_noise_args {
    int32_t batch, frames, n_band, noise_bands;
    int32_t target, _pad0;
    const float* amp; int64_t a_sb, a_sc;     /* (B, n_band*noise_bands, frames) */
    const float* u;   int64_t u_sb;
    float* y;         int64_t y_sb, y_sc;     /* (B, n_band, frames*target)      */
} rave_noise_args;
int rave_noise_synth(const rave_noise_args* a, void* stream);

/* ---------------------------------------------------------------- AdaIN
 * AdaptiveInstanceNormalization.forward in eval mode (rave/blocks.py:856-919) over
 * the module's own buffers, kept on the device:
 *   stats:    (4, max_batch, channels) = mean_x, std_x, mean_y, std_y   (row = row0 + b)
 *   counters: float[2] = num_update_x, num_update_y
 * mode 0 (transfer):  y = transfer(x) if num_update_x and num_update_y else x
 * mode 1 (learn_x):   mean_x/std_x[row] += (stat(x) - ·)/(num_update_x + 1); num_update_x += 1;
 *                     then as mode 0
 * mode 2 (learn_y):   mean_y/std_y[row] += (stat(x) - ·)/(num_update_y + 1); num_update_y += 1;
 *                     y = x
 * stat = mean / unbiased std over t; transfer(x) = (x - mean_x)/(std_x + 1e-5)*std_y + mean_y.
 * `ticket` is a zeroed uint32 the kernel uses to bump the counter once per call
 * (it is left zeroed).  y may alias x.
 */
typedef struct rave_adain_args {
    int32_t batch, channels, t_len, mode;
    int32_t max_batch, row0;
    const float* x; int64_t x_sb, x_sc;
    float* y;       int64_t y_sb, y_sc;
    float* stats;
    float* counters;
    uint32_t* ticket;
} rave_adain_args;
int rave_adain(const rave_adain_args* a, void* stream);

/* ---------------------------------------------------------------- fused residual unit
 * Residual(DilatedUnit(C, k=3, d)) in one kernel (rave/blocks.py:32-46, 84-113):
 *   y = x + W2 . act(W1 *_d act(x) + b1) + b2
 * W1: (C, C, 3) dilation d, padding (pad_left, 2d - pad_left) -- centered d, causal 2d;
 * W2: (C, C, 1).  act is the unit's activation (LeakyReLU slope / Snake with
 * alpha0 before W1 and alpha2 before W2).  weight = rave_unit_pack_weight
 * layout (rave_unit_packed_size floats).  C in {64, 128, 256, 512}; other
 * widths return RAVE_ERR_UNSUPPORTED (callers use two rave_conv1d calls).
 * y must not alias x.
 */
typedef struct rave_unit_args {
    int32_t channels, batch, t_len, dilation;
    int32_t pad_left, act;
    float leaky_slope; int32_t precision;   /* slope <= 1; RAVE_PREC_* */
    const float* x; int64_t x_sb, x_sc;
    float* y;       int64_t y_sb, y_sc;
    const float* weight;
    const float* bias1; const float* bias2;
    const float* alpha0; const float* alpha2;
    float* workspace;   /* optional, rave_unit_workspace() floats, zeroed once before its first
                           use (every launch leaves its counters zero); NULL: one workgroup per slab */
    uint32_t* status;   /* optional (cooperative form): a group whose hand-off gave up also sets
                           this word to 1 (system-scope store: host-mapped memory works), beside
                           the workspace's RAVE_SPLITK_STATUS_WORD; the caller clears it */
    int32_t x_len;      /* valid input columns (0: t_len).  Cached (streaming) form: x starts at
                           the history, pad_left = 0, x_len = 2*dilation + t_len, and no column
                           past x_len is padding (the one-shot form pads past t_len with zeros) */
    int32_t res_shift;  /* the residual of output column n is x column n + res_shift (0 one-shot;
                           cached: 2*dilation - the identity branch's delay, rave/blocks.py:32-46) */
    int32_t coop_rb;    /* cooperative group size (ABI 18): 0 = C / 128 (2 at C = 256, 4 at 512);
                           4 at C = 256 = the wide group (its weights stream through twice the
                           CUs: short inputs, e.g. streaming blocks); workspace size depends on it */
    int32_t reserved0;
} rave_unit_args;
int64_t rave_unit_packed_size(int channels);
int rave_unit_pack_weight(const float* w1, const float* w2, int channels, float* packed);
/* RAVE_PREC_SPLIT16 unit weights (C in {64, 128}): (hi, lo) f16 A-fragments of
 * W1 then W2 per 32-row block and 16-deep K-step, then the two row-scale
 * vectors.  Other widths return -1 / RAVE_ERR_UNSUPPORTED (run the unit as two
 * split16 rave_conv1d calls). */
int64_t rave_unit_split_packed_size(int channels);
int rave_unit_split_pack_weight(const float* w1, const float* w2, int channels, float* packed);
/* RAVE_PREC_F32_RING unit weights (exact fp32 on the split kernel's machinery):
 * the split image's layout with 8 fp32 values per lane and K-step, row scales 1
 * (sizes as rave_unit_split_packed_size). */
int rave_unit_ring_pack_weight(const float* w1, const float* w2, int channels, float* packed);
/* RAVE_PREC_BF16X3 unit weights (C in {64, 128, 256, 512}; else -1 / RAVE_ERR_UNSUPPORTED):
 * (hi, lo, mid) bf16 A-fragments per 32-row block and K-step, then the two
 * row-scale vectors (all 1). */
int64_t rave_unit_bf3_packed_size(int channels);
int rave_unit_bf3_pack_weight(const float* w1, const float* w2, int channels, float* packed);
/* Workspace (floats) of the cooperative fused unit (C in {256, 512}, RAVE_PREC_SPLIT16 /
 * RAVE_PREC_F32_RING): groups of C/128 workgroups share a 32-column slab, each owning
 * C/(C/128) output rows of both GEMMs, and hand the intermediate act2(h) rows to each
 * other inside the launch.  0: this shape runs one workgroup per slab.  The first
 * RAVE_SPLITK_TICKETS words are counters, like rave_conv1d_workspace's: one buffer
 * serves both when ops run in stream order. */
int64_t rave_unit_workspace(const rave_unit_args* a);
int rave_residual_unit(const rave_unit_args* a, void* stream);
/* Debug / test hook for the cooperative hand-off (process-wide, read at each launch):
 * spin_limit = polls before a member gives up (< 0: the default, 2^18); force_giveup != 0
 * makes every group report a give-up after a normal hand-off (outputs NaN, status set),
 * so the error path can be exercised deterministically. */
int rave_debug_coop(int64_t spin_limit, int force_giveup);

/* ---------------------------------------------------------------- residual stack
 * RAVE_STACK_UNITS consecutive Residual(DilatedUnit)s of one width (an
 * EncoderV2 / GeneratorV2 residual stack, rave/blocks.py:533-558, 647-664,
 * dilations e.g. 1, 3, 9) in one launch, split-f16 arithmetic: the input is
 * read once, the intermediate unit outputs stay on chip (a tile recomputes a
 * 32-column margin on each side), the stack output is written once.
 * y[:, :, t] = U3(U2(U1(x)))[:, :, t]; weights are rave_unit_split_pack_weight
 * images.  C in {64, 128}; dilation <= 16, pad_left <= 2*dilation.  x and y
 * must not overlap.  Other shapes return RAVE_ERR_UNSUPPORTED.
 * precision RAVE_PREC_BF16X3 (ABI 17): fp32 on the bf16 matrix cores (exact
 * three-way operand split, as the fused unit's), weights rave_unit_bf3_pack_weight
 * images; every unit's taps within 24 columns (pad_left <= 24, 2*dilation -
 * pad_left <= 24). */
#define RAVE_STACK_UNITS 3
typedef struct rave_stack_args {
    int32_t channels, batch, t_len, act;
    float leaky_slope; int32_t precision;   /* slope <= 1; 0 / RAVE_PREC_SPLIT16 or RAVE_PREC_BF16X3 (ABI 17) */
    int32_t dilation[RAVE_STACK_UNITS], pad_left[RAVE_STACK_UNITS];
    const float* x; int64_t x_sb, x_sc;
    float* y;       int64_t y_sb, y_sc;
    const float* weight[RAVE_STACK_UNITS];
    const float* bias1[RAVE_STACK_UNITS];
    const float* bias2[RAVE_STACK_UNITS];
    const float* alpha0[RAVE_STACK_UNITS];
    const float* alpha2[RAVE_STACK_UNITS];
} rave_stack_args;
int rave_stack_supported(int channels);
int rave_residual_stack(const rave_stack_args* a, void* stream);

/* ---------------------------------------------------------------- path edges (split-f16)
 * The PQMF end of each half of the path fused with the conv next to it; one
 * launch each, split-f16 arithmetic (RAVE_PREC_SPLIT16: every operand block is
 * scaled by a power of two from its workgroup maximum, so any finite input is
 * in range).  The intermediate never reaches HBM.
 *
 * rave_encoder_head: CachedPQMF.forward + band slice (rave/pqmf.py:269-273,
 * rave/model.py:613) then EncoderV2's first conv (rave/blocks.py:533-536):
 *   bands = rave_pqmf_analysis(x, n_out_bands = conv_c_in, pad pqmf_pad_left)
 *   y[b, m, t] = bias[m] + sum_{c, j} W[m, c, j] * bands[b, c, t + j - conv_pad_left]
 *   x: audio (B, 1, 16 * frames), x_sb; y: (B, conv_c_out, frames).
 *   filter: rave_encoder_head_pack_filter image; conv_c_in <= 8 bands, conv_c_out <= 64,
 *   conv_kernel 7.
 *   fill_channels > 0: also fill_y[b, c, t] = fill_values[c], t < fill_t (the
 *   speaker concat of RAVE.encode, rave/model.py:618-620).
 * rave_decoder_tail: GeneratorV2's act + conv (rave/blocks.py:691-696), its
 * epilogue (:699-707) and CachedPQMF.inverse (rave/pqmf.py:275-284):
 *   w = bias + conv_k(act(x))          conv_c_in 64 -> conv_c_out 32 (mode 1) / 16 (mode 2)
 *   y = rave_pqmf_synthesis(w, mode, noise, pad pqmf_pad_left)
 *   x: (B, 64, frames); y: (B, 1, 16 * frames), 16-byte aligned.  filter:
 *   rave_decoder_tail_pack_filter image; act RAVE_ACT_LEAKY / RAVE_ACT_SNAKE
 *   (alpha: 64 floats).
 * weight: the conv's rave_conv1d_split_pack_weight image (7 taps, stride 1).
 * precision RAVE_PREC_F32_RING: exact fp32 (v_mfma_f32_16x16x4 / 32x32x2) with the
 * conv's rave_conv1d_ring_pack_weight image and a *_pack_filter_f32 filter image.
 * rave_decoder_tail also takes RAVE_PREC_BF16X3 (round 5): the conv in bf16x3 (its
 * rave_conv1d_bf3_pack_weight image), the synthesis (since round 6) in bf16x3 too,
 * split in-kernel from the rave_decoder_tail_pack_filter_f32 image.
 * rave_encoder_head takes RAVE_PREC_BF16X3 (round 6, ABI 18): the analysis in
 * bf16x3 (split in-kernel from the rave_encoder_head_pack_filter_f32 image), the
 * conv in exact fp32 (the rave_conv1d_ring_pack_weight image).
 */
typedef struct rave_edge_args {
    int32_t batch, frames;          /* PQMF frames (audio samples / 16)                    */
    int32_t conv_c_in, conv_c_out, conv_kernel, conv_pad_left;
    int32_t pqmf_taps, pqmf_pad_left;
    int32_t mode, act;              /* tail: synthesis mode 1 / 2; the conv input act      */
    float leaky_slope;
    int32_t fill_channels, fill_t;
    int32_t precision;  /* 0 / RAVE_PREC_SPLIT16, or RAVE_PREC_F32_RING (exact fp32)      */
    const float* x;     int64_t x_sb, x_sc;
    float* y;           int64_t y_sb, y_sc;
    const float* weight;
    const float* bias;  /* conv_c_out floats or NULL                                       */
    const float* alpha; /* Snake alphas of the conv input (tail)                           */
    const float* filter;
    const float* noise; int64_t n_sb, n_sc;   /* tail: (B, 16, frames) or NULL             */
    float* fill_y;      int64_t f_sb, f_sc;
    const float* fill_values;
} rave_edge_args;
int rave_encoder_head(const rave_edge_args* a, void* stream);
int rave_decoder_tail(const rave_edge_args* a, void* stream);
/* `filter` of both: a pre-split image of the PQMF filter (the kernels' LDS
 * layout: f16 hi / lo planes of 16 rows x 552, scaled by 2^e with max |h 2^e|
 * in [8, 16), then the float 2^-(e+11)), RAVE_EDGE_FILTER_FLOATS floats.
 * Head: phase-packed analysis rows (8p + k) of hkf (n_band, taps) for the
 * first n_out_bands bands; tail: hki (n_band, n_band, taps) as K = tap*16 + c. */
#define RAVE_EDGE_FILTER_FLOATS 8836
int rave_encoder_head_pack_filter(const float* hkf, int n_band, int taps, int n_out_bands, float* image);
int rave_decoder_tail_pack_filter(const float* hki, int n_band, int taps, float* image);
/* exact-fp32 images (precision RAVE_PREC_F32_RING): fp32 rows of 552, scale 1 */
int rave_encoder_head_pack_filter_f32(const float* hkf, int n_band, int taps, int n_out_bands, float* image);
int rave_decoder_tail_pack_filter_f32(const float* hki, int n_band, int taps, float* image);

/* ---------------------------------------------------------------- plans
 * A plan is a recorded sequence of the ops above (the module graph of
 * RAVE.encode/decode).  Pointer fields inside an op's args may be relocated at
 * run time: a relocation (op, byte offset of the pointer field inside `args`,
 * slot, byte offset) makes the executor store slots[slot] + byte_offset there,
 * so one plan serves every call with fresh input/output buffers.
 */
enum {
    RAVE_OP_CONV = 1,
    RAVE_OP_PQMF_ANALYSIS = 2,
    RAVE_OP_PQMF_SYNTHESIS = 3,
    RAVE_OP_FILL = 4,
    RAVE_OP_RVQ_ENCODE = 5,
    RAVE_OP_RVQ_DECODE = 6,
    RAVE_OP_SHIFT_HISTORY = 7,
    RAVE_OP_COPY = 8,
    RAVE_OP_NOISE = 9,
    RAVE_OP_ADAIN = 10,
    RAVE_OP_UNIT = 11,
    RAVE_OP_STACK = 12,
    RAVE_OP_HEAD = 13,
    RAVE_OP_TAIL = 14
};

#define RAVE_OP_PAYLOAD 240
typedef struct rave_plan_op {
    int32_t kind, _pad0;
    union {
        rave_conv1d_args conv;
        rave_pqmf_analysis_args ana;
        rave_pqmf_synthesis_args syn;
        rave_fill_args fill;
        rave_rvq_args rvq;
        rave_shift_args shift;
        rave_copy_args copy;
        rave_noise_args noise;
        rave_adain_args adain;
        rave_unit_args unit;
        rave_stack_args stack;
        rave_edge_args edge;
        unsigned char raw[RAVE_OP_PAYLOAD];
    } u;
} rave_plan_op;

typedef struct rave_reloc {
    int32_t op, field_offset, slot, _pad0;
    int64_t byte_offset;
} rave_reloc;

typedef struct rave_plan rave_plan;
int rave_plan_create(const rave_plan_op* ops, int n_ops, const rave_reloc* relocs, int n_relocs,
                     rave_plan** out);
/* Threading: rave_plan_run relocates into a per-call, per-host-thread copy and
 * never writes the plan, so several threads may replay one plan at once on
 * their own streams PROVIDED each call binds its own activation / workspace
 * slots (the split-K ticket counters live in the workspace slot).  Profiling
 * (rave_plan_profile / rave_plan_op_times) keeps per-plan event state and is
 * single-threaded.  Errors are per thread (rave_last_error). */
int rave_plan_run(rave_plan* plan, void* const* slots, int n_slots, void* stream);
int rave_plan_destroy(rave_plan* plan);
int rave_plan_size(const rave_plan* plan);
/* Per-op timing (measurement only).  rave_plan_profile(plan, runs) arms event
 * sets for up to `runs` consecutive runs (0 frees them); the events ride inside
 * the op's own kernel dispatches (first kernel start -> last kernel end), so
 * timed runs need no host synchronisation and get no extra packets.
 * rave_plan_op_times waits for the recorded runs, ADDS each op's elapsed
 * milliseconds summed over them into ms[0..n), re-arms, and returns the number
 * of runs summed (>= 0) or an error status. */
int rave_plan_profile(rave_plan* plan, int enable);
int rave_plan_op_times(rave_plan* plan, float* ms, int n);

/* y[i] = lo + (hi - lo) * u_i, u_i in [0, 1) from a counter-based hash of
 * (seed, i): the device draw behind torch.rand_like of NoiseGeneratorV2
 * (rave/blocks.py:287) when the caller supplies no noise, and the scratch
 * inputs of the engine's launch-configuration timing. */
int rave_fill_uniform(float* y, int64_t n, uint64_t seed, float lo, float hi, void* stream);

/* ================================================================ edges of the path
 * Resampler (rave/resampler.py:9-66) and the SpeakerRAVE pooling head
 * (rave/CombinedRave.py:301-328); their convolutions run on rave_conv1d /
 * rave_residual_unit.  All HBM-bound VALU kernels (csrc/speaker.hip).
 *
 * rave_fir: polyphase FIR, the two cached_conv Conv1d of the Resampler
 *   y[b, t*phases + p] = sum_k h[p*taps + k] * x[b, t*stride + k - pad_left]
 * for t in [0, t_out); x columns outside [0, t_in) read as zero.  Decimation
 * (to_model_sampling_rate :60-61): phases 1, stride = ratio.  Interpolation
 * (from_model_sampling_rate :63-66, the (B, ratio, T) -> (B, 1, ratio T)
 * interleave fused): phases = ratio, stride 1.  Streaming: x = [history | block],
 * pad_left 0.  Limits: taps * phases <= 4096, taps <= 1024. */
typedef struct rave_fir_args {
    int32_t batch, t_in, t_out, phases, taps, stride, pad_left, _pad0;
    const float* x; int64_t x_sb;
    float* y;       int64_t y_sb;
    const float* h;
} rave_fir_args;
int rave_fir(const rave_fir_args* a, void* stream);

/* rave_row_stats: per (b, c) row of act(x) over t in [0, t_len):
 *   y[b*y_sb + c] = mean,  y[b*y_sb + channels + c] = sqrt(clamp(var, var_min, var_max))
 * with the unbiased variance (torch.var, rave/CombinedRave.py:316-318).
 * act: RAVE_ACT_NONE or RAVE_ACT_LEAKY (slope leaky_slope) applied on read. */
typedef struct rave_row_stats_args {
    int32_t batch, channels, t_len, act;
    float leaky_slope, var_min, var_max, _pad0;
    const float* x; int64_t x_sb, x_sc;
    float* y;       int64_t y_sb;
} rave_row_stats_args;
int rave_row_stats(const rave_row_stats_args* a, void* stream);

/* rave_attn_pool: attentive statistics pooling (rave/CombinedRave.py:320-323):
 * w = softmax_t(logits[b, c, :]),  mu = sum_t act(x) w,
 * sg = sqrt(clamp(sum_t act(x)^2 w - mu^2, var_min, var_max));
 * y[b*y_sb + c] = mu, y[b*y_sb + channels + c] = sg. */
typedef struct rave_attn_pool_args {
    int32_t batch, channels, t_len, act;
    float leaky_slope, var_min, var_max, _pad0;
    const float* x;      int64_t x_sb, x_sc;
    const float* logits; int64_t l_sb, l_sc;
    float* y;            int64_t y_sb;
} rave_attn_pool_args;
int rave_attn_pool(const rave_attn_pool_args* a, void* stream);

/* rave_linear: y[b*y_sb + o] = bias[o] + sum_i w[o*n_in + i] * x[b*x_sb + i]
 * (nn.Linear; also the per-clip bias of a conv whose input has time-constant
 * channels).  bias may be NULL. */
typedef struct rave_linear_args {
    int32_t batch, n_in, n_out, _pad0;
    const float* x; int64_t x_sb;
    const float* w;
    const float* bias;
    float* y;       int64_t y_sb;
} rave_linear_args;
int rave_linear(const rave_linear_args* a, void* stream);

/* rave_maxpool: nn.MaxPool1d(kernel) (stride = kernel, no padding):
 * y[b, c, t] = max_j x[b, c, t*kernel + j], t in [0, t_out). */
typedef struct rave_maxpool_args {
    int32_t batch, channels, t_out, kernel;
    const float* x; int64_t x_sb, x_sc;
    float* y;       int64_t y_sb, y_sc;
} rave_maxpool_args;
int rave_maxpool(const rave_maxpool_args* a, void* stream);

/* ================================================================ model engine
 * The whole RAVE.encode / decode / forward (rave/model.py:594-634) behind one
 * handle, for hosts with no Python (nn~ is C++): the model graph of
 * EncoderV2 / GeneratorV2 / NoiseGeneratorV2 (rave/blocks.py:244-291, 508-710)
 * is built from the hyper-parameters below (the reference's gin bindings,
 * rave/configs/v1.gin + v2.gin + causal / discrete / snake / adain / noise),
 * weights are uploaded once (weight norm folded, packed per arithmetic), and
 * each (call kind, batch, length) gets a launch plan built on first use
 * (optionally autotuned, see RAVE_PREC_AUTO) and replayed afterwards.
 *
 * Threading: a model (and each of its streams) is driven by one host thread
 * at a time; calls are asynchronous on the given stream.  The engine owns its
 * device memory (weight arena, per-plan workspaces, AdaIN buffers); callers
 * own the tensors they pass.  Plans of one model share nothing mutable, but a
 * plan's workspace is reused by every call of that plan: two calls of the same
 * kind and shape must not run concurrently on different streams.
 */
#define RAVE_MAX_RATIOS 8
#define RAVE_MAX_DILATIONS 8
enum { RAVE_PREC_AUTO = 2,     /* per op the faster of F32 / SPLIT16, timed at plan build */
       RAVE_PREC_F32_TUNED = 3 /* exact fp32 on every op; launch configurations and fused /
                                  unfused unit choices timed at plan build as in AUTO */ };
/* fp32 on every op with the fused units also timed in RAVE_PREC_BF16X3 (exact
 * operand split, fp32 accumulation): per op the fastest of F32 / F32_RING / BF16X3 */
#define RAVE_PREC_F32_BF3 6

typedef struct rave_model_config {
    int32_t n_band;               /* PQMF bands (v1.gin: 16)                                */
    int32_t enc_bands;            /* bands the encoder reads (v2.gin data_size: 6)           */
    int32_t capacity;             /* 64 (v2), 96 (discrete)                                  */
    int32_t latent_size;          /* 64 (v2), 128 (discrete)                                 */
    int32_t kernel_size;          /* 3                                                       */
    int32_t speaker_size;         /* 256: width of the constant speaker embedding            */
    int32_t n_ratios;
    int32_t ratios[RAVE_MAX_RATIOS];                        /* 4, 4, 2, 2                    */
    int32_t n_dilations[RAVE_MAX_RATIOS];                   /* 3, 3, 3, 2                    */
    int32_t dilations[RAVE_MAX_RATIOS][RAVE_MAX_DILATIONS]; /* 1 3 9 / 1 3 9 / 1 3 9 / 1 3   */
    int32_t amplitude_modulation; /* 1 (v2.gin)                                              */
    int32_t causal;               /* 0 centered, 1 causal (causal.gin)                       */
    int32_t activation;           /* RAVE_ACT_LEAKY or RAVE_ACT_SNAKE (snake.gin)            */
    int32_t adain;                /* AdaIN before every residual unit (adain.gin)            */
    float leaky_slope;            /* 0.2                                                     */
    int32_t conv_bias;            /* 1 (v1.gin cc.Conv1d.bias)                               */
    int32_t convt_bias;           /* 0 (v1.gin cc.ConvTranspose1d.bias)                      */
    int32_t noise;                /* NoiseGeneratorV2 present (noise.gin)                    */
    int32_t noise_hidden;         /* 128                                                     */
    int32_t noise_bands;          /* 5                                                       */
    int32_t n_noise_ratios;
    int32_t noise_ratios[RAVE_MAX_RATIOS];                  /* 2, 2, 2                       */
    int32_t rvq_quantizers;       /* 0 = no RVQ; 16 (discrete.gin)                           */
    int32_t rvq_codebook_size;    /* 1024                                                    */
    int32_t fuse_units;           /* 1: fused Residual(DilatedUnit) / residual-stack kernels */
} rave_model_config;

/* One named parameter in the reference's state_dict naming
 * (encoder.encoder.net.*, decoder.net.*, decoder.noise_module.net.*,
 * encoder.rvq.layers.*._codebook.embed, pqmf.hk), fp32, host memory, torch
 * layout; weight-normed convs take <name>.weight_g and <name>.weight_v. */
typedef struct rave_param {
    const char* name;
    const float* data;
    int64_t numel;
} rave_param;

typedef struct rave_model rave_model;
typedef struct rave_stream rave_stream;

/* Parameter table of a config: the count, and the i-th name / element count
 * (pqmf.hk included).  Returns a negative status on a bad config. */
int rave_model_param_count(const rave_model_config* cfg);
int rave_model_param_info(const rave_model_config* cfg, int i, char* name, int name_cap, int64_t* numel);

/* Create on the calling thread's current HIP device.  `speaker`: speaker_size
 * floats (the constant embedding RAVE.encode concatenates, rave/model.py:
 * 618-620).  precision: RAVE_PREC_F32 / RAVE_PREC_SPLIT16 / RAVE_PREC_AUTO. */
int rave_model_create(const rave_model_config* cfg, const rave_param* params, int n_params,
                      const float* speaker, int precision, rave_model** out);
int rave_model_destroy(rave_model* m);

/* RAVE.encode: x (B, 1, T) -> z (B, latent + speaker, T / hop); T % hop == 0. */
int rave_model_encode(rave_model* m, const float* x, int batch, int t, float* z, void* stream);
/* RAVE.decode: z (B, latent + speaker, F) -> y (B, 1, F * hop).  noise_u: the
 * U[0,1) draw of NoiseGeneratorV2, shape rave_model_noise_shape, or NULL (the
 * engine draws it); ignored by configs without a noise synthesizer. */
int rave_model_decode(rave_model* m, const float* z, int batch, int frames, float* y,
                      const float* noise_u, void* stream);
/* decode(encode(x)) through an engine-owned latent buffer. */
int rave_model_forward(rave_model* m, const float* x, int batch, int t, float* y,
                       const float* noise_u, void* stream);
/* Discrete configs (DiscreteScriptedRAVE, scripts/export.py:503-517):
 * encoder -> rvq.encode: idx (B, n_q, T / hop) int64; rvq.decode -> cat
 * speaker -> decoder -> PQMF inverse. */
int rave_model_encode_codes(rave_model* m, const float* x, int batch, int t, int64_t* idx, void* stream);
int rave_model_decode_codes(rave_model* m, const int64_t* idx, int batch, int frames, float* y,
                            const float* noise_u, void* stream);
/* Cooperative-unit status.  The cooperative fused unit (rave_unit_workspace)
 * hands rows between workgroups inside a launch with a bounded wait; when a
 * wait gives up, that call's outputs are NaN and a host-mapped status word of
 * the model is set.  Every encode / decode / forward / stream call first checks
 * the word (no synchronisation: it reports give-ups of calls that have already
 * run) and returns RAVE_ERR_COOP, rave_last_error naming the units, clearing
 * it.  rave_model_check does the same on demand; with `wait` nonzero it first
 * synchronises `stream`, so it covers every call queued there. */
int rave_model_check(rave_model* m, int wait, void* stream);
/* dims of NoiseGeneratorV2's noise for a decode of `frames` latent frames:
 * (B, noise frames, n_band, target) written to out[0..3]. */
int rave_model_noise_shape(const rave_model* m, int batch, int frames, int64_t* out4);

/* AdaIN (rave/blocks.py:856-919; nn~ learn/reset attributes, scripts/export.py:
 * 248-265).  learn_x / learn_y: -1 keeps, 0/1 sets; reset_*: nonzero resets
 * (asynchronous on `stream`, after the work already queued there).
 * row0: first buffer row this process's batch uses (data-parallel shards);
 * existing streams pick a new row0 up at their next block. */
int rave_model_adain_control(rave_model* m, int learn_x, int learn_y, int reset_x, int reset_y, void* stream);
int rave_model_set_row0(rave_model* m, int row0);
/* Replace the constant speaker embedding the encode / decode_codes paths
 * concatenate (speaker_size floats, host or device memory) -- the nn~
 * `speaker` attribute's choice among embeddings (scripts/export.py:384-396).
 * Asynchronous on `stream`; later calls on that stream see the new value. */
int rave_model_set_speaker(rave_model* m, const float* speaker, void* stream);
int rave_model_adain_count(const rave_model* m);
/* module i: name, channels, and its buffers copied out / in (host, synchronous):
 * stats (4, max_batch, C) = mean_x, std_x, mean_y, std_y; counters[2] =
 * num_update_x, num_update_y.  set marks the statistics as loaded. */
int rave_model_adain_info(const rave_model* m, int i, char* name, int name_cap, int* channels, int* max_batch);
int rave_model_adain_get(rave_model* m, int i, float* stats, float* counters);
int rave_model_adain_set(rave_model* m, int i, const float* stats, const float* counters);

/* Launch-configuration choices of the autotuner as text ("key value ms" per
 * line), to replay them into another model without timing runs. */
int rave_model_tuning_get(const rave_model* m, char* buf, int cap);   /* bytes needed (with NUL) */
int rave_model_tuning_set(rave_model* m, const char* text);

/* Measurement (bench.py): the op list of one plan and per-op HIP-event times.
 * which: 0 encode, 1 decode, 2 encode_codes, 3 decode_codes (built if needed). */
typedef struct rave_op_info {
    int32_t kind;        /* RAVE_OP_* */
    int32_t precision;   /* RAVE_PREC_* of conv / unit ops, else -1 */
    double flops;        /* algorithmic: 2 * MACs of the fp32 op */
    double bytes;        /* algorithmic: tensors and weights read or written once */
    char label[96];      /* reference module path */
} rave_op_info;
int rave_model_plan_ops(rave_model* m, int which, int batch, int t, rave_op_info* out, int cap);
int rave_model_profile(rave_model* m, int which, int batch, int t, int runs);
int rave_model_op_times(rave_model* m, int which, int batch, int t, float* ms, int n);

/* ---------------------------------------------------------------- streaming
 * cached_conv's streaming mode (cc.use_cached_conv(True), scripts/export.py:
 * 543, any padding mode): per-call blocks of `block` samples (a multiple of
 * hop) with persistent per-layer caches (zeroed at creation and by reset),
 * each conv in its cached form (CachedConv1d / CachedConvTranspose1d,
 * Residual's AlignBranches delays).  Decoded audio lags one-shot decoding by
 * rave_stream_delay samples (928 for v2 causal, 13280 for v2 centred); a
 * causal encoder is exact.  AdaIN statistics are per block, as the reference
 * computes them per call.
 * RAVE_STREAM_GRAPH: each block replays a captured hipGraph (inputs and
 * outputs pass through stream-owned staging buffers).
 * RAVE_STREAM_ENCODE_ONLY / _DECODE_ONLY: build one direction only (half the
 * plans, workspaces and graphs).
 * Discrete configs stream indices (DiscreteScriptedRAVE, scripts/export.py:
 * 503-517): rave_stream_encode_codes -> (B, n_q, block / hop) int64,
 * rave_stream_decode_codes clamps them to the codebook; the float entry
 * points refuse such a stream, and the _codes ones any other. */
enum { RAVE_STREAM_GRAPH = 1, RAVE_STREAM_ENCODE_ONLY = 2, RAVE_STREAM_DECODE_ONLY = 4 };
int rave_stream_create(rave_model* m, int batch, int block, int flags, rave_stream** out);
int rave_stream_destroy(rave_stream* s);
int rave_stream_reset(rave_stream* s, void* stream);
int rave_stream_encode(rave_stream* s, const float* x, float* z, void* stream);
int rave_stream_decode(rave_stream* s, const float* z, float* y, const float* noise_u, void* stream);
int rave_stream_encode_codes(rave_stream* s, const float* x, int64_t* idx, void* stream);
int rave_stream_decode_codes(rave_stream* s, const int64_t* idx, float* y, const float* noise_u, void* stream);
int rave_stream_delay(const rave_stream* s);
/* Kernel launches one block issues (which 0 = encode, 1 = decode): the kernel
 * nodes of the captured graph (RAVE_STREAM_GRAPH; the copies around a replay are
 * not counted: the call copies the block's input straight into the history
 * buffer and the output out of a staging buffer, and fills the latents' speaker
 * channels outside the graph once per rave_model_set_speaker) or the plan's
 * launches (eager:
 * one per op, a run of history shifts batched into one launch as rave_plan_run
 * issues it).  Negative = status. */
int rave_stream_launches(const rave_stream* s, int which);

#ifdef __cplusplus
}
#endif
#endif /* RAVE_AMD_H */
