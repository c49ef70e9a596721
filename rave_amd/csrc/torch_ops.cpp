// TorchScript binding of the model engine (TORCH_LIBRARY): the operator seam
// nn~ needs.  nn~ (a C++ Max/PD external) loads a TorchScript module and calls
// its registered methods (scripts/export.py:58-480, export_to_ts :618); ctypes
// cannot be scripted, so the engine is exposed as the custom class
// torch.classes.rave_amd.Engine whose methods take and return tensors on
// torch's current HIP stream, and which pickles (def_pickle) so a scripted
// module holding one can be saved and loaded like any .ts file.
//
// Only tensors, ints and strings cross this file; every launch goes through
// the C-ABI (include/rave_amd.h rave_model_* / rave_stream_*).
#include <torch/custom_class.h>
#include <torch/script.h>

#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>

#include <memory>
#include <string>
#include <vector>

#include "../../include/rave_amd.h"

namespace {

void check(int rc, const char* what) {
    if (rc == RAVE_OK) return;
    const std::string msg = std::string(what) + ": " + rave_last_error();
    if (rc == RAVE_ERR_ARG) TORCH_CHECK_VALUE(false, msg);
    if (rc == RAVE_ERR_UNSUPPORTED) TORCH_CHECK_NOT_IMPLEMENTED(false, msg);
    TORCH_CHECK(false, msg, " (status ", rc, ")");
}

// rave_model_config <-> a flat int list (the TorchScript-visible form) + leaky slope
// n_band .. n_ratios (7), ratios, n_dilations, dilations, am / causal / act / adain (4),
// biases (2), noise / hidden / bands / n_noise_ratios (4), noise_ratios, rvq x2 + fuse (3)
constexpr int kCfgInts = 7 + 2 * RAVE_MAX_RATIOS + RAVE_MAX_RATIOS * RAVE_MAX_DILATIONS + 4 + 2 + 4 +
                         RAVE_MAX_RATIOS + 3;

rave_model_config config_from(const std::vector<int64_t>& v, double slope) {
    TORCH_CHECK_VALUE((int)v.size() == kCfgInts, "engine config: expected ", kCfgInts, " ints, got ", v.size());
    rave_model_config c{};
    size_t i = 0;
    auto nx = [&]() { return (int32_t)v[i++]; };
    c.n_band = nx(); c.enc_bands = nx(); c.capacity = nx(); c.latent_size = nx();
    c.kernel_size = nx(); c.speaker_size = nx(); c.n_ratios = nx();
    for (int k = 0; k < RAVE_MAX_RATIOS; ++k) c.ratios[k] = nx();
    for (int k = 0; k < RAVE_MAX_RATIOS; ++k) c.n_dilations[k] = nx();
    for (int k = 0; k < RAVE_MAX_RATIOS; ++k)
        for (int j = 0; j < RAVE_MAX_DILATIONS; ++j) c.dilations[k][j] = nx();
    c.amplitude_modulation = nx(); c.causal = nx(); c.activation = nx(); c.adain = nx();
    c.conv_bias = nx(); c.convt_bias = nx();
    c.noise = nx(); c.noise_hidden = nx(); c.noise_bands = nx(); c.n_noise_ratios = nx();
    for (int k = 0; k < RAVE_MAX_RATIOS; ++k) c.noise_ratios[k] = nx();
    c.rvq_quantizers = nx(); c.rvq_codebook_size = nx(); c.fuse_units = nx();
    c.leaky_slope = (float)slope;
    return c;
}

struct Engine : torch::CustomClassHolder {
    // constructor arguments, kept for pickling
    std::vector<int64_t> cfg_ints;
    double slope;
    std::vector<std::string> names;
    std::vector<at::Tensor> params;
    at::Tensor speaker;
    int64_t precision;
    int64_t stream_block;
    // engine state
    rave_model_config cfg{};
    rave_model* m = nullptr;
    rave_stream* s_enc = nullptr;   // streaming: one state per direction (nn~'s encode / decode
    rave_stream* s_dec = nullptr;   // methods run independently), created on first use
    int64_t s_enc_b = 0, s_dec_b = 0;
    int device = 0;
    int hop = 1;

    Engine(std::vector<int64_t> ci, double sl, std::vector<std::string> nm, std::vector<at::Tensor> ps, at::Tensor spk,
           int64_t prec, int64_t block)
        : cfg_ints(std::move(ci)), slope(sl), names(std::move(nm)), params(std::move(ps)), speaker(std::move(spk)),
          precision(prec), stream_block(block) {
        TORCH_CHECK_VALUE(names.size() == params.size(), "one tensor per parameter name");
        cfg = config_from(cfg_ints, slope);
        hop = cfg.n_band;
        for (int i = 0; i < cfg.n_ratios; ++i) hop *= cfg.ratios[i];
        std::vector<at::Tensor> host;
        std::vector<rave_param> p(names.size());
        for (size_t i = 0; i < names.size(); ++i) {
            host.push_back(params[i].detach().to(at::kCPU, at::kFloat).contiguous());
            p[i] = rave_param{names[i].c_str(), host.back().data_ptr<float>(), host.back().numel()};
        }
        at::Tensor spk_h = speaker.detach().to(at::kCPU, at::kFloat).contiguous();
        device = c10::hip::current_device();
        check(rave_model_create(&cfg, p.data(), (int)p.size(), spk_h.data_ptr<float>(), (int)precision, &m),
              "rave_model_create");
    }
    ~Engine() override {
        if (s_enc) rave_stream_destroy(s_enc);
        if (s_dec) rave_stream_destroy(s_dec);
        if (m) rave_model_destroy(m);
    }

    void* cur() const { return c10::hip::getCurrentHIPStream(device).stream(); }
    void on_device(const at::Tensor& t, const char* what) const {
        TORCH_CHECK_VALUE(t.is_cuda() && t.get_device() == device, what, " must be on cuda:", device);
    }
    int64_t zc() const { return cfg.latent_size + cfg.speaker_size; }

    at::Tensor encode(at::Tensor x) {
        on_device(x, "x");
        TORCH_CHECK_VALUE(x.dim() == 3 && x.size(1) == 1 && x.scalar_type() == at::kFloat, "x must be (B, 1, T) float32");
        c10::hip::HIPGuard g((c10::DeviceIndex)device);
        x = x.contiguous();
        auto z = at::empty({x.size(0), zc(), x.size(2) / hop}, x.options());
        check(rave_model_encode(m, x.data_ptr<float>(), (int)x.size(0), (int)x.size(2), z.data_ptr<float>(), cur()),
              "encode");
        return z;
    }
    at::Tensor decode(at::Tensor z) {
        on_device(z, "z");
        TORCH_CHECK_VALUE(z.dim() == 3 && z.size(1) == zc() && z.scalar_type() == at::kFloat,
                          "z must be (B, latent + speaker, F) float32");
        c10::hip::HIPGuard g((c10::DeviceIndex)device);
        z = z.contiguous();
        auto y = at::empty({z.size(0), 1, z.size(2) * hop}, z.options());
        check(rave_model_decode(m, z.data_ptr<float>(), (int)z.size(0), (int)z.size(2), y.data_ptr<float>(), nullptr,
                                cur()),
              "decode");
        return y;
    }
    at::Tensor forward(at::Tensor x) {
        on_device(x, "x");
        TORCH_CHECK_VALUE(x.dim() == 3 && x.size(1) == 1 && x.scalar_type() == at::kFloat, "x must be (B, 1, T) float32");
        c10::hip::HIPGuard g((c10::DeviceIndex)device);
        x = x.contiguous();
        auto y = at::empty_like(x);
        check(rave_model_forward(m, x.data_ptr<float>(), (int)x.size(0), (int)x.size(2), y.data_ptr<float>(), nullptr,
                                 cur()),
              "forward");
        return y;
    }
    at::Tensor encode_codes(at::Tensor x) {
        on_device(x, "x");
        c10::hip::HIPGuard g((c10::DeviceIndex)device);
        x = x.contiguous();
        auto idx = at::empty({x.size(0), (int64_t)cfg.rvq_quantizers, x.size(2) / hop}, x.options().dtype(at::kLong));
        check(rave_model_encode_codes(m, x.data_ptr<float>(), (int)x.size(0), (int)x.size(2), idx.data_ptr<int64_t>(),
                                      cur()),
              "encode_codes");
        return idx;
    }
    at::Tensor decode_codes(at::Tensor idx) {
        on_device(idx, "idx");
        TORCH_CHECK_VALUE(idx.scalar_type() == at::kLong, "idx must be int64");
        c10::hip::HIPGuard g((c10::DeviceIndex)device);
        idx = idx.contiguous();
        auto y = at::empty({idx.size(0), 1, idx.size(2) * hop}, idx.options().dtype(at::kFloat));
        check(rave_model_decode_codes(m, idx.data_ptr<int64_t>(), (int)idx.size(0), (int)idx.size(2),
                                      y.data_ptr<float>(), nullptr, cur()),
              "decode_codes");
        return y;
    }
    // cached_conv streaming (one block of stream_block samples per call)
    // (one stream object per direction, each built for that direction only)
    rave_stream* stream_for(rave_stream*& s, int64_t& sb, int64_t batch, int direction) {
        if (!s || sb != batch) {
            if (s) rave_stream_destroy(s);
            s = nullptr;
            check(rave_stream_create(m, (int)batch, (int)stream_block, RAVE_STREAM_GRAPH | direction, &s),
                  "rave_stream_create");
            sb = batch;
        }
        return s;
    }
    at::Tensor stream_encode(at::Tensor x) {
        on_device(x, "x");
        TORCH_CHECK_VALUE(x.dim() == 3 && x.size(1) == 1 && x.size(2) == stream_block, "x must be (B, 1, block)");
        c10::hip::HIPGuard g((c10::DeviceIndex)device);
        x = x.contiguous();
        rave_stream* s = stream_for(s_enc, s_enc_b, x.size(0), RAVE_STREAM_ENCODE_ONLY);
        auto z = at::empty({x.size(0), zc(), stream_block / hop}, x.options());
        check(rave_stream_encode(s, x.data_ptr<float>(), z.data_ptr<float>(), cur()), "stream_encode");
        return z;
    }
    at::Tensor stream_decode(at::Tensor z) {
        on_device(z, "z");
        TORCH_CHECK_VALUE(z.dim() == 3 && z.size(1) == zc() && z.size(2) == stream_block / hop,
                          "z must be (B, latent + speaker, block / hop)");
        c10::hip::HIPGuard g((c10::DeviceIndex)device);
        z = z.contiguous();
        rave_stream* s = stream_for(s_dec, s_dec_b, z.size(0), RAVE_STREAM_DECODE_ONLY);
        auto y = at::empty({z.size(0), 1, stream_block}, z.options());
        check(rave_stream_decode(s, z.data_ptr<float>(), y.data_ptr<float>(), nullptr, cur()), "stream_decode");
        return y;
    }
    // discrete configs: one block of RVQ indices (B, n_q, block / hop) int64
    at::Tensor stream_encode_codes(at::Tensor x) {
        on_device(x, "x");
        TORCH_CHECK_VALUE(x.dim() == 3 && x.size(1) == 1 && x.size(2) == stream_block, "x must be (B, 1, block)");
        c10::hip::HIPGuard g((c10::DeviceIndex)device);
        x = x.contiguous();
        rave_stream* s = stream_for(s_enc, s_enc_b, x.size(0), RAVE_STREAM_ENCODE_ONLY);
        auto idx = at::empty({x.size(0), (int64_t)cfg.rvq_quantizers, stream_block / hop}, x.options().dtype(at::kLong));
        check(rave_stream_encode_codes(s, x.data_ptr<float>(), idx.data_ptr<int64_t>(), cur()), "stream_encode_codes");
        return idx;
    }
    at::Tensor stream_decode_codes(at::Tensor idx) {
        on_device(idx, "idx");
        TORCH_CHECK_VALUE(idx.dim() == 3 && idx.size(1) == cfg.rvq_quantizers && idx.size(2) == stream_block / hop &&
                              idx.scalar_type() == at::kLong,
                          "idx must be (B, n_q, block / hop) int64");
        c10::hip::HIPGuard g((c10::DeviceIndex)device);
        idx = idx.contiguous();
        rave_stream* s = stream_for(s_dec, s_dec_b, idx.size(0), RAVE_STREAM_DECODE_ONLY);
        auto y = at::empty({idx.size(0), 1, stream_block}, idx.options().dtype(at::kFloat));
        check(rave_stream_decode_codes(s, idx.data_ptr<int64_t>(), y.data_ptr<float>(), nullptr, cur()),
              "stream_decode_codes");
        return y;
    }
    void stream_reset() {
        if (s_enc) check(rave_stream_reset(s_enc, cur()), "stream_reset");
        if (s_dec) check(rave_stream_reset(s_dec, cur()), "stream_reset");
    }
    // AdaIN controls (ScriptedRAVE.update_adain): -1 keeps a flag
    void adain_control(int64_t learn_x, int64_t learn_y, bool reset_x, bool reset_y) {
        check(rave_model_adain_control(m, (int)learn_x, (int)learn_y, reset_x, reset_y, cur()), "adain_control");
    }
    // the constant speaker embedding encode concatenates (nn~ `speaker` choice)
    void set_speaker(at::Tensor emb) {
        TORCH_CHECK_VALUE(emb.numel() == cfg.speaker_size, "speaker embedding must have ", cfg.speaker_size, " values");
        c10::hip::HIPGuard g((c10::DeviceIndex)device);
        at::Tensor src = emb.detach().to(at::Device(at::kCUDA, device), at::kFloat).contiguous();
        check(rave_model_set_speaker(m, src.data_ptr<float>(), cur()), "set_speaker");
        // src came from torch's caching allocator on this stream, so freeing it on
        // return is stream-ordered after the copy
        speaker = emb.detach().cpu().to(at::kFloat).reshape({-1}).clone();    // travels with the pickle
    }
    // cooperative-unit give-ups of the calls queued so far (rave_model_check; waits for
    // the current stream); encode / decode / stream calls also raise them on entry
    void check_status() { check(rave_model_check(m, 1, cur()), "check"); }
    // launch choices (RAVE.tuning() text: "key value ms" per line), e.g. a pinned plan
    void set_tuning(const std::string& text) { check(rave_model_tuning_set(m, text.c_str()), "tuning_set"); }
    int64_t get_hop() const { return hop; }
    int64_t latent_channels() const { return zc(); }
    int64_t block() const { return stream_block; }
};

// rave_amd::fir -- the Resampler's cached_conv Conv1d (rave/resampler.py:29-58) on
// rave_fir: x (B, T) at any stride; h (P, K); y (B, P * T_out) interleaved.
// Offline: zero padding (pad_left, pad_right).  Streaming: `hist` (B, H) with
// H = pad_left + pad_right + stride_delay is the cached input (CachedConv1d),
// updated in place; T must be a multiple of the stride.
at::Tensor fir_op(at::Tensor x, at::Tensor h, int64_t stride, int64_t pad_left, int64_t pad_right,
                  c10::optional<at::Tensor> hist) {
    TORCH_CHECK_VALUE(x.is_cuda() && x.dim() == 2 && x.scalar_type() == at::kFloat, "x must be (B, T) float32 on GPU");
    TORCH_CHECK_VALUE(h.dim() == 2 && h.scalar_type() == at::kFloat, "h must be (phases, taps) float32");
    TORCH_CHECK_VALUE(stride > 0 && pad_left >= 0 && pad_right >= 0, "bad stride / padding");
    c10::hip::HIPGuard g((c10::DeviceIndex)x.get_device());
    const int64_t B = x.size(0), T = x.size(1), P = h.size(0), K = h.size(1);
    at::Tensor hd = h.to(x.device()).contiguous();
    at::Tensor src;
    int64_t t_in, t_out, pl;
    if (hist.has_value()) {
        at::Tensor hs = *hist;
        TORCH_CHECK_VALUE(hs.is_cuda() && hs.dim() == 2 && hs.size(0) == B && hs.scalar_type() == at::kFloat,
                          "hist must be (B, H) float32 on the GPU");
        TORCH_CHECK_VALUE(T % stride == 0, "streaming block must be a multiple of the stride");
        src = at::cat({hs, x}, 1).contiguous();
        t_in = src.size(1);
        t_out = T / stride;
        pl = 0;
    } else {
        src = x.contiguous();
        t_in = T;
        t_out = (T + pad_left + pad_right - K) / stride + 1;
        pl = pad_left;
    }
    TORCH_CHECK_VALUE(t_out > 0, "input too short");
    auto y = at::empty({B, P * t_out}, x.options());
    rave_fir_args a{};
    a.batch = (int)B; a.t_in = (int)t_in; a.t_out = (int)t_out; a.phases = (int)P; a.taps = (int)K;
    a.stride = (int)stride; a.pad_left = (int)pl;
    a.x = src.data_ptr<float>(); a.x_sb = src.stride(0);
    a.y = y.data_ptr<float>(); a.y_sb = y.stride(0);
    a.h = hd.data_ptr<float>();
    check(rave_fir(&a, c10::hip::getCurrentHIPStream(x.get_device()).stream()), "fir");
    if (hist.has_value()) {
        at::Tensor hs = *hist;
        hs.copy_(src.narrow(1, T, hs.size(1)));      // newest H samples become the cache
    }
    return y;
}

// ============================================================== operator seam
// The cc.* operators the reference's blocks construct (rave/blocks.py:65,97,
// 182,566; rave/__init__.py:14-27) and CachedPQMF's two convolutions
// (rave/pqmf.py:234-284), as torch.ops.rave_amd.* -- the kernels behind the
// rave_amd.cc nn.Modules.  Tensors on the GPU, time contiguous; launches on
// torch's current HIP stream; every op goes through the C-ABI.
void seam_tensor(const at::Tensor& t, const char* what) {
    TORCH_CHECK_VALUE(t.is_cuda() && t.scalar_type() == at::kFloat, what, " must be a float32 GPU tensor");
    TORCH_CHECK_VALUE(t.dim() == 3 && t.stride(2) == 1, what, " must be (B, C, T) with T contiguous");
}
void* cur_stream(const at::Tensor& t) { return c10::hip::getCurrentHIPStream(t.get_device()).stream(); }

// rave_amd::pack_conv1d -- rave_conv1d_pack_weight / rave_conv1d_split_pack_weight
// on the host (torch layout in: Conv1d (c_out, c_in, k), ConvTranspose1d
// (c_in, c_out, k)); a CPU float tensor out
at::Tensor pack_conv1d_op(at::Tensor w, int64_t c_in, int64_t c_out, int64_t kernel, int64_t stride, int64_t dilation,
                          bool transposed, int64_t out_shift, int64_t precision) {
    TORCH_CHECK_VALUE(precision == RAVE_PREC_F32 || precision == RAVE_PREC_SPLIT16, "precision: 0 (f32) or 1 (split16)");
    at::Tensor wc = w.detach().to(at::kCPU, at::kFloat).contiguous();
    TORCH_CHECK_VALUE(wc.numel() == c_in * c_out * kernel, "weight has ", wc.numel(), " values, expected ",
                      c_in * c_out * kernel);
    const bool sp = precision == RAVE_PREC_SPLIT16;
    const int64_t n = sp ? rave_conv1d_split_packed_size((int)c_in, (int)c_out, (int)kernel, (int)stride, (int)dilation,
                                                         transposed)
                         : rave_conv1d_packed_size((int)c_in, (int)c_out, (int)kernel, (int)stride, (int)dilation,
                                                   transposed);
    TORCH_CHECK_NOT_IMPLEMENTED(n > 0, "conv1d: unsupported layer shape (c_in ", c_in, ", kernel ", kernel, ", stride ",
                                stride, ", dilation ", dilation, ")");
    at::Tensor out = at::zeros({n}, at::kFloat);
    check(sp ? rave_conv1d_split_pack_weight(wc.data_ptr<float>(), (int)c_in, (int)c_out, (int)kernel, (int)stride,
                                             (int)dilation, transposed, (int)out_shift, out.data_ptr<float>())
             : rave_conv1d_pack_weight(wc.data_ptr<float>(), (int)c_in, (int)c_out, (int)kernel, (int)stride,
                                       (int)dilation, transposed, (int)out_shift, out.data_ptr<float>()),
          "pack_conv1d");
    return out;
}

// rave_amd::conv1d -- rave_conv1d: act(x) conv W (+ bias) (+ residual).
// transposed: the polyphase ConvTranspose1d (offline: pad_left 0, out_shift
// stride/2; cached: x starts with one history column, pad_left 1, out_shift 0).
at::Tensor conv1d_op(at::Tensor x, at::Tensor packed, c10::optional<at::Tensor> bias, c10::optional<at::Tensor> alpha,
                     c10::optional<at::Tensor> residual, int64_t c_out, int64_t kernel, int64_t stride, int64_t dilation,
                     int64_t pad_left, int64_t pad_right, bool transposed, int64_t out_shift, int64_t act, double slope,
                     int64_t precision) {
    seam_tensor(x, "x");
    c10::hip::HIPGuard g((c10::DeviceIndex)x.get_device());
    TORCH_CHECK_VALUE(packed.device() == x.device(), "packed weight must be on x's device");
    const int64_t B = x.size(0), c_in = x.size(1), T = x.size(2);
    int64_t t_out;
    if (transposed) {
        t_out = (T - pad_left) * stride;
    } else {
        const int64_t span = (kernel - 1) * dilation + 1;
        t_out = (T + pad_left + pad_right - span) / stride + 1;
    }
    TORCH_CHECK_VALUE(t_out > 0, "conv1d: input too short");
    at::Tensor y = at::empty({B, c_out, t_out}, x.options());
    rave_conv1d_args a{};
    a.c_in = (int)c_in; a.c_out = (int)c_out; a.kernel = (int)kernel; a.stride = (int)stride; a.dilation = (int)dilation;
    a.pad_left = (int)pad_left; a.pad_right = transposed ? 0 : (int)pad_right; a.transposed = transposed;
    a.out_shift = (int)out_shift; a.act = (int)act; a.leaky_slope = (float)slope; a.batch = (int)B;
    a.t_in = (int)T; a.t_out = (int)t_out; a.precision = (int)precision;
    a.x = x.data_ptr<float>(); a.x_sb = x.stride(0); a.x_sc = x.stride(1);
    a.y = y.data_ptr<float>(); a.y_sb = y.stride(0); a.y_sc = y.stride(1);
    at::Tensor res;
    if (residual.has_value()) {
        res = *residual;
        seam_tensor(res, "residual");
        TORCH_CHECK_VALUE(res.size(0) == B && res.size(1) == c_out && res.size(2) == t_out, "residual shape");
        a.residual = res.data_ptr<float>(); a.r_sb = res.stride(0); a.r_sc = res.stride(1);
    }
    a.weight = packed.data_ptr<float>();
    at::Tensor bd, ad;
    if (bias.has_value()) {
        bd = bias->to(x.device(), at::kFloat).contiguous();
        TORCH_CHECK_VALUE(bd.numel() == c_out, "bias must have c_out values");
        a.bias = bd.data_ptr<float>();
    }
    if (act == RAVE_ACT_SNAKE) {
        TORCH_CHECK_VALUE(alpha.has_value(), "Snake needs alpha");
        ad = alpha->to(x.device(), at::kFloat).contiguous();
        TORCH_CHECK_VALUE(ad.numel() == c_in, "alpha must have c_in values");
        a.alpha = ad.data_ptr<float>();
    }
    const int64_t nws = rave_conv1d_workspace(&a);
    if (nws < 0) check((int)nws, "conv1d workspace");
    at::Tensor ws;
    if (nws > 0) {
        ws = at::zeros({nws}, x.options());      // split-K arrival counters start (and end) zero
        a.partial = ws.data_ptr<float>();
    }
    check(rave_conv1d(&a, cur_stream(x)), "conv1d");
    return y;
}

// rave_amd::pqmf_analysis -- CachedPQMF.forward (rave/pqmf.py:269-273): x (B, 1, T)
// -> (B, n_out_bands, T / n_band); hkf (n_band, taps) on x's device
at::Tensor pqmf_analysis_op(at::Tensor x, at::Tensor hkf, int64_t n_out_bands, int64_t pad_left, int64_t precision) {
    seam_tensor(x, "x");
    c10::hip::HIPGuard g((c10::DeviceIndex)x.get_device());
    TORCH_CHECK_VALUE(x.size(1) == 1, "x must be (B, 1, T)");
    at::Tensor h = hkf.to(x.device(), at::kFloat).contiguous();
    const int64_t nb = h.size(0), B = x.size(0), T = x.size(2);
    TORCH_CHECK_VALUE(T % nb == 0, "T must be a multiple of n_band");
    at::Tensor y = at::empty({B, n_out_bands, T / nb}, x.options());
    rave_pqmf_analysis_args a{};
    a.n_band = (int)nb; a.taps = (int)h.size(1); a.n_out_bands = (int)n_out_bands; a.batch = (int)B;
    a.t_in = (int)T; a.pad_left = (int)pad_left; a.t_out = (int)(T / nb); a.precision = (int)precision;
    a.x = x.data_ptr<float>(); a.x_sb = x.stride(0);
    a.y = y.data_ptr<float>(); a.y_sb = y.stride(0); a.y_sc = y.stride(1);
    a.hkf = h.data_ptr<float>();
    check(rave_pqmf_analysis(&a, cur_stream(x)), "pqmf_analysis");
    return y;
}

// rave_amd::pqmf_synthesis -- CachedPQMF.inverse (rave/pqmf.py:275-284): x (B, n_band, F)
// -> (B, 1, F * n_band); hki (n_band, n_band, taps).  x_len > F: x carries
// cached history columns before the F frames (streaming, pad_left 0).
// mode 1 / 2: GeneratorV2's epilogue fused in front (rave/blocks.py:699-707):
// x holds 2 n_band channels (waveform, amplitude) and the input is
// tanh(x[:n] * sigmoid(x[n:]) + noise) (mode 1) or tanh(x + noise) (mode 2);
// noise (B, n_band, x_len) or None.
at::Tensor pqmf_synthesis_op(at::Tensor x, at::Tensor hki, int64_t pad_left, int64_t frames, int64_t frame0,
                             int64_t precision, int64_t mode, c10::optional<at::Tensor> noise) {
    seam_tensor(x, "x");
    c10::hip::HIPGuard g((c10::DeviceIndex)x.get_device());
    at::Tensor h = hki.to(x.device(), at::kFloat).contiguous();
    const int64_t nb = h.size(0), B = x.size(0), XL = x.size(2);
    TORCH_CHECK_VALUE(mode >= 0 && mode <= 2, "mode must be 0 (plain), 1 (amplitude modulation) or 2 (tanh)");
    TORCH_CHECK_VALUE(x.size(1) == (mode == 1 ? 2 * nb : nb), "x must have ", mode == 1 ? 2 * nb : nb, " channels");
    TORCH_CHECK_VALUE(mode != 0 || !noise.has_value(), "noise needs an epilogue mode");
    const int64_t F = frames > 0 ? frames : XL;
    at::Tensor y = at::empty({B, 1, F * nb}, x.options());
    rave_pqmf_synthesis_args a{};
    a.n_band = (int)nb; a.taps = (int)h.size(2); a.batch = (int)B; a.t_in = (int)F; a.pad_left = (int)pad_left;
    a.mode = (int)mode; a.frame0 = (int)frame0; a.x_len = (int)XL;
    a.x = x.data_ptr<float>(); a.x_sb = x.stride(0); a.x_sc = x.stride(1);
    at::Tensor nz;
    if (noise.has_value()) {
        nz = *noise;
        seam_tensor(nz, "noise");
        TORCH_CHECK_VALUE(nz.dim() == 3 && nz.size(0) == B && nz.size(1) == nb && nz.size(2) == XL && nz.stride(2) == 1,
                          "noise must be (B, n_band, x_len), time contiguous");
        a.noise = nz.data_ptr<float>(); a.n_sb = nz.stride(0); a.n_sc = nz.stride(1);
    }
    a.y = y.data_ptr<float>(); a.y_sb = y.stride(0);
    a.hki = h.data_ptr<float>(); a.precision = (int)precision;
    check(rave_pqmf_synthesis(&a, cur_stream(x)), "pqmf_synthesis");
    return y;
}

// rave_amd::adain -- AdaptiveInstanceNormalization.forward in eval mode
// (rave/blocks.py:856-919) on rave_adain over the module's own buffers
// (mean_x / std_x / mean_y / std_y (max_batch, C, 1), num_update_x / _y (1,)):
// mode 0 transfer (when both counters are set), 1 learn_x then transfer,
// 2 learn_y; a learning mode writes the updated statistics back.
at::Tensor adain_op(at::Tensor x, at::Tensor mean_x, at::Tensor std_x, at::Tensor mean_y, at::Tensor std_y,
                    at::Tensor num_update_x, at::Tensor num_update_y, int64_t mode) {
    seam_tensor(x, "x");
    TORCH_CHECK_VALUE(x.dim() == 3, "x must be (B, C, T)");
    TORCH_CHECK_VALUE(mode >= 0 && mode <= 2, "mode must be 0 (transfer), 1 (learn_x) or 2 (learn_y)");
    c10::hip::HIPGuard g((c10::DeviceIndex)x.get_device());
    const int64_t B = x.size(0), C = x.size(1), T = x.size(2), mb = mean_x.size(0);
    for (const at::Tensor* t : {&mean_x, &std_x, &mean_y, &std_y})
        TORCH_CHECK_VALUE(t->dim() == 3 && t->size(0) == mb && t->size(1) == C && t->size(2) == 1,
                          "AdaIN statistics must be (max_batch, C, 1)");
    TORCH_CHECK_VALUE(B <= mb, "batch exceeds the AdaIN buffers' max_batch");
    TORCH_CHECK_VALUE(T >= 2 || mode == 0, "learning needs at least 2 samples (unbiased std)");
    at::Tensor xc = x.contiguous();
    at::Tensor stats = at::stack({mean_x, std_x, mean_y, std_y}).to(x.device(), at::kFloat).reshape({4, mb, C})
                           .contiguous();
    at::Tensor cnt = at::cat({num_update_x.reshape({1}), num_update_y.reshape({1})}).to(x.device(), at::kFloat)
                         .contiguous();
    at::Tensor ticket = at::zeros({1}, x.options().dtype(at::kInt));
    at::Tensor y = at::empty_like(xc);
    rave_adain_args a{};
    a.batch = (int)B; a.channels = (int)C; a.t_len = (int)T; a.mode = (int)mode; a.max_batch = (int)mb; a.row0 = 0;
    a.x = xc.data_ptr<float>(); a.x_sb = xc.stride(0); a.x_sc = xc.stride(1);
    a.y = y.data_ptr<float>(); a.y_sb = y.stride(0); a.y_sc = y.stride(1);
    a.stats = stats.data_ptr<float>();
    a.counters = cnt.data_ptr<float>();
    a.ticket = reinterpret_cast<uint32_t*>(ticket.data_ptr<int32_t>());
    check(rave_adain(&a, cur_stream(x)), "adain");
    if (mode == 1) {
        mean_x.copy_(stats[0].reshape(mean_x.sizes()));
        std_x.copy_(stats[1].reshape(std_x.sizes()));
        num_update_x.copy_(cnt.narrow(0, 0, 1).reshape(num_update_x.sizes()));
    } else if (mode == 2) {
        mean_y.copy_(stats[2].reshape(mean_y.sizes()));
        std_y.copy_(stats[3].reshape(std_y.sizes()));
        num_update_y.copy_(cnt.narrow(0, 1, 1).reshape(num_update_y.sizes()));
    }
    return y;
}

// rave_amd::noise_synth -- NoiseGeneratorV2's filter stage after its conv stack
// (rave/blocks.py:281-291, rave/core.py:66-129) on rave_noise_synth: amp
// (B, n_band * noise_bands, F) pre-sigmoid, u (B, F, n_band, target) U[0,1)
// (torch.rand_like(ir)) -> noise (B, n_band, F * target).
at::Tensor noise_synth_op(at::Tensor amp, at::Tensor u, int64_t n_band, int64_t noise_bands) {
    seam_tensor(amp, "amp");
    TORCH_CHECK_VALUE(u.is_cuda() && u.scalar_type() == at::kFloat, "u must be a float32 GPU tensor");
    c10::hip::HIPGuard g((c10::DeviceIndex)amp.get_device());
    TORCH_CHECK_VALUE(amp.dim() == 3 && amp.size(1) == n_band * noise_bands, "amp must be (B, n_band * noise_bands, F)");
    const int64_t B = amp.size(0), F = amp.size(2);
    TORCH_CHECK_VALUE(u.dim() == 4 && u.size(0) == B && u.size(1) == F && u.size(2) == n_band,
                      "u must be (B, F, n_band, target)");
    const int64_t target = u.size(3);
    at::Tensor ac = amp.contiguous(), uc = u.contiguous();
    at::Tensor y = at::empty({B, n_band, F * target}, amp.options());
    rave_noise_args a{};
    a.batch = (int)B; a.frames = (int)F; a.n_band = (int)n_band; a.noise_bands = (int)noise_bands;
    a.target = (int)target;
    a.amp = ac.data_ptr<float>(); a.a_sb = ac.stride(0); a.a_sc = ac.stride(1);
    a.u = uc.data_ptr<float>(); a.u_sb = uc.stride(0);
    a.y = y.data_ptr<float>(); a.y_sb = y.stride(0); a.y_sc = y.stride(1);
    check(rave_noise_synth(&a, cur_stream(amp)), "noise_synth");
    return y;
}

// rave_amd::delay_line -- cached_conv's CachedPadding1d on rave_copy: returns
// [state[:B] | x] (B, C, P + T), or its first T columns when `crop` (a pure
// P-sample delay), and keeps the newest P columns in `state` (max_batch, C, P).
at::Tensor delay_line_op(at::Tensor x, at::Tensor state, bool crop) {
    seam_tensor(x, "x");
    seam_tensor(state, "state");
    c10::hip::HIPGuard g((c10::DeviceIndex)x.get_device());
    TORCH_CHECK_VALUE(x.dim() == 3 && state.dim() == 3 && state.size(1) == x.size(1) && state.size(0) >= x.size(0) &&
                          state.is_contiguous(),
                      "state must be a contiguous (max_batch, C, P) buffer with x's channels");
    const int64_t B = x.size(0), C = x.size(1), T = x.size(2), P = state.size(2);
    at::Tensor xc = x.contiguous();
    at::Tensor full = at::empty({B, C, P + T}, x.options());
    void* st = cur_stream(x);
    auto copy = [&](const float* src, int64_t s_sb, int64_t s_sc, float* dst, int64_t d_sb, int64_t d_sc, int64_t n) {
        if (n <= 0) return;
        rave_copy_args a{};
        a.batch = (int)B; a.channels = (int)C; a.t_len = (int)n;
        a.x = src; a.x_sb = s_sb; a.x_sc = s_sc;
        a.y = dst; a.y_sb = d_sb; a.y_sc = d_sc;
        check(rave_copy(&a, st), "delay_line");
    };
    float* f = full.data_ptr<float>();
    float* sp = state.data_ptr<float>();
    copy(sp, C * P, P, f, C * (P + T), P + T, P);                                   // history
    copy(xc.data_ptr<float>(), xc.stride(0), xc.stride(1), f + P, C * (P + T), P + T, T);   // block
    copy(f + T, C * (P + T), P + T, sp, C * P, P, P);                               // newest P -> state
    return crop ? full.narrow(2, 0, T) : full;
}

// rave_amd::rvq_encode / rvq_decode -- ResidualVectorQuantization.encode / decode
// (rave/quantization.py:302-318): z (B, D, T), codebooks (n_q, K, D) -> idx (B, n_q, T) int64
at::Tensor rvq_encode_op(at::Tensor z, at::Tensor codebooks) {
    seam_tensor(z, "z");
    c10::hip::HIPGuard g((c10::DeviceIndex)z.get_device());
    at::Tensor cb = codebooks.to(z.device(), at::kFloat).contiguous();
    TORCH_CHECK_VALUE(cb.dim() == 3 && cb.size(2) == z.size(1), "codebooks must be (n_q, K, D)");
    const int64_t B = z.size(0), D = z.size(1), T = z.size(2), nq = cb.size(0);
    at::Tensor idx = at::empty({B, nq, T}, z.options().dtype(at::kLong));
    rave_rvq_args a{};
    a.n_q = (int)nq; a.codebook_size = (int)cb.size(1); a.dim = (int)D; a.batch = (int)B; a.t_len = (int)T;
    a.codebooks = cb.data_ptr<float>();
    a.z = z.data_ptr<float>(); a.z_sb = z.stride(0); a.z_sc = z.stride(1);
    a.idx = idx.data_ptr<int64_t>(); a.i_sb = nq * T; a.i_sq = T;
    const int64_t nw = rave_rvq_workspace(&a);
    if (nw < 0) check((int)nw, "rvq_workspace");
    at::Tensor work = at::empty({std::max<int64_t>(nw, 1)}, z.options());
    a.work = work.data_ptr<float>();
    check(rave_rvq_encode(&a, cur_stream(z)), "rvq_encode");
    return idx;
}

at::Tensor rvq_decode_op(at::Tensor idx, at::Tensor codebooks) {
    TORCH_CHECK_VALUE(idx.is_cuda() && idx.scalar_type() == at::kLong && idx.dim() == 3, "idx must be (B, n_q, T) int64");
    c10::hip::HIPGuard g((c10::DeviceIndex)idx.get_device());
    at::Tensor ic = idx.contiguous();
    at::Tensor cb = codebooks.to(idx.device(), at::kFloat).contiguous();
    TORCH_CHECK_VALUE(cb.dim() == 3 && cb.size(0) == idx.size(1), "codebooks must be (n_q, K, D)");
    const int64_t B = idx.size(0), nq = idx.size(1), T = idx.size(2), D = cb.size(2);
    at::Tensor y = at::empty({B, D, T}, idx.options().dtype(at::kFloat));
    rave_rvq_args a{};
    a.n_q = (int)nq; a.codebook_size = (int)cb.size(1); a.dim = (int)D; a.batch = (int)B; a.t_len = (int)T;
    a.codebooks = cb.data_ptr<float>();
    a.idx = ic.data_ptr<int64_t>(); a.i_sb = nq * T; a.i_sq = T;
    a.y = y.data_ptr<float>(); a.y_sb = D * T; a.y_sc = T;
    check(rave_rvq_decode(&a, cur_stream(idx)), "rvq_decode");
    return y;
}

using State = std::tuple<std::vector<int64_t>, double, std::vector<std::string>, std::vector<at::Tensor>, at::Tensor,
                         int64_t, int64_t>;

}  // namespace

TORCH_LIBRARY(rave_amd, lib) {
    lib.def("fir(Tensor x, Tensor h, int stride, int pad_left, int pad_right, Tensor? hist) -> Tensor", &fir_op);
    lib.def("pack_conv1d(Tensor w, int c_in, int c_out, int kernel, int stride, int dilation, bool transposed, "
            "int out_shift, int precision) -> Tensor", &pack_conv1d_op);
    lib.def("conv1d(Tensor x, Tensor packed, Tensor? bias, Tensor? alpha, Tensor? residual, int c_out, int kernel, "
            "int stride, int dilation, int pad_left, int pad_right, bool transposed, int out_shift, int act, "
            "float slope, int precision) -> Tensor", &conv1d_op);
    lib.def("pqmf_analysis(Tensor x, Tensor hkf, int n_out_bands, int pad_left, int precision) -> Tensor",
            &pqmf_analysis_op);
    lib.def("pqmf_synthesis(Tensor x, Tensor hki, int pad_left, int frames, int frame0, int precision, int mode=0, "
            "Tensor? noise=None) -> Tensor",
            &pqmf_synthesis_op);
    lib.def("adain(Tensor x, Tensor(a!) mean_x, Tensor(b!) std_x, Tensor(c!) mean_y, Tensor(d!) std_y, "
            "Tensor(e!) num_update_x, Tensor(f!) num_update_y, int mode) -> Tensor",
            &adain_op);
    lib.def("noise_synth(Tensor amp, Tensor u, int n_band, int noise_bands) -> Tensor", &noise_synth_op);
    lib.def("delay_line(Tensor x, Tensor(a!) state, bool crop) -> Tensor", &delay_line_op);
    lib.def("rvq_encode(Tensor z, Tensor codebooks) -> Tensor", &rvq_encode_op);
    lib.def("rvq_decode(Tensor idx, Tensor codebooks) -> Tensor", &rvq_decode_op);
    lib.class_<Engine>("Engine")
        .def(torch::init<std::vector<int64_t>, double, std::vector<std::string>, std::vector<at::Tensor>, at::Tensor,
                         int64_t, int64_t>())
        .def("encode", &Engine::encode)
        .def("decode", &Engine::decode)
        .def("forward", &Engine::forward)
        .def("encode_codes", &Engine::encode_codes)
        .def("decode_codes", &Engine::decode_codes)
        .def("stream_encode", &Engine::stream_encode)
        .def("stream_decode", &Engine::stream_decode)
        .def("stream_encode_codes", &Engine::stream_encode_codes)
        .def("stream_decode_codes", &Engine::stream_decode_codes)
        .def("stream_reset", &Engine::stream_reset)
        .def("adain_control", &Engine::adain_control)
        .def("set_speaker", &Engine::set_speaker)
        .def("check", &Engine::check_status)
        .def("set_tuning", &Engine::set_tuning)
        .def("hop", &Engine::get_hop)
        .def("latent_channels", &Engine::latent_channels)
        .def("block", &Engine::block)
        .def_pickle(
            [](const c10::intrusive_ptr<Engine>& e) -> State {
                std::vector<at::Tensor> ps;
                for (auto& p : e->params) ps.push_back(p.detach().cpu());
                return State(e->cfg_ints, e->slope, e->names, ps, e->speaker.detach().cpu(), e->precision,
                             e->stream_block);
            },
            [](State st) -> c10::intrusive_ptr<Engine> {
                return c10::make_intrusive<Engine>(std::get<0>(st), std::get<1>(st), std::get<2>(st), std::get<3>(st),
                                                   std::get<4>(st), std::get<5>(st), std::get<6>(st));
            });
}
