// Model engine: RAVE.encode / decode / forward (rave/model.py:594-634) as a
// native object (include/rave_amd.h "model engine").
//
//   * graph      -- EncoderV2 (rave/blocks.py:508-597), GeneratorV2 (:600-710),
//                   NoiseGeneratorV2 (:244-291), Residual(DilatedUnit) (:32-113)
//                   restated as an ordered conv list named after the reference's
//                   state_dict (the same table as rave_amd/graph.py);
//   * weights    -- weight norm folded (rave/blocks.py:17-24, w = g v / ||v||),
//                   packed once per arithmetic into one device arena;
//   * plans      -- per (call, batch, length): a liveness-planned workspace,
//                   fused Residual(DilatedUnit) and residual-stack launches where
//                   they run, the AdaIN ops, the PQMF / RVQ / noise ops, replayed
//                   by the rave_plan executor with per-call I/O relocation;
//   * autotuner  -- with RAVE_PREC_AUTO every conv is timed in both arithmetics
//                   and every launch configuration, every unit fused against its
//                   two convs, every stack against its units; the fastest wins.
#include "engine.h"
#include "shift_batch.h"

#include <cstdlib>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>
#include <sstream>

namespace rave {

// =================================================================== graph
std::pair<int, int> get_padding(int k, int dilation, bool causal) {
    if (k == 1) return {0, 0};
    const int p = (k - 1) * dilation + 1;
    if (causal) return {p - 1, 0};
    return {(p - 1) / 2, p / 2};
}

int Node::out_len(int t_in) const {
    if (transposed) return (t_in - 1) * stride - 2 * (stride / 2) + kernel;
    const int span = (kernel - 1) * dilation + 1;
    return (t_in + pad_l + pad_r - span) / stride + 1;
}

std::vector<const Node*> Graph::convs() const {
    std::vector<const Node*> v;
    for (auto* l : {&encoder, &decoder, &noise})
        for (const Node& n : *l) v.push_back(&n);
    return v;
}

static void check_config(const rave_model_config& c) {
    auto bad = [](const std::string& m) { fail(RAVE_ERR_ARG, "model config: " + m); };
    if (c.n_band <= 0 || c.enc_bands <= 0 || c.enc_bands > c.n_band) bad("n_band / enc_bands");
    if (c.capacity <= 0 || c.latent_size <= 0 || c.kernel_size <= 0 || c.speaker_size < 0) bad("sizes");
    if (c.n_ratios <= 0 || c.n_ratios > RAVE_MAX_RATIOS) bad("n_ratios");
    for (int i = 0; i < c.n_ratios; ++i) {
        if (c.ratios[i] <= 0) bad("ratios");
        if (c.n_dilations[i] < 0 || c.n_dilations[i] > RAVE_MAX_DILATIONS) bad("n_dilations");
        for (int j = 0; j < c.n_dilations[i]; ++j)
            if (c.dilations[i][j] <= 0) bad("dilations");
    }
    if (c.activation != RAVE_ACT_LEAKY && c.activation != RAVE_ACT_SNAKE) bad("activation");
    if (c.noise && (c.n_noise_ratios <= 0 || c.n_noise_ratios > RAVE_MAX_RATIOS || c.noise_bands <= 1 ||
                    c.noise_hidden <= 0))
        bad("noise");
    if (c.rvq_quantizers < 0 || (c.rvq_quantizers > 0 && c.rvq_codebook_size <= 0)) bad("rvq");
}

void build_graph(const rave_model_config& c, Graph& g) {
    check_config(c);
    const int ks = c.kernel_size;
    const bool causal = c.causal != 0;
    int tid = 0;
    auto new_t = [&](char p) { return std::string(1, p) + std::to_string(++tid); };
    auto act_of = [&](const std::string& module, Node& n) {
        n.act = c.activation;
        if (c.activation == RAVE_ACT_SNAKE) n.alpha = module + ".alpha";
    };
    auto conv = [&](const std::string& name, int ci, int co, int k, int stride, int dil, std::pair<int, int> pad,
                    const std::string& src, const std::string& dst) {
        Node n;
        n.name = name;
        n.c_in = ci;
        n.c_out = co;
        n.kernel = k;
        n.stride = stride;
        n.dilation = dil;
        n.pad_l = pad.first;
        n.pad_r = pad.second;
        n.bias = c.conv_bias != 0;
        n.src = src;
        n.dst = dst;
        return n;
    };
    // Residual(DilatedUnit(ch, ks, d)): act -> conv(k, d) -> act -> conv 1x1, + x
    auto unit = [&](std::vector<Node>& out, const std::string& res, int ch, int d, const std::string& src,
                    const std::string& adain) {
        const std::string u = res + ".aligned.branches.0.net";
        const char pfx = &out == &g.encoder ? 'e' : 'd';
        const std::string mid = new_t(pfx);
        const std::string dst = new_t(pfx);
        Node a = conv(u + ".1", ch, ch, ks, 1, d, get_padding(ks, d, causal), src, mid);
        act_of(u + ".0", a);
        a.adain = adain;
        out.push_back(a);
        Node b = conv(u + ".3", ch, ch, 1, 1, 1, {0, 0}, mid, dst);
        act_of(u + ".2", b);
        b.residual = src;
        b.res_delay = (a.pad_r + a.stride_delay()) / a.stride;   // Residual's AlignBranches(delays=[d, 0])
        out.push_back(b);
    };

    // ---------------------------------------------------------- encoder
    std::string pre = "encoder.encoder.net";
    int idx = 0;
    std::string cur = new_t('e');
    g.encoder.push_back(conv(pre + "." + std::to_string(idx), c.enc_bands, c.capacity, 2 * ks + 1, 1, 1,
                             get_padding(2 * ks + 1, 1, causal), "enc_in", cur));
    ++idx;
    int ch = c.capacity;
    for (int i = 0; i < c.n_ratios; ++i) {
        const int r = c.ratios[i];
        for (int j = 0; j < c.n_dilations[i]; ++j) {
            std::string adain;
            if (c.adain) {
                adain = pre + "." + std::to_string(idx);
                g.adain_modules.push_back({adain, ch});
                ++idx;
            }
            unit(g.encoder, pre + "." + std::to_string(idx), ch, c.dilations[i][j], cur, adain);
            cur = g.encoder.back().dst;
            ++idx;
        }
        const std::string act_mod = pre + "." + std::to_string(idx);
        ++idx;
        const std::string nxt = new_t('e');
        Node n = conv(pre + "." + std::to_string(idx), ch, 2 * ch, 2 * r, r, 1, get_padding(2 * r, 1, causal), cur, nxt);
        act_of(act_mod, n);
        g.encoder.push_back(n);
        cur = nxt;
        ++idx;
        ch *= 2;
    }
    {
        const std::string act_mod = pre + "." + std::to_string(idx);
        ++idx;
        Node n = conv(pre + "." + std::to_string(idx), ch, c.latent_size, ks, 1, 1, get_padding(ks, 1, causal), cur,
                      "latent");
        act_of(act_mod, n);
        g.encoder.push_back(n);
    }

    // ---------------------------------------------------------- decoder
    pre = "decoder.net";
    idx = 0;
    ch = (1 << c.n_ratios) * c.capacity;
    const int dec_in = c.latent_size + c.speaker_size;
    cur = new_t('d');
    g.decoder.push_back(conv(pre + ".0", dec_in, ch, ks, 1, 1, get_padding(ks, 1, causal), "dec_in", cur));
    ++idx;
    for (int i = c.n_ratios - 1; i >= 0; --i) {
        const int r = c.ratios[i];
        const std::string act_mod = pre + "." + std::to_string(idx);
        ++idx;
        const std::string nxt = new_t('d');
        Node n = conv(pre + "." + std::to_string(idx), ch, ch / 2, 2 * r, r, 1, {r / 2, r / 2}, cur, nxt);
        n.transposed = true;
        n.bias = c.convt_bias != 0;
        act_of(act_mod, n);
        g.decoder.push_back(n);
        cur = nxt;
        ++idx;
        ch /= 2;
        for (int j = 0; j < c.n_dilations[i]; ++j) {
            std::string adain;
            if (c.adain) {
                adain = pre + "." + std::to_string(idx);
                g.adain_modules.push_back({adain, ch});
                ++idx;
            }
            unit(g.decoder, pre + "." + std::to_string(idx), ch, c.dilations[i][j], cur, adain);
            cur = g.decoder.back().dst;
            ++idx;
        }
    }
    const std::string act_mod = pre + "." + std::to_string(idx);
    ++idx;
    const std::string wave_name = c.noise ? std::string("decoder.waveform_module") : pre + "." + std::to_string(idx);
    const int dec_out = c.amplitude_modulation ? 2 * c.n_band : c.n_band;
    Node w = conv(wave_name, ch, dec_out, 2 * ks + 1, 1, 1, get_padding(2 * ks + 1, 1, causal), cur, "wave");
    act_of(act_mod, w);
    g.decoder.push_back(w);

    // ---------------------------------------------------------- noise synthesizer
    if (c.noise) {
        std::vector<int> chans{ch};
        for (int i = 0; i + 1 < c.n_noise_ratios; ++i) chans.push_back(c.noise_hidden);
        chans.push_back(c.n_band * c.noise_bands);
        std::string src = cur;
        const std::string npre = "decoder.noise_module.net";
        int j = 0;
        for (int i = 0; i < c.n_noise_ratios; ++i) {
            const int r = c.noise_ratios[i];
            const std::string dst = i == c.n_noise_ratios - 1 ? std::string("noise_amp") : new_t('n');
            Node n = conv(npre + "." + std::to_string(j), chans[i], chans[i + 1], 2 * r, r, 1, {r, 0}, src, dst);
            n.weight_norm = false;
            if (i == 0) {   // consumes the activated decoder features: the waveform conv's activation
                n.act = w.act;
                n.alpha = w.alpha;
            } else {
                act_of(npre + "." + std::to_string(j - 1), n);
            }
            g.noise.push_back(n);
            src = dst;
            j += (i != c.n_noise_ratios - 1) ? 2 : 1;
        }
    }
}

std::vector<std::pair<std::string, std::vector<int64_t>>> param_table(const rave_model_config& c) {
    Graph g;
    build_graph(c, g);
    std::vector<std::pair<std::string, std::vector<int64_t>>> out;
    std::set<std::string> seen;
    for (const Node* n : g.convs()) {
        std::vector<int64_t> ws = n->transposed ? std::vector<int64_t>{n->c_in, n->c_out, n->kernel}
                                                : std::vector<int64_t>{n->c_out, n->c_in, n->kernel};
        if (n->weight_norm) {
            out.push_back({n->name + ".weight_g", {ws[0], 1, 1}});
            out.push_back({n->name + ".weight_v", ws});
        } else {
            out.push_back({n->name + ".weight", ws});
        }
        if (n->bias) out.push_back({n->name + ".bias", {n->c_out}});
        if (n->act == RAVE_ACT_SNAKE && !seen.count(n->alpha)) {
            seen.insert(n->alpha);
            out.push_back({n->alpha, {n->c_in, 1}});
        }
    }
    for (int i = 0; i < c.rvq_quantizers; ++i)
        out.push_back({"encoder.rvq.layers." + std::to_string(i) + "._codebook.embed",
                       {c.rvq_codebook_size, c.latent_size}});
    out.push_back({"pqmf.hk", {}});
    return out;
}

// =================================================================== workspace / plan
int64_t Workspace::alloc(int64_t n) {
    n = round(n);
    for (size_t i = 0; i < free_.size(); ++i) {
        if (free_[i].second >= n) {
            const int64_t off = free_[i].first;
            if (free_[i].second == n) free_.erase(free_.begin() + i);
            else free_[i] = {off + n, free_[i].second - n};
            return off;
        }
    }
    const int64_t off = top;
    top += n;
    return off;
}

void Workspace::release(int64_t off, int64_t n) {
    n = round(n);
    free_.push_back({off, n});
    std::sort(free_.begin(), free_.end());
    std::vector<std::pair<int64_t, int64_t>> merged;
    for (auto& f : free_) {
        if (!merged.empty() && merged.back().first + merged.back().second == f.first) merged.back().second += f.second;
        else merged.push_back(f);
    }
    free_ = merged;
}

Plan::~Plan() {
    if (handle) rave_plan_destroy(handle);
    if (ws_dev) (void)hipFree(ws_dev);
}

void Plan::finalize(const void* arena) {
    // the split-K slab is live at different points than any tensor: bump-allocate it past everything
    const int64_t splitk_off = ws.top;
    ws.top += Workspace::round(splitk_max);
    ws_floats = std::max<int64_t>(ws.top, 64);
    RAVE_HIP_OR_THROW(hipMalloc(&ws_dev, (size_t)ws_floats * 4));
    RAVE_HIP_OR_THROW(hipMemset(ws_dev, 0, (size_t)ws_floats * 4));   // split-K counters start zero
    std::vector<rave_plan_op> raw(ops.size());
    std::vector<rave_reloc> relocs;
    for (size_t i = 0; i < ops.size(); ++i) {
        raw[i] = ops[i].op;
        for (auto& fp : ops[i].ptrs) {
            void* val = nullptr;
            const PRef& r = fp.second;
            switch (r.kind) {
                case PRef::NONE: break;
                case PRef::WS: val = (char*)ws_dev + r.off; break;
                case PRef::SPLITK: val = (char*)ws_dev + splitk_off * 4; break;
                case PRef::ARENA: val = (char*)arena + r.off; break;
                case PRef::ABS: val = (void*)(uintptr_t)r.off; break;
                case PRef::IO: {
                    rave_reloc rl{};
                    rl.op = (int)i;
                    rl.field_offset = fp.first;
                    rl.slot = r.slot;
                    rl.byte_offset = r.off;
                    relocs.push_back(rl);
                    break;
                }
            }
            std::memcpy(raw[i].u.raw + fp.first, &val, sizeof(void*));
        }
    }
    check_rc(rave_plan_create(raw.data(), (int)raw.size(), relocs.data(), (int)relocs.size(), &handle),
             "plan_create");
}

void Plan::run(void* const* slots, int n_slots, hipStream_t st) {
    check_rc(rave_plan_run(handle, slots, n_slots, st), "plan_run");
}

// =================================================================== model
struct Model {
    rave_model_config cfg{};
    Graph g;
    std::vector<int> precs;
    bool autotune = false;
    int hop = 1, dec_in = 0, dec_out = 0, noise_target = 0;
    // weight arena (floats)
    std::vector<float> host;
    float* arena = nullptr;
    std::map<std::pair<std::string, int>, int64_t> w_pack, w_pack_stream, unit_pack;
    std::map<std::string, int64_t> bias_off, alpha_off;
    std::set<std::string> unit_ok;     // k=3 names of units with a fused pack in some arithmetic
    int64_t hkf_off = 0, hki_off = 0, spk_off = 0, cb_off = -1;
    int64_t head_filt_off = -1, tail_filt_off = -1;   // rave_*_pack_filter images (-1: shape unsupported)
    int64_t head_filt32_off = -1, tail_filt32_off = -1;   // exact-fp32 images (*_pack_filter_f32)
    // the edges' arithmetic: split16 where the model has it, else the exact-fp32 ring (-1: none)
    int edge_prec() const {
        if (std::find(precs.begin(), precs.end(), RAVE_PREC_SPLIT16) != precs.end()) return RAVE_PREC_SPLIT16;
        if (std::find(precs.begin(), precs.end(), RAVE_PREC_F32_RING) != precs.end()) return RAVE_PREC_F32_RING;
        return -1;
    }
    int taps_a = 0, taps_s = 0;
    // AdaIN buffers (rave/blocks.py:858-868), device
    int max_batch = 64;
    float* ad_stats = nullptr;
    float* ad_init = nullptr;          // the reset image of ad_stats (mean 0, std 1)
    float* ad_counters = nullptr;
    uint32_t* ad_tickets = nullptr;
    std::vector<int64_t> ad_off;
    std::map<std::string, int> ad_index;
    bool learn_x = false, learn_y = false, touched = false;
    int row0 = 0;
    int spk_version = 0;               // bumped by rave_model_set_speaker (stream graphs refill)
    // autotuner choices: key -> (choice, ms)
    std::map<std::string, std::pair<int64_t, double>> tuned;
    std::map<std::string, std::unique_ptr<Plan>> plans;
    // forward's latent, decode's drawn noise, timing scratch
    float* fwd_z = nullptr;
    int64_t fwd_z_n = 0;
    float* noise = nullptr;
    int64_t noise_n = 0;
    uint64_t noise_calls = 0;
    float* scratch = nullptr;
    int64_t scratch_n = 0;
    hipStream_t cur_stream = nullptr;    // stream of the call that builds plans (timing runs)
    // cooperative units' give-up words: host-mapped, one per cooperative op of any
    // plan (rave_unit_args.status), read without synchronisation by coop_check
    static constexpr int kCoopSlots = 256;
    uint32_t* coop_host = nullptr;
    uint32_t* coop_dev = nullptr;
    std::vector<std::string> coop_labels;
    View coop_status(const std::string& label);
    void coop_check();

    ~Model();
    int64_t add(const float* p, int64_t n) {
        const int64_t off = (int64_t)host.size();
        host.insert(host.end(), p, p + n);
        host.resize((host.size() + 63) / 64 * 64, 0.f);
        return off;
    }
    int64_t add(const std::vector<float>& v) { return add(v.data(), (int64_t)v.size()); }
    const float* aptr(int64_t off) const { return arena + off; }
    View arena_view(int64_t off) const {
        View v;
        v.p.kind = PRef::ARENA;
        v.p.off = off * 4;
        return v;
    }
    bool adain_active() const { return touched || learn_x || learn_y; }
    int adain_mode() const { return learn_y ? 2 : (learn_x ? 1 : 0); }
    std::string adain_key() const {
        if (ad_index.empty()) return "";
        return "|ad" + std::to_string(adain_active()) + std::to_string(adain_mode()) + "r" + std::to_string(row0);
    }
    float* scratch_buf(int64_t n);

    // planning
    std::pair<int, int> conv_launch(const Node& n, const rave_conv1d_args& scalars, bool stream_form, bool timed,
                                    bool allow_ring = true);
    rave_conv1d_args conv_desc(const Node& n, int B, int t_in, const View& src, const View& dst, const View* res,
                               int& t_out) const;
    void conv_op(Plan& p, const Node& n, int B, int t_in, const View& src, const View& dst, const View* res);
    double unit_time(const Node& k3, const Node& k1, int B, int T);
    int unit_pick(const Node& k3, int B, int T, bool timed);
    int unit_coop(const Node& k3, int B, int T);
    bool fuse_unit(const Node& k3, const Node& k1, int B, int T);
    double unit_best_ms(const Node& k3, const Node& k1, int B, int T);
    rave_unit_args unit_desc(const Node& k3, const Node& k1, int B, int T, int prec) const;
    void unit_op(Plan& p, const Node& k3, const Node& k1, int B, int T, const View& src, const View& dst,
                 int x_len = 0, int res_shift = 0);
    rave_stack_args stack_desc(const std::vector<std::pair<const Node*, const Node*>>& run, int B, int T) const;
    int stack_prec() const;
    bool use_stack(const std::vector<std::pair<const Node*, const Node*>>& run, int B, int T);
    void stack_op(Plan& p, const std::vector<std::pair<const Node*, const Node*>>& run, int B, int T,
                  const View& src, const View& dst);
    void adain_op(Plan& p, const std::string& name, int B, int C, int T, const View& x);
    std::vector<std::pair<const Node*, const Node*>> unit_pairs(const std::vector<const Node*>& nodes) const;
    std::map<std::string, std::vector<std::pair<const Node*, const Node*>>> stack_runs(
        const std::vector<const Node*>& nodes) const;
    std::map<std::string, std::pair<View, int>> run_stack(Plan& p, const std::vector<const Node*>& nodes, int B,
                                                          const std::map<std::string, std::pair<View, int>>& inputs,
                                                          const std::map<std::string, View>& outputs,
                                                          const std::map<std::string, int64_t>& owned = {});
    void analysis_op(Plan& p, int B, int T, const View& x, const View& y, int n_out, int pad, int t_in);
    void synthesis_op(Plan& p, int B, int F, const View& x, const View& y, const View* noise, int pad, int frame0,
                      int x_len);
    void fill_speaker(Plan& p, int B, int Fz, const View& z);
    // PQMF + edge-conv fusions (csrc/edge_split.hip), split-f16 only
    rave_edge_args head_desc(int B, int F) const;
    bool use_head(int B, int T);
    int head_pick(int B, int T);
    bool head_ok(int ep, int B, int T);
    void head_op(Plan& p, int B, int T, const View& x, const View& y, const View* fill_z);
    rave_edge_args tail_desc(int B, int F) const;
    bool use_tail(int B, int F);
    int tail_pick(int B, int F);
    bool tail_ok(int ep, int B, int F);
    void tail_op(Plan& p, int B, int F, const View& x, const View& y, const View* noise);
    void rvq_encode_op(Plan& p, int B, int Fz, const View& lat, const View& idx);
    void rvq_decode_op(Plan& p, int B, int Fz, const View& idx, const View& z);
    Plan& encode_plan(int B, int T, bool codes);
    Plan& decode_plan(int B, int Fz, bool codes);
    Plan& plan_of(int which, int B, int T);
    void run_kind(int which, int batch, int t, const void* in, void* out, const float* noise, hipStream_t st);
    const float* noise_ptr(const float* u, int B, int Fz, hipStream_t st);
    template <typename F>
    double time_native(F&& fn, int reps = 5);
    int pqmf_prec(const std::string& key, const std::function<int(int, hipStream_t)>& run);
};

Model::~Model() {
    plans.clear();
    if (coop_host) (void)hipHostFree(coop_host);
    for (void* p : {(void*)arena, (void*)ad_stats, (void*)ad_init, (void*)ad_counters, (void*)ad_tickets, (void*)fwd_z, (void*)noise,
                    (void*)scratch})
        if (p) (void)hipFree(p);
}

float* Model::scratch_buf(int64_t n) {
    if (n > scratch_n) {
        if (scratch) RAVE_HIP_OR_THROW(hipFree(scratch));
        scratch = nullptr;
        RAVE_HIP_OR_THROW(hipMalloc(&scratch, (size_t)n * 4));
        scratch_n = n;
        check_rc(rave_fill_uniform(scratch, n, 0x5eed, -1.f, 1.f, cur_stream), "fill_uniform");
    }
    return scratch;
}

template <typename F>
double Model::time_native(F&& fn, int reps) {
    hipStream_t st = cur_stream;
    for (int i = 0; i < 2; ++i) {
        const int rc = fn(st);
        if (rc != RAVE_OK) return -1.0 - (double)(-rc);   // caller decides
    }
    hipEvent_t e0, e1;
    RAVE_HIP_OR_THROW(hipEventCreate(&e0));
    RAVE_HIP_OR_THROW(hipEventCreate(&e1));
    RAVE_HIP_OR_THROW(hipEventRecord(e0, st));
    for (int i = 0; i < reps; ++i) fn(st);
    RAVE_HIP_OR_THROW(hipEventRecord(e1, st));
    RAVE_HIP_OR_THROW(hipEventSynchronize(e1));
    float ms = 0.f;
    RAVE_HIP_OR_THROW(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return ms / reps;
}

// ------------------------------------------------------------------ conv
rave_conv1d_args Model::conv_desc(const Node& n, int B, int t_in, const View& src, const View& dst, const View* res,
                                  int& t_out) const {
    rave_conv1d_args a{};
    t_out = n.out_len(t_in);
    a.c_in = n.c_in;
    a.c_out = n.c_out;
    a.kernel = n.kernel;
    a.stride = n.stride;
    a.dilation = n.dilation;
    a.act = n.act;
    a.leaky_slope = cfg.leaky_slope;
    a.batch = B;
    a.t_in = t_in;
    a.t_out = t_out;
    a.x_sb = src.sb;
    a.x_sc = src.sc;
    a.y_sb = dst.sb;
    a.y_sc = dst.sc;
    a.r_sb = res ? res->sb : 0;
    a.r_sc = res ? res->sc : 0;
    if (n.transposed) {
        a.pad_left = 0;
        a.pad_right = 0;
        a.transposed = 1;
        a.out_shift = n.stride / 2;
    } else {
        a.pad_left = n.pad_l;
        a.pad_right = n.pad_r;
    }
    return a;
}

template <typename Parts>
static std::string key_join(const Parts& parts) {
    std::string k;
    for (auto& p : parts) {
        if (!k.empty()) k += '|';
        k += p;
    }
    return k;
}
static std::string key_of(std::initializer_list<std::string> parts) { return key_join(parts); }
static std::string key_of(const std::vector<std::string>& parts) { return key_join(parts); }

// (precision, launch config) of one conv op; with autotune every arithmetic and
// every configuration rave_conv1d_configs lists is timed on scratch tensors of
// the op's shape and the fastest kept (its time is recorded for fusion choices).
// allow_ring = false: the op's input rows are not 16-byte pieces (a stream
// plan's history buffers), which the fp32 ring kernels need
std::pair<int, int> Model::conv_launch(const Node& n, const rave_conv1d_args& s, bool stream_form, bool timed,
                                       bool allow_ring) {
    auto& pack = stream_form ? w_pack_stream : w_pack;
    // (a choice made without the ring / bf16x3 kernels has a key of its own, so a
    // one-shot plan's ring choice is never replayed on unaligned stream rows and a
    // stream plan's restricted choice never limits a one-shot plan)
    std::vector<std::string> kp = {"conv", n.name, std::to_string(stream_form), std::to_string(s.batch),
                                   std::to_string(s.t_in)};
    if (!allow_ring) kp.push_back("noring");
    const std::string key = key_of(kp);
    if (!tuned.count(key) && (precs.size() > 1 || timed || autotune)) {
        const int B = s.batch;
        const int64_t nx = (int64_t)B * n.c_in * s.t_in, ny = (int64_t)B * n.c_out * s.t_out;
        rave_conv1d_args base = s;
        base.x_sb = (int64_t)n.c_in * s.t_in;
        base.x_sc = s.t_in;
        base.y_sb = base.r_sb = (int64_t)n.c_out * s.t_out;
        base.y_sc = base.r_sc = s.t_out;
        const bool has_res = !n.residual.empty();
        float* sc = scratch_buf(nx + 2 * ny + 256);
        base.x = sc;
        base.y = sc + nx + 64;
        base.residual = has_res ? sc + nx + ny + 128 : nullptr;
        base.bias = n.bias ? aptr(bias_off.at(n.name)) : nullptr;
        base.alpha = n.act == RAVE_ACT_SNAKE ? aptr(alpha_off.at(n.alpha)) : nullptr;
        base.partial = nullptr;
        std::vector<std::pair<int, int>> cands;
        for (int pr : precs) {
            if (!allow_ring && (pr == RAVE_PREC_F32_RING || pr == RAVE_PREC_BF16X3)) continue;
            if (!pack.count({n.name, pr})) continue;     // (an arithmetic of the fused units only)
            base.precision = pr;
            base.weight = aptr(pack.at({n.name, pr}));
            cands.push_back({pr, 0});
            if (autotune || precs.size() > 1) {
                int32_t buf[1024];
                const int cnt = rave_conv1d_configs(&base, buf, 1024);
                check_rc(cnt < 0 ? cnt : RAVE_OK, "conv1d_configs " + n.name);
                for (int i = 0; i < std::min(cnt, 1024); ++i) cands.push_back({pr, buf[i]});
            }
        }
        int64_t nws = 0;
        for (auto& c : cands) {
            base.precision = c.first;
            base.config = c.second;
            base.weight = aptr(pack.at({n.name, c.first}));
            nws = std::max(nws, rave_conv1d_workspace(&base));
        }
        float* ws = nullptr;
        if (nws > 0) {
            RAVE_HIP_OR_THROW(hipMalloc(&ws, (size_t)nws * 4));
            RAVE_HIP_OR_THROW(hipMemsetAsync(ws, 0, (size_t)nws * 4, cur_stream));
        }
        double best_ms = 1e30;
        std::pair<int, int> best{-1, -1};
        std::set<int> bad;                           // arithmetics whose default launch failed
        std::string why;
        for (auto& c : cands) {
            if (bad.count(c.first)) continue;
            rave_conv1d_args a = base;
            a.precision = c.first;
            a.config = c.second;
            a.weight = aptr(pack.at({n.name, c.first}));
            a.partial = ws;
            const double ms = time_native([&](hipStream_t st) { return rave_conv1d(&a, st); });
            if (ms < 0) {
                // a failing default launch rules its arithmetic out for this shape
                // (e.g. the fp32 ring kernels on rows that are not 16-byte pieces)
                if (c.second == 0) {
                    bad.insert(c.first);
                    why = rave_last_error();
                }
                continue;
            }
            if (ms < best_ms) {
                best_ms = ms;
                best = c;
            }
        }
        if (ws) RAVE_HIP_OR_THROW(hipFree(ws));
        if (best.first < 0) fail(RAVE_ERR_STATE, "conv " + n.name + ": default configuration failed: " + why);
        tuned[key] = {(int64_t)best.first * 65536 + best.second, best_ms};
    }
    auto it = tuned.find(key);
    if (it != tuned.end()) return {(int)(it->second.first / 65536), (int)(it->second.first % 65536)};
    return {precs[0], 0};
}

void Model::conv_op(Plan& p, const Node& n, int B, int t_in, const View& src, const View& dst, const View* res) {
    int t_out;
    rave_conv1d_args a = conv_desc(n, B, t_in, src, dst, res, t_out);
    const auto pc = conv_launch(n, a, false, false);
    a.precision = pc.first;
    a.config = pc.second;
    // split-K slab the launcher wants (shapes only)
    rave_conv1d_args q = a;
    q.x = q.weight = q.alpha = (const float*)arena;
    q.y = (float*)arena;
    q.residual = res ? (const float*)arena : nullptr;
    q.weight = aptr(w_pack.at({n.name, pc.first}));
    const int64_t nsk = rave_conv1d_workspace(&q);
    if (nsk < 0) fail(RAVE_ERR_ARG, "conv " + n.name + ": workspace query failed: " + rave_last_error());
    PlanOp& o = p.add(RAVE_OP_CONV, a, n.name);
    View wv = arena_view(w_pack.at({n.name, pc.first}));
    View bv = n.bias ? arena_view(bias_off.at(n.name)) : View{};
    View av = n.act == RAVE_ACT_SNAKE ? arena_view(alpha_off.at(n.alpha)) : View{};
    View sk = p.splitk(nsk);
    rave_conv1d_args& A = *reinterpret_cast<rave_conv1d_args*>(o.op.u.raw);
    p.bind(o, A, A.x, &src);
    p.bind(o, A, A.y, &dst);
    p.bind(o, A, A.residual, res);
    p.bind(o, A, A.weight, &wv);
    p.bind(o, A, A.bias, n.bias ? &bv : nullptr);
    p.bind(o, A, A.alpha, n.act == RAVE_ACT_SNAKE ? &av : nullptr);
    p.bind(o, A, A.partial, nsk > 0 ? &sk : nullptr);
    o.prec = pc.first;
    const double taps = n.transposed ? 2.0 : (double)n.kernel;
    o.flops = 2.0 * B * n.c_out * t_out * n.c_in * taps;
    o.bytes = 4.0 * ((double)B * n.c_in * t_in + (double)B * n.c_out * t_out * (res ? 2 : 1) +
                     (double)n.c_in * n.c_out * n.kernel);
}

// ------------------------------------------------------------------ fused units
std::vector<std::pair<const Node*, const Node*>> Model::unit_pairs(const std::vector<const Node*>& nodes) const {
    std::vector<std::pair<const Node*, const Node*>> out;
    for (size_t i = 0; i + 1 < nodes.size(); ++i) {
        const Node& a = *nodes[i];
        const Node& b = *nodes[i + 1];
        if (a.kernel == 3 && a.stride == 1 && !a.transposed && b.kernel == 1 && b.src == a.dst &&
            b.residual == a.src && a.c_in == a.c_out && a.c_out == b.c_out && a.act == b.act && a.bias == b.bias)
            out.push_back({&a, &b});
    }
    return out;
}

rave_unit_args Model::unit_desc(const Node& k3, const Node& k1, int B, int T, int prec) const {
    rave_unit_args u{};
    u.channels = k3.c_in;
    u.batch = B;
    u.t_len = T;
    u.dilation = k3.dilation;
    u.pad_left = k3.pad_l;
    u.act = k3.act;
    u.leaky_slope = cfg.leaky_slope;
    u.precision = prec;
    u.weight = aptr(unit_pack.at({k3.name, prec}));
    u.bias1 = k3.bias ? aptr(bias_off.at(k3.name)) : nullptr;
    u.bias2 = k1.bias ? aptr(bias_off.at(k1.name)) : nullptr;
    u.alpha0 = k3.act == RAVE_ACT_SNAKE ? aptr(alpha_off.at(k3.alpha)) : nullptr;
    u.alpha2 = k1.act == RAVE_ACT_SNAKE ? aptr(alpha_off.at(k1.alpha)) : nullptr;
    return u;
}

double Model::unit_time(const Node& k3, const Node& k1, int B, int T) {
    unit_pick(k3, B, T, true);
    return tuned.at(key_of({"unit", k3.name, std::to_string(B), std::to_string(T)})).second;
}

// the faster arithmetic of the fused unit kernel for this shape (timed when
// there is a choice or its time is wanted)
int Model::unit_pick(const Node& k3, int B, int T, bool timed) {
    std::vector<int> cands;
    for (int pr : precs)
        if (unit_pack.count({k3.name, pr})) cands.push_back(pr);
    if (cands.empty()) fail(RAVE_ERR_STATE, "unit " + k3.name + ": no fused pack");
    if (cands.size() == 1 && !timed) {
        rave_unit_args q{};
        q.channels = k3.c_in;
        q.batch = B;
        q.t_len = T;
        q.precision = cands[0];
        if (rave_unit_workspace(&q) <= 0) return cands[0];   // one form: nothing to time
    }
    const std::string key = key_of({"unit", k3.name, std::to_string(B), std::to_string(T)});
    if (!tuned.count(key)) {
        const Node* k1 = nullptr;
        for (const Node* n : g.convs())
            if (n->src == k3.dst && n->kernel == 1) k1 = n;
        const int64_t n_el = (int64_t)B * k3.c_in * T;
        int64_t nws = 0;
        for (int pr : cands) {
            rave_unit_args q = unit_desc(k3, *k1, B, T, pr);
            nws = std::max(nws, rave_unit_workspace(&q));
            q.coop_rb = 4;                                // the wide group at C = 256
            nws = std::max(nws, rave_unit_workspace(&q));
        }
        float* sc = scratch_buf(2 * n_el + 128 + nws);
        float* ws = nws > 0 ? sc + 2 * n_el + 128 : nullptr;   // (64-float aligned)
        if (ws) RAVE_HIP_OR_THROW(hipMemset(ws, 0, (size_t)RAVE_SPLITK_TICKETS * 4));   // counters at rest
        double best = 1e30;
        int bp = cands[0];
        for (int pr : cands) {
            rave_unit_args u = unit_desc(k3, *k1, B, T, pr);
            u.x = sc;
            u.y = sc + n_el + 64;
            u.x_sb = u.y_sb = (int64_t)k3.c_in * T;
            u.x_sc = u.y_sc = T;
            // both forms where the cooperative one exists (one workgroup per slab /
            // groups of workgroups sharing a slab), and at C = 256 the wide group
            // (coop 2: groups of 4, round 6): value = precision | coop << 8
            const int ncoop = rave_unit_workspace(&u) > 0 ? (k3.c_in == 256 ? 2 : 1) : 0;
            for (int coop = 0; coop <= ncoop; ++coop) {
                u.coop_rb = coop == 2 ? 4 : 0;
                u.workspace = coop ? ws : nullptr;
                const double ms = time_native([&](hipStream_t st) { return rave_residual_unit(&u, st); });
                if (ms >= 0 && ms < best) {
                    best = ms;
                    bp = pr | (coop << 8);
                }
            }
        }
        tuned[key] = {bp, best};
    }
    return (int)tuned.at(key).first & 255;
}

// the cooperative form the tuning chose: 0 none, 1 groups of C / 128, 2 the wide group
int Model::unit_coop(const Node& k3, int B, int T) {
    const std::string key = key_of({"unit", k3.name, std::to_string(B), std::to_string(T)});
    auto it = tuned.find(key);
    return it != tuned.end() ? ((int)it->second.first >> 8) : 0;
}

// Residual(DilatedUnit) as the fused kernel (true) or as its two convs (false):
// with several arithmetics the faster by measurement.
bool Model::fuse_unit(const Node& k3, const Node& k1, int B, int T) {
    if (precs.size() == 1) return true;
    const std::string key = key_of({"fuse", k3.name, std::to_string(B), std::to_string(T)});
    if (!tuned.count(key)) {
        const double fused = unit_time(k3, k1, B, T);
        View src = ws_view(0, (int64_t)k3.c_in * T, T), tmp = ws_view(0, (int64_t)k3.c_out * T, T);
        int t3, t1;
        rave_conv1d_args s3 = conv_desc(k3, B, T, src, tmp, nullptr, t3);
        conv_launch(k3, s3, false, true);
        rave_conv1d_args s1 = conv_desc(k1, B, T, tmp, tmp, &src, t1);
        conv_launch(k1, s1, false, true);
        const double split =
            tuned.at(key_of({"conv", k3.name, "0", std::to_string(B), std::to_string(T)})).second +
            tuned.at(key_of({"conv", k1.name, "0", std::to_string(B), std::to_string(T)})).second;
        tuned[key] = {fused <= split ? 1 : 0, std::min(fused, split)};
    }
    return tuned.at(key).first != 0;
}

double Model::unit_best_ms(const Node& k3, const Node& k1, int B, int T) {
    if (precs.size() > 1) {
        fuse_unit(k3, k1, B, T);
        return tuned.at(key_of({"fuse", k3.name, std::to_string(B), std::to_string(T)})).second;
    }
    return unit_time(k3, k1, B, T);
}

void Model::unit_op(Plan& p, const Node& k3, const Node& k1, int B, int T, const View& src, const View& dst,
                    int x_len, int res_shift) {
    const int pr = unit_pick(k3, B, T, false);
    rave_unit_args u = unit_desc(k3, k1, B, T, pr);
    if (x_len > 0) {
        // cached form: x from the history start, no zero padding, residual shifted
        u.pad_left = 0;
        u.x_len = x_len;
        u.res_shift = res_shift;
    }
    u.x_sb = src.sb;
    u.x_sc = src.sc;
    u.y_sb = dst.sb;
    u.y_sc = dst.sc;
    const std::string label = k3.name.substr(0, k3.name.rfind(".net.")) + ".unit";
    // cooperative form (when timed faster): the plan's split-K buffer
    const int coop = unit_coop(k3, B, T);
    u.coop_rb = coop == 2 ? 4 : 0;
    const int64_t nws = coop ? rave_unit_workspace(&u) : 0;
    if (nws < 0) fail(RAVE_ERR_ARG, "unit " + k3.name + ": workspace query failed: " + rave_last_error());
    PlanOp& o = p.add(RAVE_OP_UNIT, u, label);
    rave_unit_args& U = *reinterpret_cast<rave_unit_args*>(o.op.u.raw);
    View wv = arena_view(unit_pack.at({k3.name, pr}));
    View b1 = k3.bias ? arena_view(bias_off.at(k3.name)) : View{};
    View b2 = k1.bias ? arena_view(bias_off.at(k1.name)) : View{};
    View a0 = k3.act == RAVE_ACT_SNAKE ? arena_view(alpha_off.at(k3.alpha)) : View{};
    View a2 = k1.act == RAVE_ACT_SNAKE ? arena_view(alpha_off.at(k1.alpha)) : View{};
    p.bind(o, U, U.x, &src);
    p.bind(o, U, U.y, &dst);
    p.bind(o, U, U.weight, &wv);
    p.bind(o, U, U.bias1, k3.bias ? &b1 : nullptr);
    p.bind(o, U, U.bias2, k1.bias ? &b2 : nullptr);
    p.bind(o, U, U.alpha0, k3.act == RAVE_ACT_SNAKE ? &a0 : nullptr);
    p.bind(o, U, U.alpha2, k1.act == RAVE_ACT_SNAKE ? &a2 : nullptr);
    View sk = p.splitk(nws);
    p.bind(o, U, U.workspace, nws > 0 ? &sk : nullptr);
    View sv = nws > 0 ? coop_status(label + " (B=" + std::to_string(B) + ", T=" + std::to_string(T) + ")") : View{};
    p.bind(o, U, U.status, nws > 0 ? &sv : nullptr);
    o.prec = pr;
    const double C_ = k3.c_in;
    o.flops = 2.0 * B * T * C_ * C_ * 4;
    o.bytes = 4.0 * (2.0 * B * C_ * T + 4.0 * C_ * C_);
}

// A status word for one cooperative unit op (the last slot is shared once
// kCoopSlots ops exist).
View Model::coop_status(const std::string& label) {
    if (!coop_host) {
        void* h = nullptr;
        RAVE_HIP_OR_THROW(hipHostMalloc(&h, kCoopSlots * 4, hipHostMallocMapped | hipHostMallocCoherent));
        std::memset(h, 0, kCoopSlots * 4);
        void* d = nullptr;
        RAVE_HIP_OR_THROW(hipHostGetDevicePointer(&d, h, 0));
        coop_host = static_cast<uint32_t*>(h);
        coop_dev = static_cast<uint32_t*>(d);
    }
    const int slot = std::min<int>((int)coop_labels.size(), kCoopSlots - 1);
    if (slot < kCoopSlots - 1) coop_labels.push_back(label);
    else if (coop_labels.size() == kCoopSlots - 1) coop_labels.push_back(label + " (or a later cooperative unit)");
    return abs_view(coop_dev + slot);
}

// Report (and clear) give-ups of cooperative units that have already run.
void Model::coop_check() {
    if (!coop_host) return;
    std::string which;
    for (size_t i = 0; i < coop_labels.size(); ++i) {
        volatile uint32_t* w = coop_host + i;
        if (*w == 0) continue;
        *w = 0;
        which += (which.empty() ? "" : ", ") + coop_labels[i];
    }
    if (!which.empty())
        fail(RAVE_ERR_COOP, "cooperative residual unit hand-off gave up (outputs of that call are NaN): " + which);
}

// ------------------------------------------------------------------ residual stacks
std::map<std::string, std::vector<std::pair<const Node*, const Node*>>> Model::stack_runs(
    const std::vector<const Node*>& nodes) const {
    std::map<std::string, std::vector<std::pair<const Node*, const Node*>>> out;
    const auto pairs = unit_pairs(nodes);
    const bool ad_on = !ad_index.empty() && adain_active();
    size_t i = 0;
    const size_t U = RAVE_STACK_UNITS;
    while (i + U <= pairs.size()) {
        std::vector<std::pair<const Node*, const Node*>> run(pairs.begin() + i, pairs.begin() + i + U);
        const Node& a0 = *run[0].first;
        bool ok = rave_stack_supported(a0.c_in) != 0;
        for (size_t k = 0; k + 1 < U && ok; ++k) ok = run[k + 1].first->src == run[k].second->dst;
        int dil[RAVE_STACK_UNITS], padl[RAVE_STACK_UNITS];
        for (size_t k = 0; k < U; ++k) {
            const Node& k3 = *run[k].first;
            ok = ok && k3.c_in == a0.c_in && k3.act == a0.act && k3.bias == a0.bias &&
                 unit_pack.count({k3.name, stack_prec()}) && !(ad_on && !k3.adain.empty());
            dil[k] = k3.dilation;
            padl[k] = k3.pad_l;
        }
        // the shapes the stack kernel takes (its margin, the bf16x3 plane halo):
        // a tuned or pinned stack choice is only ever consulted for these
        ok = ok && stack_shape_fits(stack_prec() == RAVE_PREC_BF16X3, dil, padl, (int)U);
        if (ok) {
            out[a0.name] = run;
            i += U;
        } else {
            ++i;
        }
    }
    return out;
}

// the stack's arithmetic: split16 where the model has it (auto / split16),
// else bf16x3 (f32_bf3); -1: no stack form
int Model::stack_prec() const {
    if (std::find(precs.begin(), precs.end(), (int)RAVE_PREC_SPLIT16) != precs.end()) return RAVE_PREC_SPLIT16;
    if (std::find(precs.begin(), precs.end(), (int)RAVE_PREC_BF16X3) != precs.end()) return RAVE_PREC_BF16X3;
    return -1;
}

rave_stack_args Model::stack_desc(const std::vector<std::pair<const Node*, const Node*>>& run, int B, int T) const {
    rave_stack_args s{};
    const Node& a0 = *run[0].first;
    const int sp = stack_prec();
    s.precision = sp;
    s.channels = a0.c_in;
    s.batch = B;
    s.t_len = T;
    s.act = a0.act;
    s.leaky_slope = cfg.leaky_slope;
    for (size_t u = 0; u < run.size(); ++u) {
        const Node& k3 = *run[u].first;
        const Node& k1 = *run[u].second;
        s.dilation[u] = k3.dilation;
        s.pad_left[u] = k3.pad_l;
        s.weight[u] = aptr(unit_pack.at({k3.name, sp}));
        s.bias1[u] = k3.bias ? aptr(bias_off.at(k3.name)) : nullptr;
        s.bias2[u] = k1.bias ? aptr(bias_off.at(k1.name)) : nullptr;
        s.alpha0[u] = k3.act == RAVE_ACT_SNAKE ? aptr(alpha_off.at(k3.alpha)) : nullptr;
        s.alpha2[u] = k1.act == RAVE_ACT_SNAKE ? aptr(alpha_off.at(k1.alpha)) : nullptr;
    }
    return s;
}

// one rave_residual_stack launch instead of the units: always in split16-only
// mode, else when it measures faster than the units' best (auto: split16
// stacks; f32_bf3: bf16x3 stacks)
bool Model::use_stack(const std::vector<std::pair<const Node*, const Node*>>& run, int B, int T) {
    if (stack_prec() < 0) return false;
    if (precs.size() == 1 && !autotune) return true;
    const std::string key = key_of({"stack", run[0].first->name, std::to_string(B), std::to_string(T)});
    if (!tuned.count(key)) {
        rave_stack_args s = stack_desc(run, B, T);
        const int64_t n_el = (int64_t)B * s.channels * T;
        float* sc = scratch_buf(2 * n_el + 128);
        s.x = sc;
        s.y = sc + n_el + 64;
        s.x_sb = s.y_sb = (int64_t)s.channels * T;
        s.x_sc = s.y_sc = T;
        const double st_ms = time_native([&](hipStream_t st) { return rave_residual_stack(&s, st); });
        if (st_ms < 0) {
            tuned[key] = {0, 0.0};
            return false;
        }
        double units = 0;
        for (auto& pr : run) units += unit_best_ms(*pr.first, *pr.second, B, T);
        tuned[key] = {st_ms <= units ? 1 : 0, std::min(st_ms, units)};
    }
    return tuned.at(key).first != 0;
}

void Model::stack_op(Plan& p, const std::vector<std::pair<const Node*, const Node*>>& run, int B, int T,
                     const View& src, const View& dst) {
    rave_stack_args s = stack_desc(run, B, T);
    s.x_sb = src.sb;
    s.x_sc = src.sc;
    s.y_sb = dst.sb;
    s.y_sc = dst.sc;
    const std::string& n0 = run[0].first->name;
    const size_t cut = n0.find(".net.");
    PlanOp& o = p.add(RAVE_OP_STACK, s, n0.substr(0, cut) + ".stack");
    rave_stack_args& S = *reinterpret_cast<rave_stack_args*>(o.op.u.raw);
    p.bind(o, S, S.x, &src);
    p.bind(o, S, S.y, &dst);
    for (size_t u = 0; u < run.size(); ++u) {
        const Node& k3 = *run[u].first;
        const Node& k1 = *run[u].second;
        View wv = arena_view(unit_pack.at({k3.name, s.precision}));
        View b1 = k3.bias ? arena_view(bias_off.at(k3.name)) : View{};
        View b2 = k1.bias ? arena_view(bias_off.at(k1.name)) : View{};
        View a0 = k3.act == RAVE_ACT_SNAKE ? arena_view(alpha_off.at(k3.alpha)) : View{};
        View a2 = k1.act == RAVE_ACT_SNAKE ? arena_view(alpha_off.at(k1.alpha)) : View{};
        p.bind(o, S, S.weight[u], &wv);
        p.bind(o, S, S.bias1[u], k3.bias ? &b1 : nullptr);
        p.bind(o, S, S.bias2[u], k1.bias ? &b2 : nullptr);
        p.bind(o, S, S.alpha0[u], k3.act == RAVE_ACT_SNAKE ? &a0 : nullptr);
        p.bind(o, S, S.alpha2[u], k1.act == RAVE_ACT_SNAKE ? &a2 : nullptr);
    }
    o.prec = s.precision;
    const double C_ = s.channels;
    o.flops = 2.0 * B * T * C_ * C_ * 4 * run.size();
    o.bytes = 4.0 * (2.0 * B * C_ * T + 4.0 * C_ * C_ * run.size());
}

// AdaIN in place on the residual unit's input (both its conv input and its
// residual; no other reader)
void Model::adain_op(Plan& p, const std::string& name, int B, int C, int T, const View& x) {
    if (row0 + B > max_batch)
        fail(RAVE_ERR_ARG, "AdaIN statistics hold " + std::to_string(max_batch) + " batch rows (cc.MAX_BATCH_SIZE); batch " +
                               std::to_string(B) + " at row " + std::to_string(row0) + " exceeds them");
    const int i = ad_index.at(name);
    rave_adain_args a{};
    a.batch = B;
    a.channels = C;
    a.t_len = T;
    a.mode = adain_mode();
    a.max_batch = max_batch;
    a.row0 = row0;
    a.x_sb = a.y_sb = x.sb;
    a.x_sc = a.y_sc = x.sc;
    PlanOp& o = p.add(RAVE_OP_ADAIN, a, "adain:" + name);
    rave_adain_args& A = *reinterpret_cast<rave_adain_args*>(o.op.u.raw);
    View st = abs_view(ad_stats + ad_off[i]), cn = abs_view(ad_counters + 2 * i), tk = abs_view(ad_tickets + i);
    p.bind(o, A, A.x, &x);
    p.bind(o, A, A.y, &x);
    p.bind(o, A, A.stats, &st);
    p.bind(o, A, A.counters, &cn);
    p.bind(o, A, A.ticket, &tk);
}

// Lay a conv sequence into the plan, allocating workspace tensors with
// liveness-based reuse.  inputs: tensor -> (view, T); outputs: fixed views.
// owned: inputs that live in the plan's workspace (floats), released after their last use
std::map<std::string, std::pair<View, int>> Model::run_stack(Plan& p, const std::vector<const Node*>& nodes, int B,
                                                             const std::map<std::string, std::pair<View, int>>& inputs,
                                                             const std::map<std::string, View>& outputs,
                                                             const std::map<std::string, int64_t>& owned) {
    std::map<std::string, int> last_use;
    for (size_t i = 0; i < nodes.size(); ++i) {
        last_use[nodes[i]->src] = (int)i;
        if (!nodes[i]->residual.empty()) last_use[nodes[i]->residual] = (int)i;
    }
    struct T_ {
        View v;
        int t;
        int64_t size;   // floats owned in the workspace (-1: not owned)
    };
    std::map<std::string, T_> ts;
    for (auto& kv : inputs) {
        auto ow = owned.find(kv.first);
        ts[kv.first] = {kv.second.first, kv.second.second, ow != owned.end() ? ow->second : -1};
    }
    std::map<std::string, const Node*> fused;
    if (cfg.fuse_units)
        for (auto& pr : unit_pairs(nodes))
            if (unit_ok.count(pr.first->name)) fused[pr.first->name] = pr.second;
    auto stacks = (cfg.fuse_units && !unit_ok.empty()) ? stack_runs(nodes)
                                                       : std::map<std::string, std::vector<std::pair<const Node*, const Node*>>>{};
    std::set<std::string> skip;
    auto release = [&](const std::string& name) {
        auto it = ts.find(name);
        if (it == ts.end() || outputs.count(name)) return;
        if (it->second.size > 0 && it->second.v.p.kind == PRef::WS) {
            p.ws.release(it->second.v.p.off / 4, it->second.size);
            it->second.size = -1;
        }
    };
    auto out_view = [&](const std::string& name, int c, int t, int64_t& size) {
        auto it = outputs.find(name);
        if (it != outputs.end()) {
            size = -1;
            return it->second;
        }
        size = (int64_t)B * c * t;
        return ws_view(p.ws.alloc(size), (int64_t)c * t, t);
    };
    for (size_t i = 0; i < nodes.size(); ++i) {
        const Node& n = *nodes[i];
        if (skip.count(n.name)) continue;
        const T_ in = ts.at(n.src);
        const int t_in = in.t;
        if (!n.adain.empty() && !ad_index.empty() && adain_active()) adain_op(p, n.adain, B, n.c_in, t_in, in.v);
        auto st = stacks.find(n.name);
        if (st != stacks.end() && use_stack(st->second, B, t_in)) {
            const auto& run = st->second;
            const Node& last = *run.back().second;
            for (auto& pr : run) {
                skip.insert(pr.first->name);
                skip.insert(pr.second->name);
            }
            int64_t size;
            View dst = out_view(last.dst, last.c_out, t_in, size);
            stack_op(p, run, B, t_in, in.v, dst);
            ts[last.dst] = {dst, t_in, size};
            if (last_use.count(n.src) && last_use[n.src] <= (int)(i + 2 * run.size() - 1)) release(n.src);
            continue;
        }
        auto fu = fused.find(n.name);
        if (fu != fused.end() && fuse_unit(n, *fu->second, B, t_in)) {
            const Node& k1 = *fu->second;
            skip.insert(k1.name);
            int64_t size;
            View dst = out_view(k1.dst, k1.c_out, t_in, size);
            unit_op(p, n, k1, B, t_in, in.v, dst);
            ts[k1.dst] = {dst, t_in, size};
            if (last_use.count(n.src) && last_use[n.src] == (int)i + 1) release(n.src);
            continue;
        }
        const int t_out = n.out_len(t_in);
        int64_t size;
        View dst = out_view(n.dst, n.c_out, t_out, size);
        const View* res = n.residual.empty() ? nullptr : &ts.at(n.residual).v;
        conv_op(p, n, B, t_in, in.v, dst, res);
        ts[n.dst] = {dst, t_out, size};
        for (const std::string& name : {n.src, n.residual})
            if (!name.empty() && last_use.count(name) && last_use[name] == (int)i) release(name);
    }
    std::map<std::string, std::pair<View, int>> out;
    for (auto& kv : ts) out[kv.first] = {kv.second.v, kv.second.t};
    return out;
}

// ------------------------------------------------------------------ PQMF / misc ops
// Arithmetic of a PQMF op: exact fp32 in an fp32 model, split-f16 in a split16
// model, and with RAVE_PREC_AUTO the faster of the two, timed on scratch
// operands of the op's own shape (`run(precision, stream)` launches it).
int Model::pqmf_prec(const std::string& key, const std::function<int(int, hipStream_t)>& run) {
    if (precs.size() == 1) return precs[0];
    if (!tuned.count(key)) {
        double best = 1e30;
        int bp = RAVE_PREC_F32;
        for (int pr : precs) {
            const double ms = time_native([&](hipStream_t st) { return run(pr, st); });
            if (ms >= 0 && ms < best) {
                best = ms;
                bp = pr;
            }
        }
        tuned[key] = {bp, best};
    }
    return (int)tuned.at(key).first;
}

void Model::analysis_op(Plan& p, int B, int T, const View& x, const View& y, int n_out, int pad, int t_in) {
    const int F = T / cfg.n_band;
    rave_pqmf_analysis_args a{};
    a.n_band = cfg.n_band;
    a.taps = taps_a;
    a.n_out_bands = n_out;
    a.batch = B;
    a.t_in = t_in;
    a.pad_left = pad;
    a.t_out = F;
    a.x_sb = x.sb;
    a.y_sb = y.sb;
    a.y_sc = y.sc;
    {
        rave_pqmf_analysis_args q = a;            // scratch operands, the op's strides
        const int64_t nx = (int64_t)(B - 1) * x.sb + t_in, ny = (int64_t)(B - 1) * y.sb + (int64_t)n_out * y.sc;
        float* sc = scratch_buf(nx + ny + 128);
        q.x = sc;
        q.y = sc + nx + 64;
        q.hkf = arena + hkf_off;
        a.precision = pqmf_prec(key_of({"pqa", std::to_string(B), std::to_string(T), std::to_string(t_in)}),
                                [&](int pr, hipStream_t st) {
                                    q.precision = pr;
                                    return rave_pqmf_analysis(&q, st);
                                });
    }
    PlanOp& o = p.add(RAVE_OP_PQMF_ANALYSIS, a, "pqmf_analysis");
    o.prec = a.precision;
    rave_pqmf_analysis_args& A = *reinterpret_cast<rave_pqmf_analysis_args*>(o.op.u.raw);
    View h = arena_view(hkf_off);
    p.bind(o, A, A.x, &x);
    p.bind(o, A, A.y, &y);
    p.bind(o, A, A.hkf, &h);
    o.flops = 2.0 * B * n_out * F * taps_a;
    o.bytes = 4.0 * ((double)B * T + (double)B * n_out * F);
}

void Model::synthesis_op(Plan& p, int B, int F, const View& x, const View& y, const View* noise, int pad, int frame0,
                         int x_len) {
    rave_pqmf_synthesis_args a{};
    a.n_band = cfg.n_band;
    a.taps = taps_s;
    a.batch = B;
    a.t_in = F;
    a.pad_left = pad;
    a.mode = cfg.amplitude_modulation ? 1 : 2;
    a.frame0 = frame0;
    a.x_len = x_len;
    a.x_sb = x.sb;
    a.x_sc = x.sc;
    a.n_sb = noise ? noise->sb : 0;
    a.n_sc = noise ? noise->sc : 0;
    a.y_sb = y.sb;
    {
        rave_pqmf_synthesis_args q = a;           // scratch operands (no noise), the op's strides
        const int xl = x_len > 0 ? x_len : F;
        const int64_t nx = (int64_t)(B - 1) * x.sb + (int64_t)(2 * cfg.n_band - 1) * x.sc + xl;
        const int64_t ny = (int64_t)(B - 1) * y.sb + (int64_t)F * cfg.n_band;
        float* sc = scratch_buf(nx + ny + 128);
        q.x = sc;
        q.y = sc + ((nx + 63) / 64 + 1) * 64;     // 16-byte aligned
        q.noise = nullptr;
        q.hki = arena + hki_off;
        a.precision = pqmf_prec(key_of({"pqs", std::to_string(B), std::to_string(F), std::to_string(x_len),
                                        std::to_string(pad)}),
                                [&](int pr, hipStream_t st) {
                                    q.precision = pr;
                                    return rave_pqmf_synthesis(&q, st);
                                });
    }
    PlanOp& o = p.add(RAVE_OP_PQMF_SYNTHESIS, a, "pqmf_synthesis");
    o.prec = a.precision;
    rave_pqmf_synthesis_args& A = *reinterpret_cast<rave_pqmf_synthesis_args*>(o.op.u.raw);
    View h = arena_view(hki_off);
    p.bind(o, A, A.x, &x);
    p.bind(o, A, A.y, &y);
    p.bind(o, A, A.noise, noise);
    p.bind(o, A, A.hki, &h);
    o.flops = 2.0 * B * F * cfg.n_band * cfg.n_band * taps_s;
    o.bytes = 4.0 * (2.0 * B * F * cfg.n_band + (noise ? (double)B * F * cfg.n_band : 0.0));
}

void Model::fill_speaker(Plan& p, int B, int Fz, const View& z) {
    if (cfg.speaker_size == 0) return;
    rave_fill_args a{};
    a.batch = B;
    a.channels = cfg.speaker_size;
    a.t_len = Fz;
    a.y_sb = z.sb;
    a.y_sc = z.sc;
    PlanOp& o = p.add(RAVE_OP_FILL, a, "fill");
    rave_fill_args& A = *reinterpret_cast<rave_fill_args*>(o.op.u.raw);
    View s = arena_view(spk_off);
    p.bind(o, A, A.y, &z);
    p.bind(o, A, A.values, &s);
}

// ------------------------------------------------------------------ path edges
// The PQMF op and the conv next to it as one split-f16 launch: the encoder head
// (analysis -> EncoderV2's first conv, + the speaker fill) and the decoder tail
// (GeneratorV2's last conv + epilogue -> synthesis).  Used where split-f16 is
// one of the model's arithmetics, the shapes are the kernels', and (with
// autotuning) the fused launch beats the two separate ops at their best.
rave_edge_args Model::head_desc(int B, int F) const {
    const Node& n = g.encoder.front();
    rave_edge_args a{};
    a.batch = B;
    a.frames = F;
    a.conv_c_in = n.c_in;
    a.conv_c_out = n.c_out;
    a.conv_kernel = n.kernel;
    a.conv_pad_left = n.pad_l;
    a.pqmf_taps = taps_a;
    a.pqmf_pad_left = get_padding(taps_a, 1, cfg.causal).first;
    a.act = n.act;
    a.leaky_slope = cfg.leaky_slope;
    return a;
}

rave_edge_args Model::tail_desc(int B, int F) const {
    const Node& n = g.decoder.back();
    rave_edge_args a{};
    a.batch = B;
    a.frames = F;
    a.conv_c_in = n.c_in;
    a.conv_c_out = n.c_out;
    a.conv_kernel = n.kernel;
    a.conv_pad_left = n.pad_l;
    a.pqmf_taps = taps_s;
    a.pqmf_pad_left = get_padding(taps_s, 1, cfg.causal).first;
    a.mode = cfg.amplitude_modulation ? 1 : 2;
    a.act = n.act;
    a.leaky_slope = cfg.leaky_slope;
    return a;
}

// RAVE_EDGES=0 in the environment keeps both edges unfused (same-box A/B runs)
static bool edges_enabled() {
    const char* e = std::getenv("RAVE_EDGES");
    return !(e && e[0] == '0');
}

// the fused head's arithmetic for (B, T), or -1 for the two separate ops: the
// model's edge arithmetic, and in f32_bf3 models also the bf16x3 analysis form
// (exact-fp32 conv), whichever is timed faster
int Model::head_pick(int B, int T) {
    std::vector<int> cands = {edge_prec()};
    if (edge_prec() == RAVE_PREC_F32_RING && std::find(precs.begin(), precs.end(), (int)RAVE_PREC_BF16X3) != precs.end())
        cands.push_back(RAVE_PREC_BF16X3);
    int best = -1;
    double bms = 1e30;
    for (int ep : cands) {
        if (!head_ok(ep, B, T)) continue;
        const double ms = tuned.at(key_of({"head", std::to_string(ep), std::to_string(B), std::to_string(T)})).second;
        if (best < 0 || ms < bms) {
            best = ep;
            bms = ms;
        }
    }
    return best;
}

bool Model::use_head(int B, int T) { return head_pick(B, T) >= 0; }

// the head's conv weight image: the ring image for the exact-fp32 and bf16x3 forms
static int head_wprec(int ep) { return ep == RAVE_PREC_BF16X3 ? RAVE_PREC_F32_RING : ep; }

bool Model::head_ok(int ep, int B, int T) {
    const int64_t filt = ep == RAVE_PREC_SPLIT16 ? head_filt_off : head_filt32_off;
    if (!edges_enabled() || ep < 0 || filt < 0) return false;
    const Node& n = g.encoder.front();
    const int F = T / cfg.n_band;
    if (!w_pack.count({n.name, head_wprec(ep)})) return false;
    if (cfg.n_band != 16 || n.kernel != 7 || n.stride != 1 || n.dilation != 1 || n.act != RAVE_ACT_NONE ||
        n.transposed || n.c_in > 8 || n.c_out > 64 || !n.adain.empty() || F * cfg.n_band != T)
        return false;
    const std::string key = key_of({"head", std::to_string(ep), std::to_string(B), std::to_string(T)});
    if (!tuned.count(key)) {
        rave_edge_args a = head_desc(B, F);
        const int64_t nx = (int64_t)B * T, ny = (int64_t)B * n.c_out * F, nb = (int64_t)B * n.c_in * F;
        float* sc = scratch_buf(nx + ny + nb + 256);
        a.x = sc;
        a.x_sb = T;
        a.y = sc + nx + 64;
        a.y_sb = (int64_t)n.c_out * F;
        a.y_sc = F;
        a.weight = aptr(w_pack.at({n.name, head_wprec(ep)}));
        a.bias = n.bias ? aptr(bias_off.at(n.name)) : nullptr;
        a.filter = aptr(filt);
        a.precision = ep;
        const double fused = time_native([&](hipStream_t st) { return rave_encoder_head(&a, st); });
        double split = 1e30;
        if (precs.size() == 1) {
            split = fused >= 0 ? 1e30 : -1.0;
        } else {
            // the two ops at their best: analysis in either arithmetic, the conv's tuned launch
            rave_pqmf_analysis_args q{};
            q.n_band = cfg.n_band;
            q.taps = taps_a;
            q.n_out_bands = n.c_in;
            q.batch = B;
            q.t_in = T;
            q.pad_left = a.pqmf_pad_left;
            q.t_out = F;
            q.x = sc;
            q.x_sb = T;
            q.y = sc + nx + ny + 128;
            q.y_sb = (int64_t)n.c_in * F;
            q.y_sc = F;
            q.hkf = aptr(hkf_off);
            double ta = 1e30;
            for (int pr : {RAVE_PREC_F32, RAVE_PREC_SPLIT16}) {
                if (pr == RAVE_PREC_SPLIT16 && ep != RAVE_PREC_SPLIT16) continue;   // the exact model's own ops
                q.precision = pr;
                const double ms = time_native([&](hipStream_t st) { return rave_pqmf_analysis(&q, st); });
                if (ms >= 0) ta = std::min(ta, ms);
            }
            View dummy;
            int t_out;
            const rave_conv1d_args cd = conv_desc(n, B, F, dummy, dummy, nullptr, t_out);
            (void)conv_launch(n, cd, false, true);
            const auto it = tuned.find(key_of({"conv", n.name, "0", std::to_string(B), std::to_string(F)}));
            split = ta + (it != tuned.end() ? it->second.second : 1e30);
        }
        tuned[key] = {fused >= 0 && fused < split ? 1 : 0, fused};
    }
    return tuned.at(key).first == 1;
}

void Model::head_op(Plan& p, int B, int T, const View& x, const View& y, const View* fill_z) {
    const Node& n = g.encoder.front();
    const int F = T / cfg.n_band;
    rave_edge_args a = head_desc(B, F);
    a.x_sb = x.sb;
    a.y_sb = y.sb;
    a.y_sc = y.sc;
    if (fill_z && cfg.speaker_size > 0) {
        a.fill_channels = cfg.speaker_size;
        a.fill_t = T / hop;
        a.f_sb = fill_z->sb;
        a.f_sc = fill_z->sc;
    }
    const int ep = head_pick(B, T);
    if (ep < 0) fail(RAVE_ERR_STATE, "encoder head: no fused form for this shape");
    a.precision = ep;
    PlanOp& o = p.add(RAVE_OP_HEAD, a, "encoder_head:pqmf_analysis+" + n.name);
    rave_edge_args& A = *reinterpret_cast<rave_edge_args*>(o.op.u.raw);
    View wv = arena_view(w_pack.at({n.name, head_wprec(ep)}));
    View bv = n.bias ? arena_view(bias_off.at(n.name)) : View{};
    View hv = arena_view(ep == RAVE_PREC_SPLIT16 ? head_filt_off : head_filt32_off);
    View sv = arena_view(spk_off);
    p.bind(o, A, A.x, &x);
    p.bind(o, A, A.y, &y);
    p.bind(o, A, A.weight, &wv);
    p.bind(o, A, A.bias, n.bias ? &bv : nullptr);
    p.bind(o, A, A.filter, &hv);
    p.bind(o, A, A.fill_y, a.fill_channels ? fill_z : nullptr);
    p.bind(o, A, A.fill_values, a.fill_channels ? &sv : nullptr);
    o.prec = ep;
    o.flops = 2.0 * B * F * ((double)n.c_in * taps_a + (double)n.c_out * n.c_in * n.kernel);
    o.bytes = 4.0 * ((double)B * T + (double)B * n.c_out * F);
}

// the fused tail's arithmetic for (B, F), or -1 for the two separate ops: the
// model's edge arithmetic, and in f32_bf3 models also the bf16x3 conv form
// (exact-fp32 synthesis), whichever is timed faster
int Model::tail_pick(int B, int F) {
    std::vector<int> cands = {edge_prec()};
    if (edge_prec() == RAVE_PREC_F32_RING && std::find(precs.begin(), precs.end(), (int)RAVE_PREC_BF16X3) != precs.end())
        cands.push_back(RAVE_PREC_BF16X3);
    int best = -1;
    double bms = 1e30;
    for (int ep : cands) {
        if (!tail_ok(ep, B, F)) continue;
        const double ms = tuned.at(key_of({"tail", std::to_string(ep), std::to_string(B), std::to_string(F)})).second;
        if (best < 0 || ms < bms) {
            best = ep;
            bms = ms;
        }
    }
    return best;
}

bool Model::use_tail(int B, int F) { return tail_pick(B, F) >= 0; }

bool Model::tail_ok(int ep, int B, int F) {
    const int64_t filt = ep == RAVE_PREC_SPLIT16 ? tail_filt_off : tail_filt32_off;
    if (!edges_enabled() || ep < 0 || filt < 0) return false;
    const Node& n = g.decoder.back();
    if (!w_pack.count({n.name, ep})) return false;
    const int c_want = cfg.amplitude_modulation ? 2 * cfg.n_band : cfg.n_band;
    if (cfg.n_band != 16 || n.kernel != 7 || n.stride != 1 || n.dilation != 1 || n.transposed || n.c_in != 64 ||
        n.c_out != c_want || (n.act != RAVE_ACT_LEAKY && n.act != RAVE_ACT_SNAKE) || !n.adain.empty())
        return false;
    const std::string key = key_of({"tail", std::to_string(ep), std::to_string(B), std::to_string(F)});
    if (!tuned.count(key)) {
        rave_edge_args a = tail_desc(B, F);
        const int64_t nx = (int64_t)B * n.c_in * F, nw = (int64_t)B * n.c_out * F, ny = (int64_t)B * F * cfg.n_band;
        float* sc = scratch_buf(nx + nw + ny + 256);
        a.x = sc;
        a.x_sb = (int64_t)n.c_in * F;
        a.x_sc = F;
        a.y = sc + ((nx + nw + 63) / 64 + 1) * 64;     // 16-byte aligned
        a.y_sb = (int64_t)F * cfg.n_band;
        a.weight = aptr(w_pack.at({n.name, ep}));
        a.bias = n.bias ? aptr(bias_off.at(n.name)) : nullptr;
        a.alpha = n.act == RAVE_ACT_SNAKE ? aptr(alpha_off.at(n.alpha)) : nullptr;
        a.filter = aptr(filt);
        a.precision = ep;
        const double fused = time_native([&](hipStream_t st) { return rave_decoder_tail(&a, st); });
        double split = 1e30;
        if (precs.size() == 1) {
            split = fused >= 0 ? 1e30 : -1.0;
        } else {
            rave_pqmf_synthesis_args q{};
            q.n_band = cfg.n_band;
            q.taps = taps_s;
            q.batch = B;
            q.t_in = F;
            q.pad_left = a.pqmf_pad_left;
            q.mode = a.mode;
            q.x = sc + nx + 64;
            q.x_sb = (int64_t)n.c_out * F;
            q.x_sc = F;
            q.y = a.y;
            q.y_sb = a.y_sb;
            q.hki = aptr(hki_off);
            double ts = 1e30;
            for (int pr : {RAVE_PREC_F32, RAVE_PREC_SPLIT16}) {
                if (pr == RAVE_PREC_SPLIT16 && ep != RAVE_PREC_SPLIT16) continue;   // the exact model's own ops
                q.precision = pr;
                const double ms = time_native([&](hipStream_t st) { return rave_pqmf_synthesis(&q, st); });
                if (ms >= 0) ts = std::min(ts, ms);
            }
            View dummy;
            int t_out;
            const rave_conv1d_args cd = conv_desc(n, B, F, dummy, dummy, nullptr, t_out);
            (void)conv_launch(n, cd, false, true);
            const auto it = tuned.find(key_of({"conv", n.name, "0", std::to_string(B), std::to_string(F)}));
            split = ts + (it != tuned.end() ? it->second.second : 1e30);
        }
        tuned[key] = {fused >= 0 && fused < split ? 1 : 0, fused};
    }
    return tuned.at(key).first == 1;
}

void Model::tail_op(Plan& p, int B, int F, const View& x, const View& y, const View* noise) {
    const Node& n = g.decoder.back();
    rave_edge_args a = tail_desc(B, F);
    a.x_sb = x.sb;
    a.x_sc = x.sc;
    a.y_sb = y.sb;
    a.n_sb = noise ? noise->sb : 0;
    a.n_sc = noise ? noise->sc : 0;
    const int ep = tail_pick(B, F);
    if (ep < 0) fail(RAVE_ERR_STATE, "decoder tail: no fused form for this shape");
    a.precision = ep;
    PlanOp& o = p.add(RAVE_OP_TAIL, a, "decoder_tail:" + n.name + "+pqmf_synthesis");
    rave_edge_args& A = *reinterpret_cast<rave_edge_args*>(o.op.u.raw);
    View wv = arena_view(w_pack.at({n.name, ep}));
    View bv = n.bias ? arena_view(bias_off.at(n.name)) : View{};
    View av = n.act == RAVE_ACT_SNAKE ? arena_view(alpha_off.at(n.alpha)) : View{};
    View hv = arena_view(ep == RAVE_PREC_SPLIT16 ? tail_filt_off : tail_filt32_off);
    p.bind(o, A, A.x, &x);
    p.bind(o, A, A.y, &y);
    p.bind(o, A, A.weight, &wv);
    p.bind(o, A, A.bias, n.bias ? &bv : nullptr);
    p.bind(o, A, A.alpha, n.act == RAVE_ACT_SNAKE ? &av : nullptr);
    p.bind(o, A, A.filter, &hv);
    p.bind(o, A, A.noise, noise);
    o.prec = ep;
    o.flops = 2.0 * B * F * ((double)n.c_out * n.c_in * n.kernel + (double)cfg.n_band * cfg.n_band * taps_s);
    o.bytes = 4.0 * ((double)B * n.c_in * F + (double)B * F * cfg.n_band + (noise ? (double)B * cfg.n_band * F : 0.0));
}

// ResidualVectorQuantization.encode (rave/quantization.py:302-310): latents
// (B, latent, Fz) at `lat` -> indices (B, n_q, Fz) int64 at `idx`
void Model::rvq_encode_op(Plan& p, int B, int Fz, const View& lat, const View& idx) {
    rave_rvq_args r{};
    r.n_q = cfg.rvq_quantizers;
    r.codebook_size = cfg.rvq_codebook_size;
    r.dim = cfg.latent_size;
    r.batch = B;
    r.t_len = Fz;
    r.z_sb = lat.sb;
    r.z_sc = lat.sc;
    r.i_sb = (int64_t)cfg.rvq_quantizers * Fz;
    r.i_sq = Fz;
    const int64_t nw = rave_rvq_workspace(&r);
    if (nw < 0) fail(RAVE_ERR_ARG, std::string("rvq_workspace: ") + rave_last_error());
    View work = ws_view(p.ws.alloc(std::max<int64_t>(nw, 1)), 0, 0);
    PlanOp& o = p.add(RAVE_OP_RVQ_ENCODE, r, "rvq_encode");
    rave_rvq_args& R = *reinterpret_cast<rave_rvq_args*>(o.op.u.raw);
    View cb = arena_view(cb_off);
    p.bind(o, R, R.codebooks, &cb);
    p.bind(o, R, R.z, &lat);
    p.bind(o, R, R.idx, &idx);
    p.bind(o, R, R.y, nullptr);
    p.bind(o, R, R.work, &work);
}

// ResidualVectorQuantization.decode (rave/quantization.py:312-318) with
// DiscreteScriptedRAVE's clamp (scripts/export.py:507-509): indices at `idx`
// -> the latent channels of `z`
void Model::rvq_decode_op(Plan& p, int B, int Fz, const View& idx, const View& z) {
    rave_rvq_args r{};
    r.n_q = cfg.rvq_quantizers;
    r.codebook_size = cfg.rvq_codebook_size;
    r.dim = cfg.latent_size;
    r.batch = B;
    r.t_len = Fz;
    r.i_sb = (int64_t)cfg.rvq_quantizers * Fz;
    r.i_sq = Fz;
    r.y_sb = z.sb;
    r.y_sc = z.sc;
    PlanOp& o = p.add(RAVE_OP_RVQ_DECODE, r, "rvq_decode");
    rave_rvq_args& R = *reinterpret_cast<rave_rvq_args*>(o.op.u.raw);
    View cb = arena_view(cb_off);
    p.bind(o, R, R.codebooks, &cb);
    p.bind(o, R, R.z, nullptr);
    p.bind(o, R, R.idx, &idx);
    p.bind(o, R, R.y, &z);
    p.bind(o, R, R.work, nullptr);
}

// ------------------------------------------------------------------ plans
static std::vector<const Node*> ptrs_of(const std::vector<Node>& v) {
    std::vector<const Node*> out;
    for (const Node& n : v) out.push_back(&n);
    return out;
}

Plan& Model::encode_plan(int B, int T, bool codes) {
    const std::string key = std::string(codes ? "enc_codes" : "enc") + "|" + std::to_string(B) + "|" +
                            std::to_string(T) + adain_key();
    auto it = plans.find(key);
    if (it != plans.end()) return *it->second;
    auto plan = std::make_unique<Plan>();
    Plan& p = *plan;
    const int F = T / cfg.n_band, Fz = T / hop;
    View lat;
    if (codes) lat = ws_view(p.ws.alloc((int64_t)B * cfg.latent_size * Fz), (int64_t)cfg.latent_size * Fz, Fz);
    else lat = io_view(1, (int64_t)(cfg.latent_size + cfg.speaker_size) * Fz, Fz);
    const View spk_z = lat.at((int64_t)cfg.latent_size * Fz);
    std::vector<const Node*> nodes = ptrs_of(g.encoder);
    if (use_head(B, T)) {
        // analysis + the first conv (+ the speaker fill) in one launch
        const Node& n0 = *nodes.front();
        // workspace laid out as the two-op path lays it (the bands tensor's slot,
        // then the conv's output, freed after its last use), so every later tensor
        // lands at the same offset with or without the fusion
        const int64_t n_bands = (int64_t)B * cfg.enc_bands * F, n_h0 = (int64_t)B * n0.c_out * F;
        (void)p.ws.alloc(n_bands);
        View h0 = ws_view(p.ws.alloc(n_h0), (int64_t)n0.c_out * F, F);
        head_op(p, B, T, io_view(0, T, T), h0, codes ? nullptr : &spk_z);
        nodes.erase(nodes.begin());
        run_stack(p, nodes, B, {{n0.dst, {h0, F}}}, {{"latent", lat}}, {{n0.dst, n_h0}});
        if (codes) rvq_encode_op(p, B, Fz, lat, io_view(1, 0, 0));
    } else {
        View bands = ws_view(p.ws.alloc((int64_t)B * cfg.enc_bands * F), (int64_t)cfg.enc_bands * F, F);
        analysis_op(p, B, T, io_view(0, T, T), bands, cfg.enc_bands, get_padding(taps_a, 1, cfg.causal).first, T);
        run_stack(p, nodes, B, {{"enc_in", {bands, F}}}, {{"latent", lat}});
        if (codes) rvq_encode_op(p, B, Fz, lat, io_view(1, 0, 0));
        else fill_speaker(p, B, Fz, spk_z);
    }
    p.finalize(arena);
    return *(plans[key] = std::move(plan));
}

Plan& Model::decode_plan(int B, int Fz, bool codes) {
    const std::string key = std::string(codes ? "dec_codes" : "dec") + "|" + std::to_string(B) + "|" +
                            std::to_string(Fz) + adain_key();
    auto it = plans.find(key);
    if (it != plans.end()) return *it->second;
    auto plan = std::make_unique<Plan>();
    Plan& p = *plan;
    View z;
    if (codes) {
        z = ws_view(p.ws.alloc((int64_t)B * dec_in * Fz), (int64_t)dec_in * Fz, Fz);
        rvq_decode_op(p, B, Fz, io_view(0, 0, 0), z);
        fill_speaker(p, B, Fz, z.at((int64_t)cfg.latent_size * Fz));
    } else {
        z = io_view(0, (int64_t)dec_in * Fz, Fz);
    }
    const int F = Fz * hop / cfg.n_band;
    const bool tail = use_tail(B, F);
    const Node& wnode = g.decoder.back();
    std::map<std::string, View> outputs;
    View wave, feat;
    if (tail) {
        // the waveform conv runs inside the fused tail: its input is the stack's output
        feat = ws_view(p.ws.alloc((int64_t)B * wnode.c_in * F), (int64_t)wnode.c_in * F, F);
        outputs[wnode.src] = feat;
    } else {
        wave = ws_view(p.ws.alloc((int64_t)B * dec_out * F), (int64_t)dec_out * F, F);
        outputs["wave"] = wave;
    }
    int Fn = 0, na = 0;
    if (cfg.noise) {
        Fn = F / noise_target;
        na = cfg.n_band * cfg.noise_bands;
        outputs["noise_amp"] = ws_view(p.ws.alloc((int64_t)B * na * Fn), (int64_t)na * Fn, Fn);
    }
    std::vector<const Node*> nodes = ptrs_of(g.decoder);
    if (tail) nodes.pop_back();
    for (const Node& n : g.noise) nodes.push_back(&n);
    run_stack(p, nodes, B, {{"dec_in", {z, Fz}}}, outputs);
    View noise_v;
    if (cfg.noise) {
        // NoiseGeneratorV2's filter stage; the uniform noise is I/O slot 2
        noise_v = ws_view(p.ws.alloc((int64_t)B * cfg.n_band * F), (int64_t)cfg.n_band * F, F);
        const View& amp = outputs["noise_amp"];
        rave_noise_args a{};
        a.batch = B;
        a.frames = Fn;
        a.n_band = cfg.n_band;
        a.noise_bands = cfg.noise_bands;
        a.target = noise_target;
        a.a_sb = amp.sb;
        a.a_sc = amp.sc;
        a.u_sb = (int64_t)Fn * cfg.n_band * noise_target;
        a.y_sb = noise_v.sb;
        a.y_sc = noise_v.sc;
        PlanOp& o = p.add(RAVE_OP_NOISE, a, "noise_synth");
        rave_noise_args& N = *reinterpret_cast<rave_noise_args*>(o.op.u.raw);
        View u = io_view(2, 0, 0);
        p.bind(o, N, N.amp, &amp);
        p.bind(o, N, N.u, &u);
        p.bind(o, N, N.y, &noise_v);
    }
    const int T = F * cfg.n_band;
    if (tail)
        tail_op(p, B, F, feat, io_view(1, T, T), cfg.noise ? &noise_v : nullptr);
    else
        synthesis_op(p, B, F, wave, io_view(1, T, T), cfg.noise ? &noise_v : nullptr,
                     get_padding(taps_s, 1, cfg.causal).first, 0, 0);
    p.finalize(arena);
    return *(plans[key] = std::move(plan));
}

Plan& Model::plan_of(int which, int B, int T) {
    switch (which) {
        case 0: return encode_plan(B, T, false);
        case 1: return decode_plan(B, T, false);
        case 2: return encode_plan(B, T, true);
        case 3: return decode_plan(B, T, true);
        default: fail(RAVE_ERR_ARG, "plan kind must be 0..3");
    }
}

// One call of a plan kind over `batch` items: I/O slot 0 = in, 1 = out, 2 = noise.
void Model::run_kind(int which, int batch, int t, const void* in, void* out, const float* noise, hipStream_t st) {
    cur_stream = st;
    Plan& p = plan_of(which, batch, t);
    void* slots[3] = {(void*)in, out, (void*)noise};
    p.run(slots, (which == 1 || which == 3) && cfg.noise ? 3 : 2, st);
}

const float* Model::noise_ptr(const float* u, int B, int Fz, hipStream_t st) {
    if (!cfg.noise) return nullptr;
    if (u) return u;
    const int F = Fz * hop / cfg.n_band;
    const int64_t n = (int64_t)B * (F / noise_target) * cfg.n_band * noise_target;
    if (n > noise_n) {
        if (noise) RAVE_HIP_OR_THROW(hipFree(noise));
        noise = nullptr;
        RAVE_HIP_OR_THROW(hipMalloc(&noise, (size_t)n * 4));
        noise_n = n;
    }
    check_rc(rave_fill_uniform(noise, n, 0x243F6A8885A308D3ull + 0x9E3779B97F4A7C15ull * ++noise_calls, 0.f, 1.f, st),
             "noise draw");
    return noise;
}

// ------------------------------------------------------------------ weights
static std::vector<float> fold_wn(const float* g, const float* v, int64_t rows, int64_t per_row) {
    std::vector<float> w((size_t)(rows * per_row));
    for (int64_t r = 0; r < rows; ++r) {
        double ss = 0;
        for (int64_t i = 0; i < per_row; ++i) ss += (double)v[r * per_row + i] * v[r * per_row + i];
        const double s = (double)g[r] / std::sqrt(ss);
        for (int64_t i = 0; i < per_row; ++i) w[r * per_row + i] = (float)((double)v[r * per_row + i] * s);
    }
    return w;
}

static Model* create_model(const rave_model_config& cfg, const rave_param* params, int n_params,
                           const float* speaker, int precision) {
    auto m = std::make_unique<Model>();
    m->cfg = cfg;
    build_graph(cfg, m->g);
    if (precision == RAVE_PREC_AUTO) m->precs = {RAVE_PREC_F32, RAVE_PREC_SPLIT16};
    else if (precision == RAVE_PREC_F32 || precision == RAVE_PREC_SPLIT16) m->precs = {precision};
    else if (precision == RAVE_PREC_F32_TUNED) m->precs = {RAVE_PREC_F32, RAVE_PREC_F32_RING};
    else if (precision == RAVE_PREC_F32_BF3) m->precs = {RAVE_PREC_F32, RAVE_PREC_F32_RING, RAVE_PREC_BF16X3};
    else fail(RAVE_ERR_ARG, "precision must be RAVE_PREC_F32, RAVE_PREC_SPLIT16, RAVE_PREC_AUTO, RAVE_PREC_F32_TUNED "
                            "or RAVE_PREC_F32_BF3");
    m->autotune = precision == RAVE_PREC_AUTO || precision == RAVE_PREC_F32_TUNED || precision == RAVE_PREC_F32_BF3;
    m->hop = cfg.n_band;
    for (int i = 0; i < cfg.n_ratios; ++i) m->hop *= cfg.ratios[i];
    m->dec_in = cfg.latent_size + cfg.speaker_size;
    m->dec_out = cfg.amplitude_modulation ? 2 * cfg.n_band : cfg.n_band;
    if (cfg.noise) {
        m->noise_target = 1;
        for (int i = 0; i < cfg.n_noise_ratios; ++i) m->noise_target *= cfg.noise_ratios[i];
    }
    // parameters by name, every expected one present with its size
    std::map<std::string, std::pair<const float*, int64_t>> P;
    for (int i = 0; i < n_params; ++i) {
        if (!params[i].name || !params[i].data) fail(RAVE_ERR_ARG, "null parameter entry");
        P[params[i].name] = {params[i].data, params[i].numel};
    }
    for (auto& e : param_table(cfg)) {
        auto it = P.find(e.first);
        if (it == P.end()) fail(RAVE_ERR_ARG, "missing parameter " + e.first);
        if (!e.second.empty()) {
            int64_t n = 1;
            for (int64_t d : e.second) n *= d;
            if (it->second.second != n)
                fail(RAVE_ERR_ARG, e.first + ": expected " + std::to_string(n) + " values, got " +
                                       std::to_string(it->second.second));
        }
    }
    if (!speaker && cfg.speaker_size > 0) fail(RAVE_ERR_ARG, "speaker embedding is required");
    auto get = [&](const std::string& n) { return P.at(n).first; };
    // conv weights, per arithmetic (ConvTranspose also in its cached streaming form)
    for (const Node* n : m->g.convs()) {
        const int64_t rows = n->transposed ? n->c_in : n->c_out;
        const int64_t per_row = (n->transposed ? n->c_out : n->c_in) * (int64_t)n->kernel;
        std::vector<float> w = n->weight_norm ? fold_wn(get(n->name + ".weight_g"), get(n->name + ".weight_v"), rows, per_row)
                                              : std::vector<float>(get(n->name + ".weight"),
                                                                   get(n->name + ".weight") + rows * per_row);
        for (int pr : m->precs) {
            for (int form = 0; form < (n->transposed ? 2 : 1); ++form) {
                const int os = n->transposed ? (form == 0 ? n->stride / 2 : 0) : 0;
                // split16 and the fp32 ring path share the fragment image layout
                const bool sp = pr == RAVE_PREC_SPLIT16 || pr == RAVE_PREC_F32_RING;
                const int64_t sz = pr == RAVE_PREC_BF16X3
                                       ? rave_conv1d_bf3_packed_size(n->c_in, n->c_out, n->kernel, n->stride,
                                                                     n->dilation, n->transposed)
                                   : sp ? rave_conv1d_split_packed_size(n->c_in, n->c_out, n->kernel, n->stride,
                                                                        n->dilation, n->transposed)
                                        : rave_conv1d_packed_size(n->c_in, n->c_out, n->kernel, n->stride, n->dilation,
                                                                  n->transposed);
                if (sz <= 0) fail(RAVE_ERR_UNSUPPORTED, "conv " + n->name + ": unsupported layer shape");
                std::vector<float> packed((size_t)sz, 0.f);
                const int rc =
                    pr == RAVE_PREC_SPLIT16
                        ? rave_conv1d_split_pack_weight(w.data(), n->c_in, n->c_out, n->kernel, n->stride, n->dilation,
                                                        n->transposed, os, packed.data())
                    : pr == RAVE_PREC_F32_RING
                        ? rave_conv1d_ring_pack_weight(w.data(), n->c_in, n->c_out, n->kernel, n->stride, n->dilation,
                                                       n->transposed, os, packed.data())
                    : pr == RAVE_PREC_BF16X3
                        ? rave_conv1d_bf3_pack_weight(w.data(), n->c_in, n->c_out, n->kernel, n->stride, n->dilation,
                                                      n->transposed, os, packed.data())
                        : rave_conv1d_pack_weight(w.data(), n->c_in, n->c_out, n->kernel, n->stride, n->dilation,
                                                  n->transposed, os, packed.data());
                check_rc(rc, "pack " + n->name);
                (form == 0 ? m->w_pack : m->w_pack_stream)[{n->name, pr}] = m->add(packed);
            }
        }
        if (n->bias) m->bias_off[n->name] = m->add(get(n->name + ".bias"), n->c_out);
        if (n->act == RAVE_ACT_SNAKE && !m->alpha_off.count(n->alpha))
            m->alpha_off[n->alpha] = m->add(get(n->alpha), n->c_in);
    }
    // fused Residual(DilatedUnit) weights
    if (cfg.fuse_units) {
        std::vector<const Node*> all = m->g.convs();
        for (auto& pr : m->unit_pairs(all)) {
            const Node& k3 = *pr.first;
            const Node& k1 = *pr.second;
            const int C_ = k3.c_in;
            std::vector<float> w1 = fold_wn(get(k3.name + ".weight_g"), get(k3.name + ".weight_v"), C_, (int64_t)C_ * 3);
            std::vector<float> w2 = fold_wn(get(k1.name + ".weight_g"), get(k1.name + ".weight_v"), C_, C_);
            for (int p : m->precs) {
                // split16 and the fp32 ring kernel share the fragment image layout
                const bool sp = p == RAVE_PREC_SPLIT16 || p == RAVE_PREC_F32_RING;
                const int64_t sz = p == RAVE_PREC_BF16X3 ? rave_unit_bf3_packed_size(C_)
                                   : sp                  ? rave_unit_split_packed_size(C_)
                                                         : rave_unit_packed_size(C_);
                if (sz <= 0) continue;
                std::vector<float> packed((size_t)sz, 0.f);
                check_rc(p == RAVE_PREC_SPLIT16    ? rave_unit_split_pack_weight(w1.data(), w2.data(), C_, packed.data())
                         : p == RAVE_PREC_F32_RING ? rave_unit_ring_pack_weight(w1.data(), w2.data(), C_, packed.data())
                         : p == RAVE_PREC_BF16X3   ? rave_unit_bf3_pack_weight(w1.data(), w2.data(), C_, packed.data())
                                                   : rave_unit_pack_weight(w1.data(), w2.data(), C_, packed.data()),
                         "unit pack " + k3.name);
                m->unit_pack[{k3.name, p}] = m->add(packed);
                m->unit_ok.insert(k3.name);
            }
        }
    }
    // PQMF kernels of CachedPQMF.__init__ (rave/pqmf.py:236-263): hkf = make_odd(hk),
    // hki = flip + "c (t m) -> m c t" polyphase rearrange, made odd
    {
        const auto& hk = P.at("pqmf.hk");
        const int nb = cfg.n_band;
        if (hk.second <= 0 || hk.second % nb) fail(RAVE_ERR_ARG, "pqmf.hk must be (n_band, L)");
        const int L = (int)(hk.second / nb);
        if (L % nb) fail(RAVE_ERR_ARG, "pqmf.hk length must be a multiple of n_band");
        m->taps_a = L % 2 == 0 ? L + 1 : L;
        std::vector<float> hkf((size_t)nb * m->taps_a, 0.f);
        for (int b = 0; b < nb; ++b)
            for (int j = 0; j < L; ++j) hkf[(size_t)b * m->taps_a + j] = hk.first[(size_t)b * L + j];
        const int tl = L / nb;
        m->taps_s = tl % 2 == 0 ? tl + 1 : tl;
        std::vector<float> hki((size_t)nb * nb * m->taps_s, 0.f);
        for (int mm = 0; mm < nb; ++mm)
            for (int c = 0; c < nb; ++c)
                for (int t = 0; t < tl; ++t)
                    hki[((size_t)mm * nb + c) * m->taps_s + t] = hk.first[(size_t)c * L + (L - 1 - (t * nb + mm))];
        m->hkf_off = m->add(hkf);
        m->hki_off = m->add(hki);
        // the fused edges' pre-split filter images (split16 models; shapes the kernels build)
        std::vector<float> img(RAVE_EDGE_FILTER_FLOATS, 0.f);
        if (rave_encoder_head_pack_filter(hkf.data(), nb, m->taps_a, cfg.enc_bands, img.data()) == RAVE_OK)
            m->head_filt_off = m->add(img);
        if (rave_decoder_tail_pack_filter(hki.data(), nb, m->taps_s, img.data()) == RAVE_OK)
            m->tail_filt_off = m->add(img);
        if (rave_encoder_head_pack_filter_f32(hkf.data(), nb, m->taps_a, cfg.enc_bands, img.data()) == RAVE_OK)
            m->head_filt32_off = m->add(img);
        if (rave_decoder_tail_pack_filter_f32(hki.data(), nb, m->taps_s, img.data()) == RAVE_OK)
            m->tail_filt32_off = m->add(img);
    }
    m->spk_off = cfg.speaker_size > 0 ? m->add(speaker, cfg.speaker_size) : 0;
    if (cfg.rvq_quantizers > 0) {
        std::vector<float> cbs;
        for (int i = 0; i < cfg.rvq_quantizers; ++i) {
            const float* e = get("encoder.rvq.layers." + std::to_string(i) + "._codebook.embed");
            cbs.insert(cbs.end(), e, e + (int64_t)cfg.rvq_codebook_size * cfg.latent_size);
        }
        m->cb_off = m->add(cbs);
    }
    RAVE_HIP_OR_THROW(hipMalloc(&m->arena, std::max<size_t>(m->host.size(), 64) * 4));
    RAVE_HIP_OR_THROW(hipMemcpy(m->arena, m->host.data(), m->host.size() * 4, hipMemcpyHostToDevice));
    m->host.clear();
    m->host.shrink_to_fit();
    // AdaIN buffers: mean_x 0, std_x 1, mean_y 0, std_y 1, counters 0
    if (!m->g.adain_modules.empty()) {
        int64_t off = 0;
        for (size_t i = 0; i < m->g.adain_modules.size(); ++i) {
            m->ad_index[m->g.adain_modules[i].first] = (int)i;
            m->ad_off.push_back(off);
            off += 4LL * m->max_batch * m->g.adain_modules[i].second;
        }
        std::vector<float> init((size_t)off, 0.f);
        for (size_t i = 0; i < m->g.adain_modules.size(); ++i) {
            const int64_t plane = (int64_t)m->max_batch * m->g.adain_modules[i].second;
            std::fill(init.begin() + m->ad_off[i] + plane, init.begin() + m->ad_off[i] + 2 * plane, 1.f);
            std::fill(init.begin() + m->ad_off[i] + 3 * plane, init.begin() + m->ad_off[i] + 4 * plane, 1.f);
        }
        const size_t na = m->g.adain_modules.size();
        RAVE_HIP_OR_THROW(hipMalloc(&m->ad_stats, init.size() * 4));
        RAVE_HIP_OR_THROW(hipMemcpy(m->ad_stats, init.data(), init.size() * 4, hipMemcpyHostToDevice));
        RAVE_HIP_OR_THROW(hipMalloc(&m->ad_init, init.size() * 4));
        RAVE_HIP_OR_THROW(hipMemcpy(m->ad_init, init.data(), init.size() * 4, hipMemcpyHostToDevice));
        RAVE_HIP_OR_THROW(hipMalloc(&m->ad_counters, na * 2 * 4));
        RAVE_HIP_OR_THROW(hipMemset(m->ad_counters, 0, na * 2 * 4));
        RAVE_HIP_OR_THROW(hipMalloc(&m->ad_tickets, na * 4));
        RAVE_HIP_OR_THROW(hipMemset(m->ad_tickets, 0, na * 4));
    }
    return m.release();
}

}  // namespace rave

// =================================================================== C-ABI
using namespace rave;

struct rave_model {
    std::unique_ptr<rave::Model> m;
};

template <typename F>
static int guarded(F&& f) {
    try {
        f();
        return RAVE_OK;
    } catch (const EngineError& e) {
        set_error(e.msg);
        return e.code;
    } catch (const std::exception& e) {
        set_error(std::string("engine: ") + e.what());
        return RAVE_ERR_STATE;
    }
}

namespace rave {
static Model* model_of(rave_model* h) {
    if (!h || !h->m) fail(RAVE_ERR_STATE, "null model");
    return h->m.get();
}
}  // namespace rave

extern "C" int rave_model_param_count(const rave_model_config* cfg) {
    int n = 0;
    int rc = guarded([&] {
        if (!cfg) fail(RAVE_ERR_ARG, "null config");
        n = (int)param_table(*cfg).size();
    });
    return rc == RAVE_OK ? n : rc;
}

extern "C" int rave_model_param_info(const rave_model_config* cfg, int i, char* name, int name_cap, int64_t* numel) {
    return guarded([&] {
        if (!cfg) fail(RAVE_ERR_ARG, "null config");
        auto t = param_table(*cfg);
        if (i < 0 || i >= (int)t.size()) fail(RAVE_ERR_ARG, "parameter index out of range");
        if (name && name_cap > 0) {
            std::strncpy(name, t[i].first.c_str(), (size_t)name_cap - 1);
            name[name_cap - 1] = 0;
        }
        if (numel) {
            int64_t n = t[i].second.empty() ? -1 : 1;
            for (int64_t d : t[i].second) n *= d;
            *numel = n;
        }
    });
}

extern "C" int rave_model_create(const rave_model_config* cfg, const rave_param* params, int n_params,
                                 const float* speaker, int precision, rave_model** out) {
    return guarded([&] {
        if (!cfg || !out || (n_params > 0 && !params)) fail(RAVE_ERR_ARG, "model_create: null argument");
        *out = nullptr;
        auto h = std::make_unique<rave_model>();
        h->m.reset(create_model(*cfg, params, n_params, speaker, precision));
        *out = h.release();
    });
}

extern "C" int rave_model_destroy(rave_model* m) {
    delete m;
    return RAVE_OK;
}

// NoiseGeneratorV2 reshapes its amplitudes per noise frame (rave/blocks.py:283-285):
// the band-rate length must divide by prod(noise ratios), as the reference's
// reshape requires
static void check_noise_frames(Model* m, int frames) {
    if (!m->cfg.noise) return;
    const int64_t F = (int64_t)frames * m->hop / m->cfg.n_band;
    if (F % m->noise_target)
        fail(RAVE_ERR_ARG, "noise synthesizer: " + std::to_string(F) + " band frames do not divide by prod(noise ratios) = " +
                               std::to_string(m->noise_target));
}

static void check_len(Model* m, int batch, int t) {
    if (batch <= 0 || t <= 0) fail(RAVE_ERR_ARG, "batch and length must be positive");
    if (t % m->hop) fail(RAVE_ERR_ARG, "T=" + std::to_string(t) + " must be a multiple of " + std::to_string(m->hop) +
                                           " (n_band * prod(ratios))");
    check_noise_frames(m, t / m->hop);
}

extern "C" int rave_model_encode(rave_model* h, const float* x, int batch, int t, float* z, void* stream) {
    return guarded([&] {
        Model* m = model_of(h);
        m->coop_check();
        if (!x || !z) fail(RAVE_ERR_ARG, "encode: null tensor");
        check_len(m, batch, t);
        m->run_kind(0, batch, t, x, z, nullptr, as_stream(stream));
    });
}

extern "C" int rave_model_decode(rave_model* h, const float* z, int batch, int frames, float* y,
                                 const float* noise_u, void* stream) {
    return guarded([&] {
        Model* m = model_of(h);
        m->coop_check();
        if (!z || !y) fail(RAVE_ERR_ARG, "decode: null tensor");
        if (batch <= 0 || frames <= 0) fail(RAVE_ERR_ARG, "batch and frames must be positive");
        check_noise_frames(m, frames);
        m->run_kind(1, batch, frames, z, y, m->noise_ptr(noise_u, batch, frames, as_stream(stream)),
                    as_stream(stream));
    });
}

extern "C" int rave_model_forward(rave_model* h, const float* x, int batch, int t, float* y, const float* noise_u,
                                  void* stream) {
    return guarded([&] {
        Model* m = model_of(h);
        m->coop_check();
        if (!x || !y) fail(RAVE_ERR_ARG, "forward: null tensor");
        check_len(m, batch, t);
        const int Fz = t / m->hop;
        const int64_t nz = (int64_t)batch * m->dec_in * Fz;
        if (nz > m->fwd_z_n) {
            if (m->fwd_z) RAVE_HIP_OR_THROW(hipFree(m->fwd_z));
            m->fwd_z = nullptr;
            RAVE_HIP_OR_THROW(hipMalloc(&m->fwd_z, (size_t)nz * 4));
            m->fwd_z_n = nz;
        }
        if (m->cfg.rvq_quantizers > 0) fail(RAVE_ERR_ARG, "forward of a discrete config: use encode_codes / decode_codes");
        m->run_kind(0, batch, t, x, m->fwd_z, nullptr, as_stream(stream));
        m->run_kind(1, batch, Fz, m->fwd_z, y, m->noise_ptr(noise_u, batch, Fz, as_stream(stream)), as_stream(stream));
    });
}

extern "C" int rave_model_encode_codes(rave_model* h, const float* x, int batch, int t, int64_t* idx, void* stream) {
    return guarded([&] {
        Model* m = model_of(h);
        m->coop_check();
        if (m->cfg.rvq_quantizers <= 0) fail(RAVE_ERR_ARG, "encode_codes needs a discrete (RVQ) config");
        if (!x || !idx) fail(RAVE_ERR_ARG, "encode_codes: null tensor");
        check_len(m, batch, t);
        m->run_kind(2, batch, t, x, idx, nullptr, as_stream(stream));
    });
}

extern "C" int rave_model_decode_codes(rave_model* h, const int64_t* idx, int batch, int frames, float* y,
                                       const float* noise_u, void* stream) {
    return guarded([&] {
        Model* m = model_of(h);
        m->coop_check();
        if (m->cfg.rvq_quantizers <= 0) fail(RAVE_ERR_ARG, "decode_codes needs a discrete (RVQ) config");
        if (!idx || !y) fail(RAVE_ERR_ARG, "decode_codes: null tensor");
        if (batch <= 0 || frames <= 0) fail(RAVE_ERR_ARG, "batch and frames must be positive");
        check_noise_frames(m, frames);
        m->run_kind(3, batch, frames, idx, y, m->noise_ptr(noise_u, batch, frames, as_stream(stream)),
                    as_stream(stream));
    });
}

extern "C" int rave_model_check(rave_model* h, int wait, void* stream) {
    return guarded([&] {
        Model* m = model_of(h);
        if (wait) RAVE_HIP_OR_THROW(hipStreamSynchronize(as_stream(stream)));
        m->coop_check();
    });
}

extern "C" int rave_model_noise_shape(const rave_model* h, int batch, int frames, int64_t* out4) {
    return guarded([&] {
        const Model* m = model_of(const_cast<rave_model*>(h));
        if (!out4) fail(RAVE_ERR_ARG, "null output");
        if (!m->cfg.noise) fail(RAVE_ERR_ARG, "config has no noise synthesizer");
        const int F = frames * m->hop / m->cfg.n_band;
        out4[0] = batch;
        out4[1] = F / m->noise_target;
        out4[2] = m->cfg.n_band;
        out4[3] = m->noise_target;
    });
}

// ------------------------------------------------------------------ AdaIN controls
extern "C" int rave_model_adain_control(rave_model* h, int learn_x, int learn_y, int reset_x, int reset_y,
                                        void* stream) {
    return guarded([&] {
        Model* m = model_of(h);
        if (m->ad_index.empty()) return;
        if (learn_x >= 0) m->learn_x = learn_x != 0;
        if (learn_y >= 0) m->learn_y = learn_y != 0;
        if (m->learn_x || m->learn_y) m->touched = true;
        // resets are ordered on the caller's stream after the learning-mode
        // kernels already queued there (device-to-device from the reset image)
        hipStream_t st = as_stream(stream);
        for (size_t i = 0; i < m->g.adain_modules.size() && (reset_x || reset_y); ++i) {
            const int64_t plane = (int64_t)m->max_batch * m->g.adain_modules[i].second;
            float* base = m->ad_stats + m->ad_off[i];
            const float* init = m->ad_init + m->ad_off[i];
            if (reset_x) {   // AdaptiveInstanceNormalization.reset_x (rave/blocks.py:876-879)
                RAVE_HIP_OR_THROW(hipMemcpyAsync(base, init, 2 * plane * 4, hipMemcpyDeviceToDevice, st));
                RAVE_HIP_OR_THROW(hipMemsetAsync(m->ad_counters + 2 * i, 0, 4, st));
            }
            if (reset_y) {   // reset_y (rave/blocks.py:881-884)
                RAVE_HIP_OR_THROW(hipMemcpyAsync(base + 2 * plane, init + 2 * plane, 2 * plane * 4,
                                                 hipMemcpyDeviceToDevice, st));
                RAVE_HIP_OR_THROW(hipMemsetAsync(m->ad_counters + 2 * i + 1, 0, 4, st));
            }
        }
    });
}

extern "C" int rave_model_set_row0(rave_model* h, int row0) {
    return guarded([&] {
        Model* m = model_of(h);
        if (row0 < 0) fail(RAVE_ERR_ARG, "row0 must be >= 0");
        m->row0 = row0;
    });
}

extern "C" int rave_model_set_speaker(rave_model* h, const float* speaker, void* stream) {
    return guarded([&] {
        Model* m = model_of(h);
        if (!speaker) fail(RAVE_ERR_ARG, "set_speaker: null embedding");
        if (m->cfg.speaker_size == 0) fail(RAVE_ERR_ARG, "set_speaker: the model has no speaker channels");
        // host or device source (unified addressing); ordered on the caller's stream
        // before every later encode/decode (and streaming graph replay) on it
        RAVE_HIP_OR_THROW(hipMemcpyAsync(m->arena + m->spk_off, speaker, sizeof(float) * m->cfg.speaker_size,
                                         hipMemcpyDefault, as_stream(stream)));
        ++m->spk_version;
    });
}

extern "C" int rave_model_adain_count(const rave_model* h) {
    int n = 0;
    int rc = guarded([&] { n = (int)model_of(const_cast<rave_model*>(h))->g.adain_modules.size(); });
    return rc == RAVE_OK ? n : rc;
}

extern "C" int rave_model_adain_info(const rave_model* h, int i, char* name, int name_cap, int* channels,
                                     int* max_batch) {
    return guarded([&] {
        const Model* m = model_of(const_cast<rave_model*>(h));
        if (i < 0 || i >= (int)m->g.adain_modules.size()) fail(RAVE_ERR_ARG, "AdaIN index out of range");
        if (name && name_cap > 0) {
            std::strncpy(name, m->g.adain_modules[i].first.c_str(), (size_t)name_cap - 1);
            name[name_cap - 1] = 0;
        }
        if (channels) *channels = m->g.adain_modules[i].second;
        if (max_batch) *max_batch = m->max_batch;
    });
}

extern "C" int rave_model_adain_get(rave_model* h, int i, float* stats, float* counters) {
    return guarded([&] {
        Model* m = model_of(h);
        if (i < 0 || i >= (int)m->g.adain_modules.size()) fail(RAVE_ERR_ARG, "AdaIN index out of range");
        RAVE_HIP_OR_THROW(hipDeviceSynchronize());
        const int64_t n = 4LL * m->max_batch * m->g.adain_modules[i].second;
        if (stats) RAVE_HIP_OR_THROW(hipMemcpy(stats, m->ad_stats + m->ad_off[i], n * 4, hipMemcpyDeviceToHost));
        if (counters) RAVE_HIP_OR_THROW(hipMemcpy(counters, m->ad_counters + 2 * i, 8, hipMemcpyDeviceToHost));
    });
}

extern "C" int rave_model_adain_set(rave_model* h, int i, const float* stats, const float* counters) {
    return guarded([&] {
        Model* m = model_of(h);
        if (i < 0 || i >= (int)m->g.adain_modules.size()) fail(RAVE_ERR_ARG, "AdaIN index out of range");
        RAVE_HIP_OR_THROW(hipDeviceSynchronize());
        const int64_t n = 4LL * m->max_batch * m->g.adain_modules[i].second;
        if (stats) RAVE_HIP_OR_THROW(hipMemcpy(m->ad_stats + m->ad_off[i], stats, n * 4, hipMemcpyHostToDevice));
        if (counters) RAVE_HIP_OR_THROW(hipMemcpy(m->ad_counters + 2 * i, counters, 8, hipMemcpyHostToDevice));
        if (stats || counters) m->touched = true;
    });
}

// ------------------------------------------------------------------ tuning
extern "C" int rave_model_tuning_get(const rave_model* h, char* buf, int cap) {
    std::string text;
    int rc = guarded([&] {
        const Model* m = model_of(const_cast<rave_model*>(h));
        std::ostringstream os;
        os.precision(9);
        for (auto& kv : m->tuned) os << kv.first << ' ' << kv.second.first << ' ' << kv.second.second << '\n';
        text = os.str();
    });
    if (rc != RAVE_OK) return rc;
    if (buf && cap > 0) {
        std::strncpy(buf, text.c_str(), (size_t)cap - 1);
        buf[cap - 1] = 0;
    }
    return (int)text.size() + 1;
}

extern "C" int rave_model_tuning_set(rave_model* h, const char* text) {
    return guarded([&] {
        Model* m = model_of(h);
        if (!text) fail(RAVE_ERR_ARG, "null tuning text");
        std::istringstream is(text);
        std::string key;
        int64_t choice;
        double ms;
        while (is >> key >> choice >> ms) m->tuned[key] = {choice, ms};
    });
}

// ------------------------------------------------------------------ measurement
extern "C" int rave_model_plan_ops(rave_model* h, int which, int batch, int t, rave_op_info* out, int cap) {
    int n = 0;
    int rc = guarded([&] {
        Model* m = model_of(h);
        Plan& p = m->plan_of(which, batch, t);
        n = (int)p.ops.size();
        for (int i = 0; i < n && i < cap && out; ++i) {
            rave_op_info& o = out[i];
            o.kind = p.ops[i].kind;
            o.precision = p.ops[i].prec;
            o.flops = p.ops[i].flops;
            o.bytes = p.ops[i].bytes;
            std::strncpy(o.label, p.ops[i].label.c_str(), sizeof(o.label) - 1);
            o.label[sizeof(o.label) - 1] = 0;
        }
    });
    return rc == RAVE_OK ? n : rc;
}

extern "C" int rave_model_profile(rave_model* h, int which, int batch, int t, int runs) {
    return guarded([&] {
        Model* m = model_of(h);
        check_rc(rave_plan_profile(m->plan_of(which, batch, t).handle, runs), "plan_profile");
    });
}

extern "C" int rave_model_op_times(rave_model* h, int which, int batch, int t, float* ms, int n) {
    int runs = 0;
    int rc = guarded([&] {
        Model* m = model_of(h);
        runs = rave_plan_op_times(m->plan_of(which, batch, t).handle, ms, n);
        if (runs < 0) fail(runs, std::string("op_times: ") + rave_last_error());
    });
    return rc == RAVE_OK ? runs : rc;
}


// =================================================================== streaming
// cached_conv's streaming mode (third-party cached-conv>=2.5.0, selected by
// cc.use_cached_conv(True), scripts/export.py:543) restated on the same
// kernels, for causal and centred (non-causal) padding alike:
//   * CachedConv1d with padding (l, r) prepends a cache of the last l + r
//     input samples (CachedPadding1d(l + r)) after a stride_delay crop-pad,
//     then convolves with padding 0: it is a conv over the persistent buffer
//     [history | block] read from history offset l + r + stride_delay.  Its
//     output lags the offline (zero-padded) conv by (r + stride_delay) / stride
//     frames -- 0 in causal mode.  After each block the newest `history`
//     columns move to the front (one batched SHIFT_HISTORY launch).  Cached
//     values are pre-activation (the activation is the conv prologue; act(0)
//     = 0 keeps the zero start state identical);
//   * Residual = AlignBranches(unit, Identity, delays=[d, 0]) (rave/blocks.py:
//     32-46): the identity branch is delayed by the unit's cumulative delay d
//     (its k3 conv's r), i.e. the residual add reads the unit's input buffer d
//     columns back;
//   * CachedConvTranspose1d (overlap-add of a 2*(r//2) cache) is the polyphase
//     2-tap conv with one input history column and no output crop; it lags by
//     r//2 output samples in both padding modes;
//   * CachedPQMF: analysis keeps taps-1 audio samples, synthesis taps-1 frames
//     (its conv padding (256,256)/(16,16) centred, (512,0)/(32,0) causal: the
//     same l + r either way);
//   * NoiseGeneratorV2's convs (padding (r, 0), stride r) keep r samples; its
//     filter stage is per noise frame, so it streams as is, into a buffer with
//     the synthesis history so the noise lines up with the waveform bands as
//     the reference's per-call tensors do;
//   * AdaIN runs on the block's columns (its statistics are per call, as the
//     reference computes them on each streamed chunk), in place, so the history
//     holds the normalised values the cached conv saw;
//   * discrete configs (DiscreteScriptedRAVE, scripts/export.py:503-517): the
//     encoder plan ends with rvq.encode of the block's frames, the decoder plan
//     starts with rvq.decode (clamped) + the speaker channels.
namespace rave {

Stream::~Stream() {
    if (enc_exec) (void)hipGraphExecDestroy(enc_exec);
    if (dec_exec) (void)hipGraphExecDestroy(dec_exec);
    if (enc_graph) (void)hipGraphDestroy(enc_graph);
    if (dec_graph) (void)hipGraphDestroy(dec_graph);
    if (cap) (void)hipStreamDestroy(cap);
    if (stage) (void)hipFree(stage);
}

// history columns the cached form of a conv reads before the block
static int stream_need(const Node& n) {
    if (n.transposed) return 1;
    return n.pad_l + n.pad_r + n.stride_delay();
}

static void tensor_sizes(const std::vector<const Node*>& nodes, std::map<std::string, std::pair<int, int>>& sizes) {
    for (const Node* n : nodes) {
        const int t_in = sizes.at(n->src).second;
        sizes[n->dst] = {n->c_out, n->transposed ? t_in * n->stride : t_in / n->stride};
    }
}

static std::map<std::string, StreamBuf> stream_buffers(Plan& p, const std::vector<const Node*>& nodes, int B,
                                                       const std::map<std::string, std::pair<int, int>>& sizes,
                                                       std::map<std::string, int> need) {
    for (const Node* n : nodes) {
        need[n->src] = std::max(need[n->src], stream_need(*n));
        if (!n->residual.empty()) need[n->residual] = std::max(need[n->residual], n->res_delay);
    }
    std::map<std::string, StreamBuf> bufs;
    for (auto& kv : sizes) {
        StreamBuf b;
        b.c = kv.second.first;
        b.t = kv.second.second;
        b.h = need.count(kv.first) ? need[kv.first] : 0;
        const int64_t width = b.h + b.t;
        b.v = ws_view(p.ws.alloc((int64_t)B * b.c * width), (int64_t)b.c * width, width);
        bufs[kv.first] = b;
    }
    return bufs;
}

static void conv_stream(Model* m, Plan& p, const Node& n, int B, std::map<std::string, StreamBuf>& bufs,
                        std::vector<int>& adain_ops) {
    const StreamBuf& src = bufs.at(n.src);
    const StreamBuf& dst = bufs.at(n.dst);
    const int need = stream_need(n);
    const int sd = n.stride_delay();
    if (!n.adain.empty() && !m->ad_index.empty()) {
        adain_ops.push_back((int)p.ops.size());
        m->adain_op(p, n.adain, B, n.c_in, src.t, src.v.at(src.h));
    }
    const View x = src.v.at(src.h - need);
    const View y = dst.v.p.kind == PRef::WS ? dst.v.at(dst.h) : dst.v;
    View res;
    const bool has_res = !n.residual.empty();
    if (has_res) {
        const StreamBuf& rb = bufs.at(n.residual);
        res = rb.v.at(rb.h - n.res_delay);    // AlignBranches: the identity branch, delayed
    }
    rave_conv1d_args a{};
    a.c_in = n.c_in;
    a.c_out = n.c_out;
    a.kernel = n.kernel;
    a.stride = n.stride;
    a.dilation = n.dilation;
    a.pad_left = n.transposed ? 1 : 0;
    a.transposed = n.transposed;
    a.out_shift = 0;
    a.act = n.act;
    a.leaky_slope = m->cfg.leaky_slope;
    a.batch = B;
    a.t_in = need - sd + src.t;       // [cache l+r | block delayed by sd]
    a.t_out = dst.t;
    a.x_sb = x.sb;
    a.x_sc = x.sc;
    a.y_sb = y.sb;
    a.y_sc = y.sc;
    a.r_sb = has_res ? res.sb : 0;
    a.r_sc = has_res ? res.sc : 0;
    // the fp32 ring kernels read 16-byte row pieces: workspace rows whose stride
    // and start (the history offset) are multiples of 4 floats, t_in % 4 == 0
    const bool vec_rows = x.p.kind == PRef::WS && x.sc % 4 == 0 && x.sb % 4 == 0 && x.p.off % 16 == 0 &&
                          a.t_in % 4 == 0;
    const auto pc = m->conv_launch(n, a, n.transposed, false, vec_rows);
    a.precision = pc.first;
    a.config = pc.second;
    auto& pack = n.transposed ? m->w_pack_stream : m->w_pack;   // ConvTranspose: the cached (out_shift 0) form
    rave_conv1d_args q = a;
    q.x = q.alpha = (const float*)m->arena;
    q.y = (float*)m->arena;
    q.residual = has_res ? (const float*)m->arena : nullptr;
    q.weight = m->aptr(pack.at({n.name, pc.first}));
    const int64_t nsk = rave_conv1d_workspace(&q);
    if (nsk < 0) fail(RAVE_ERR_ARG, "conv " + n.name + ": workspace query failed: " + rave_last_error());
    PlanOp& o = p.add(RAVE_OP_CONV, a, n.name);
    rave_conv1d_args& A = *reinterpret_cast<rave_conv1d_args*>(o.op.u.raw);
    View wv = m->arena_view(pack.at({n.name, pc.first}));
    View bv = n.bias ? m->arena_view(m->bias_off.at(n.name)) : View{};
    View av = n.act == RAVE_ACT_SNAKE ? m->arena_view(m->alpha_off.at(n.alpha)) : View{};
    View sk = p.splitk(nsk);
    p.bind(o, A, A.x, &x);
    p.bind(o, A, A.y, &y);
    p.bind(o, A, A.residual, has_res ? &res : nullptr);
    p.bind(o, A, A.weight, &wv);
    p.bind(o, A, A.bias, n.bias ? &bv : nullptr);
    p.bind(o, A, A.alpha, n.act == RAVE_ACT_SNAKE ? &av : nullptr);
    p.bind(o, A, A.partial, nsk > 0 ? &sk : nullptr);
    o.prec = pc.first;
}

// The cached conv sequence of one stream plan.  A Residual(DilatedUnit) whose
// fused kernel is timed faster than its two convs (Model::fuse_unit, the
// one-shot decision at the block's length) runs as ONE cached unit launch: the
// k=3 window reads the input's history (pad_left 0, x_len = need + T) and the
// residual is the same buffer shifted by need - delay (AlignBranches,
// rave/blocks.py:32-46); the intermediate tensor is never written.
// RAVE_STREAM_UNITS=0 keeps every conv separate (A/B).
static void stream_convs(Model* m, Plan& p, const std::vector<const Node*>& nodes, int B,
                         std::map<std::string, StreamBuf>& bufs, std::vector<int>& adain_ops) {
    static const bool units_on = [] {
        const char* e = std::getenv("RAVE_STREAM_UNITS");
        return !(e && e[0] == '0');
    }();
    std::map<std::string, const Node*> fused;
    if (m->cfg.fuse_units && units_on)
        for (auto& pr : m->unit_pairs(nodes))
            if (m->unit_ok.count(pr.first->name) && pr.second->adain.empty()) fused[pr.first->name] = pr.second;
    std::set<std::string> skip;
    for (const Node* n : nodes) {
        if (skip.count(n->name)) continue;
        auto fu = fused.find(n->name);
        const StreamBuf& src = bufs.at(n->src);
        if (fu != fused.end() && m->fuse_unit(*n, *fu->second, B, src.t)) {
            const Node& k1 = *fu->second;
            skip.insert(k1.name);
            if (!n->adain.empty() && !m->ad_index.empty()) {
                adain_ops.push_back((int)p.ops.size());
                m->adain_op(p, n->adain, B, n->c_in, src.t, src.v.at(src.h));
            }
            const int need = stream_need(*n);
            const StreamBuf& dst = bufs.at(k1.dst);
            const View y = dst.v.p.kind == PRef::WS ? dst.v.at(dst.h) : dst.v;
            m->unit_op(p, *n, k1, B, src.t, src.v.at(src.h - need), y, need + src.t, need - k1.res_delay);
            continue;
        }
        conv_stream(m, p, *n, B, bufs, adain_ops);
    }
}

static void shift_all(Plan& p, int B, const std::map<std::string, StreamBuf>& bufs) {
    for (auto& kv : bufs) {
        const StreamBuf& b = kv.second;
        if (b.h <= 0 || b.v.p.kind != PRef::WS) continue;
        rave_shift_args s{};
        s.batch = B;
        s.channels = b.c;
        s.hist = b.h;
        s.t_new = b.t;
        s.sb = b.v.sb;
        s.sc = b.v.sc;
        PlanOp& o = p.add(RAVE_OP_SHIFT_HISTORY, s, "shift:" + kv.first);
        rave_shift_args& S = *reinterpret_cast<rave_shift_args*>(o.op.u.raw);
        p.bind(o, S, S.buf, &b.v);
    }
}

static void copy_op(Plan& p, int B, int C, int T, const View& x, const View& y) {
    rave_copy_args c{};
    c.batch = B;
    c.channels = C;
    c.t_len = T;
    c.x_sb = x.sb;
    c.x_sc = x.sc;
    c.y_sb = y.sb;
    c.y_sc = y.sc;
    PlanOp& o = p.add(RAVE_OP_COPY, c, "copy");
    rave_copy_args& A = *reinterpret_cast<rave_copy_args*>(o.op.u.raw);
    p.bind(o, A, A.x, &x);
    p.bind(o, A, A.y, &y);
}

// Samples by which the streamed decoder lags one-shot decoding: each cached
// conv adds (r + stride_delay) / stride frames at its output rate, each cached
// ConvTranspose1d multiplies the lag by its stride and adds r//2, the PQMF
// inverse conv adds its right padding (16 centred, 0 causal) in band frames.
static int decode_delay(const Model* m) {
    std::map<std::string, int> d{{"dec_in", 0}};
    for (const Node& n : m->g.decoder) {
        const int in = d.at(n.src);
        d[n.dst] = n.transposed ? in * n.stride + n.stride / 2 : (in + n.pad_r + n.stride_delay()) / n.stride;
    }
    return (d.at("wave") + get_padding(m->taps_s, 1, m->cfg.causal != 0).second) * m->cfg.n_band;
}

static void build_stream(Stream& s) {
    Model* m = s.m;
    const rave_model_config& cfg = m->cfg;
    const int B = s.B;
    // ------------------------------------------------------------ encoder
    if (!(s.flags & RAVE_STREAM_DECODE_ONLY)) {
        s.enc = std::make_unique<Plan>();
        Plan& p = *s.enc;
        std::vector<const Node*> nodes = ptrs_of(m->g.encoder);
        std::map<std::string, std::pair<int, int>> sizes{{"audio", {1, s.block}}, {"enc_in", {cfg.enc_bands, s.F}}};
        tensor_sizes(nodes, sizes);
        sizes.erase("latent");
        const int ha = m->taps_a - 1;
        s.enc_bufs = stream_buffers(p, nodes, B, sizes, {{"audio", ha}});
        const int zc = cfg.latent_size + cfg.speaker_size;
        StreamBuf lat;
        lat.v = s.codes ? ws_view(p.ws.alloc((int64_t)B * cfg.latent_size * s.Fz), (int64_t)cfg.latent_size * s.Fz, s.Fz)
                        : io_view(1, (int64_t)zc * s.Fz, s.Fz);
        lat.c = cfg.latent_size;
        lat.t = s.Fz;
        s.enc_bufs["latent"] = lat;
        const StreamBuf& a = s.enc_bufs.at("audio");
        copy_op(p, B, 1, s.block, io_view(0, s.block, s.block), a.v.at(a.h));
        const StreamBuf& e = s.enc_bufs.at("enc_in");
        m->analysis_op(p, B, s.block, a.v, e.v.at(e.h), cfg.enc_bands, 0, ha + s.block);
        stream_convs(m, p, nodes, B, s.enc_bufs, s.enc_adain);
        if (s.codes) m->rvq_encode_op(p, B, s.Fz, lat.v, io_view(1, 0, 0));
        else m->fill_speaker(p, B, s.Fz, io_view(1, (int64_t)zc * s.Fz, s.Fz).at((int64_t)cfg.latent_size * s.Fz));
        shift_all(p, B, s.enc_bufs);
        p.finalize(m->arena);
    }
    // ------------------------------------------------------------ decoder (+ noise synthesizer)
    if (!(s.flags & RAVE_STREAM_ENCODE_ONLY)) {
        s.dec = std::make_unique<Plan>();
        Plan& p = *s.dec;
        std::vector<const Node*> nodes = ptrs_of(m->g.decoder);
        for (const Node& n : m->g.noise) nodes.push_back(&n);
        std::map<std::string, std::pair<int, int>> sizes{{"dec_in", {m->dec_in, s.Fz}}};
        tensor_sizes(nodes, sizes);
        const int hw = m->taps_s - 1;
        std::map<std::string, int> need{{"wave", hw}};
        if (cfg.noise) {
            sizes["noise_sig"] = {cfg.n_band, s.F};
            need["noise_sig"] = hw;
        }
        s.dec_bufs = stream_buffers(p, nodes, B, sizes, need);
        const StreamBuf& z = s.dec_bufs.at("dec_in");
        if (s.codes) {
            m->rvq_decode_op(p, B, s.Fz, io_view(0, 0, 0), z.v.at(z.h));
            m->fill_speaker(p, B, s.Fz, z.v.at(z.h).at((int64_t)cfg.latent_size * z.v.sc));
        } else {
            copy_op(p, B, m->dec_in, s.Fz, io_view(0, (int64_t)m->dec_in * s.Fz, s.Fz), z.v.at(z.h));
        }
        stream_convs(m, p, nodes, B, s.dec_bufs, s.dec_adain);
        const StreamBuf& w = s.dec_bufs.at("wave");
        View noise_v;
        if (cfg.noise) {
            const StreamBuf& amp = s.dec_bufs.at("noise_amp");
            const StreamBuf& sig = s.dec_bufs.at("noise_sig");
            rave_noise_args a{};
            a.batch = B;
            a.frames = amp.t;
            a.n_band = cfg.n_band;
            a.noise_bands = cfg.noise_bands;
            a.target = m->noise_target;
            a.a_sb = amp.v.sb;
            a.a_sc = amp.v.sc;
            a.u_sb = (int64_t)amp.t * cfg.n_band * m->noise_target;
            a.y_sb = sig.v.sb;
            a.y_sc = sig.v.sc;
            PlanOp& o = p.add(RAVE_OP_NOISE, a, "noise_synth");
            rave_noise_args& N = *reinterpret_cast<rave_noise_args*>(o.op.u.raw);
            View av = amp.v.at(amp.h), u = io_view(2, 0, 0), yv = sig.v.at(sig.h);
            p.bind(o, N, N.amp, &av);
            p.bind(o, N, N.u, &u);
            p.bind(o, N, N.y, &yv);
            noise_v = sig.v;
        }
        m->synthesis_op(p, B, s.F, w.v, io_view(1, s.block, s.block), cfg.noise ? &noise_v : nullptr, 0, -hw,
                        hw + s.F);
        shift_all(p, B, s.dec_bufs);
        p.finalize(m->arena);
    }
    s.delay = decode_delay(m);
}

static int64_t noise_count(const Stream& s) {
    return s.m->cfg.noise ? (int64_t)s.B * (s.F / s.m->noise_target) * s.m->cfg.n_band * s.m->noise_target : 0;
}

// bytes of one block's encoder output / decoder input: latents (+ speaker) in
// floats, or int64 RVQ indices for a discrete config
static int64_t latent_bytes(const Stream& s, bool dec_side) {
    const rave_model_config& c = s.m->cfg;
    if (s.codes) return (int64_t)s.B * c.rvq_quantizers * s.Fz * 8;
    return (int64_t)s.B * (dec_side ? s.m->dec_in : c.latent_size + c.speaker_size) * s.Fz * 4;
}

// the plan's first op when it is the block's input copy into a history buffer
// whose rows the host can fill with one 2-D copy (graph mode, Stream::Direct)
static Stream::Direct direct_input(const Plan& p) {
    Stream::Direct d;
    static const bool on = [] {
        const char* e = std::getenv("RAVE_STREAM_DIRECT");
        return !(e && e[0] == '0');
    }();
    if (!on || p.ops.empty() || p.ops[0].kind != RAVE_OP_COPY) return d;
    rave_copy_args c;
    std::memcpy(&c, p.ops[0].op.u.raw, sizeof(c));
    const int yoff = (int)offsetof(rave_copy_args, y);
    for (auto& fp : p.ops[0].ptrs)
        if (fp.first == yoff && fp.second.kind == PRef::WS) d.dst = (float*)((char*)p.ws_dev + fp.second.off);
    if (!d.dst) return Stream::Direct{};
    if (c.channels == 1) {
        d.pitch = c.y_sb;
        d.rows = c.batch;
    } else if (c.y_sb == (int64_t)c.channels * c.y_sc) {
        d.pitch = c.y_sc;
        d.rows = (int64_t)c.batch * c.channels;
    } else {
        return Stream::Direct{};
    }
    d.width = c.t_len;
    return d;
}

// the encoder plan's speaker fill when it writes only the staged latents (slot
// 1), which nothing else in the graph touches: outside the graph, run once per
// speaker (RAVE_STREAM_SPK_ONCE=0 keeps it in the graph)
static int speaker_fill_op(const Stream& s) {
    static const bool on = [] {
        const char* e = std::getenv("RAVE_STREAM_SPK_ONCE");
        return !(e && e[0] == '0');
    }();
    if (!on || s.codes) return -1;
    const Plan& p = *s.enc;
    int found = -1;
    for (int i = 0; i < (int)p.ops.size(); ++i) {
        if (p.ops[i].kind != RAVE_OP_FILL) continue;
        if (found >= 0) return -1;                   // one fill only
        const int yoff = (int)offsetof(rave_fill_args, y);
        for (auto& fp : p.ops[i].ptrs)
            if (fp.first == yoff && fp.second.kind == PRef::IO && fp.second.slot == 1) found = i;
        if (found != i) return -1;
    }
    return found;
}

static void capture(Stream& s, Plan& p, void* const* slots, int n, hipGraph_t& g, hipGraphExec_t& e,
                    int first = 0, int skip = -1) {
    if (e) (void)hipGraphExecDestroy(e);
    if (g) (void)hipGraphDestroy(g);
    e = nullptr;
    g = nullptr;
    RAVE_HIP_OR_THROW(hipStreamBeginCapture(s.cap, hipStreamCaptureModeThreadLocal));
    const int rc = plan_run_from(p.handle, slots, n, s.cap, first, -1, skip);
    hipGraph_t graph = nullptr;
    const hipError_t ec = hipStreamEndCapture(s.cap, &graph);
    if (rc != RAVE_OK) {
        if (graph) (void)hipGraphDestroy(graph);
        fail(rc, std::string("stream capture: ") + rave_last_error());
    }
    RAVE_HIP_OR_THROW(ec);
    g = graph;
    RAVE_HIP_OR_THROW(hipGraphInstantiate(&e, g, nullptr, nullptr, 0));
}

static void recapture(Stream& s) {
    if (s.has_enc()) {
        void* es[2] = {s.x_st, s.z_st};
        capture(s, *s.enc, es, 2, s.enc_graph, s.enc_exec, s.enc_in.dst ? 1 : 0, s.enc_fill);
    }
    if (s.has_dec()) {
        void* ds[3] = {s.zi_st, s.y_st, s.u_st ? (void*)s.u_st : (void*)s.y_st};
        capture(s, *s.dec, ds, 3, s.dec_graph, s.dec_exec, s.dec_in.dst ? 1 : 0);
    }
}

// AdaIN ops carry the learn mode and the first buffer row in their arguments:
// patch them when the model's flags or row0 have changed since the last block
// (and re-capture the graphs)
static void sync_adain(Stream& s) {
    Model* m = s.m;
    if (m->ad_index.empty()) return;
    const int mode = m->adain_mode();
    const int row0 = m->row0;
    if (mode == s.ad_mode && row0 == s.ad_row0) return;
    if (row0 + s.B > m->max_batch)
        fail(RAVE_ERR_ARG, "AdaIN statistics hold " + std::to_string(m->max_batch) + " batch rows; stream batch " +
                               std::to_string(s.B) + " at row " + std::to_string(row0) + " exceeds them");
    const int off_mode = (int)offsetof(rave_adain_args, mode);
    const int off_row0 = (int)offsetof(rave_adain_args, row0);
    for (auto* pl : {&s.enc, &s.dec}) {
        if (!*pl) continue;
        for (int i : (pl == &s.enc ? s.enc_adain : s.dec_adain)) {
            check_rc(plan_patch((*pl)->handle, i, off_mode, &mode, 4), "plan_patch");
            check_rc(plan_patch((*pl)->handle, i, off_row0, &row0, 4), "plan_patch");
        }
    }
    s.ad_mode = mode;
    s.ad_row0 = row0;
    if (s.flags & RAVE_STREAM_GRAPH) recapture(s);
}

}  // namespace rave

struct rave_stream {
    std::unique_ptr<rave::Stream> s;
};

static rave::Stream* stream_of(rave_stream* h) {
    if (!h || !h->s) rave::fail(RAVE_ERR_STATE, "null stream");
    return h->s.get();
}

extern "C" int rave_stream_create(rave_model* mh, int batch, int block, int flags, rave_stream** out) {
    return guarded([&] {
        Model* m = model_of(mh);
        if (!out) fail(RAVE_ERR_ARG, "null output");
        *out = nullptr;
        if (flags & ~(RAVE_STREAM_GRAPH | RAVE_STREAM_ENCODE_ONLY | RAVE_STREAM_DECODE_ONLY))
            fail(RAVE_ERR_ARG, "unknown stream flags");
        if ((flags & RAVE_STREAM_ENCODE_ONLY) && (flags & RAVE_STREAM_DECODE_ONLY))
            fail(RAVE_ERR_ARG, "RAVE_STREAM_ENCODE_ONLY and RAVE_STREAM_DECODE_ONLY exclude each other");
        if (batch <= 0 || block <= 0 || block % m->hop)
            fail(RAVE_ERR_ARG, "block must be a positive multiple of " + std::to_string(m->hop));
        check_noise_frames(m, block / m->hop);
        if (!m->ad_index.empty() && m->row0 + batch > m->max_batch)
            fail(RAVE_ERR_ARG, "AdaIN statistics hold " + std::to_string(m->max_batch) + " batch rows");
        auto h = std::make_unique<rave_stream>();
        h->s = std::make_unique<Stream>();
        Stream& s = *h->s;
        s.m = m;
        s.B = batch;
        s.block = block;
        s.flags = flags;
        s.codes = m->cfg.rvq_quantizers > 0;
        s.Fz = block / m->hop;
        s.F = block / m->cfg.n_band;
        s.ad_mode = m->adain_mode();
        s.ad_row0 = m->row0;
        m->cur_stream = nullptr;
        build_stream(s);
        // staging buffers (graph mode) and the capture stream
        const int64_t nx = (int64_t)batch * block, nz = (latent_bytes(s, false) + 3) / 4,
                      nzi = (latent_bytes(s, true) + 3) / 4, nu = noise_count(s);
        const int64_t total = nx + nz + nzi + nx + std::max<int64_t>(nu, 1) + 5 * 64;
        RAVE_HIP_OR_THROW(hipMalloc(&s.stage, (size_t)total * 4));
        RAVE_HIP_OR_THROW(hipMemset(s.stage, 0, (size_t)total * 4));
        int64_t o = 0;
        auto take = [&](int64_t n) {
            float* p = s.stage + o;
            o += Workspace::round(std::max<int64_t>(n, 1));
            return p;
        };
        s.x_st = take(nx);
        s.z_st = take(nz);
        s.zi_st = take(nzi);
        s.y_st = take(nx);
        s.u_st = nu > 0 ? take(nu) : nullptr;
        // one warm run of each plan (kernel attributes are set on first launch,
        // outside any capture), then the zero start state.  The warm run must
        // not leave a trace in the model's shared AdaIN statistics (a learning
        // mode would fold the all-zero staging block into them): they are
        // saved and restored around it.
        {
            float* ad_save = nullptr;
            int64_t ad_n = 0;
            const size_t na = m->g.adain_modules.size();
            if (na) {
                for (size_t i = 0; i < na; ++i) ad_n += 4LL * m->max_batch * m->g.adain_modules[i].second;
                RAVE_HIP_OR_THROW(hipDeviceSynchronize());
                RAVE_HIP_OR_THROW(hipMalloc(&ad_save, (size_t)(ad_n + 3 * na) * 4));
                RAVE_HIP_OR_THROW(hipMemcpy(ad_save, m->ad_stats, (size_t)ad_n * 4, hipMemcpyDeviceToDevice));
                RAVE_HIP_OR_THROW(hipMemcpy(ad_save + ad_n, m->ad_counters, na * 2 * 4, hipMemcpyDeviceToDevice));
                RAVE_HIP_OR_THROW(hipMemcpy(ad_save + ad_n + 2 * na, m->ad_tickets, na * 4, hipMemcpyDeviceToDevice));
            }
            if (s.has_enc()) {
                void* es[2] = {s.x_st, s.z_st};
                s.enc->run(es, 2, nullptr);
            }
            if (s.has_dec()) {
                void* ds[3] = {s.zi_st, s.y_st, s.u_st ? (void*)s.u_st : (void*)s.y_st};
                s.dec->run(ds, 3, nullptr);
            }
            RAVE_HIP_OR_THROW(hipDeviceSynchronize());
            if (ad_save) {
                RAVE_HIP_OR_THROW(hipMemcpy(m->ad_stats, ad_save, (size_t)ad_n * 4, hipMemcpyDeviceToDevice));
                RAVE_HIP_OR_THROW(hipMemcpy(m->ad_counters, ad_save + ad_n, na * 2 * 4, hipMemcpyDeviceToDevice));
                RAVE_HIP_OR_THROW(hipMemcpy(m->ad_tickets, ad_save + ad_n + 2 * na, na * 4, hipMemcpyDeviceToDevice));
                RAVE_HIP_OR_THROW(hipFree(ad_save));
            }
            if (s.has_enc()) RAVE_HIP_OR_THROW(hipMemset(s.enc->ws_dev, 0, (size_t)s.enc->ws_floats * 4));
            if (s.has_dec()) RAVE_HIP_OR_THROW(hipMemset(s.dec->ws_dev, 0, (size_t)s.dec->ws_floats * 4));
        }
        if (flags & RAVE_STREAM_GRAPH) {
            if (s.has_enc()) {
                s.enc_in = direct_input(*s.enc);
                s.enc_fill = speaker_fill_op(s);
            }
            if (s.has_dec()) s.dec_in = direct_input(*s.dec);
            RAVE_HIP_OR_THROW(hipStreamCreateWithFlags(&s.cap, hipStreamNonBlocking));
            recapture(s);
        }
        *out = h.release();
    });
}

extern "C" int rave_stream_destroy(rave_stream* s) {
    delete s;
    return RAVE_OK;
}

extern "C" int rave_stream_reset(rave_stream* h, void* stream) {
    return guarded([&] {
        Stream* s = stream_of(h);
        if (s->has_enc())
            RAVE_HIP_OR_THROW(hipMemsetAsync(s->enc->ws_dev, 0, (size_t)s->enc->ws_floats * 4, as_stream(stream)));
        if (s->has_dec())
            RAVE_HIP_OR_THROW(hipMemsetAsync(s->dec->ws_dev, 0, (size_t)s->dec->ws_floats * 4, as_stream(stream)));
    });
}

namespace rave {
// graph mode: the block's input rows straight into the history buffer (Stream::Direct)
static void direct_copy(const Stream::Direct& d, const void* src, hipStream_t st) {
    RAVE_HIP_OR_THROW(hipMemcpy2DAsync(d.dst, (size_t)d.pitch * 4, src, (size_t)d.width * 4, (size_t)d.width * 4,
                                       (size_t)d.rows, hipMemcpyDeviceToDevice, st));
}

// one encoder block: audio (B, 1, block) -> latents or indices (latent_bytes)
static void stream_enc(Stream* s, const void* x, void* out, hipStream_t st) {
    if (!s->has_enc()) fail(RAVE_ERR_STATE, "stream was created RAVE_STREAM_DECODE_ONLY");
    sync_adain(*s);
    if (s->flags & RAVE_STREAM_GRAPH) {
        if (s->enc_in.dst) direct_copy(s->enc_in, x, st);
        else RAVE_HIP_OR_THROW(hipMemcpyAsync(s->x_st, x, (size_t)s->B * s->block * 4, hipMemcpyDeviceToDevice, st));
        if (s->enc_fill >= 0 && s->spk_seen != s->m->spk_version) {
            void* es[2] = {s->x_st, s->z_st};
            check_rc(plan_run_from(s->enc->handle, es, 2, st, s->enc_fill, s->enc_fill + 1), "speaker fill");
            s->spk_seen = s->m->spk_version;
        }
        RAVE_HIP_OR_THROW(hipGraphLaunch(s->enc_exec, st));
        RAVE_HIP_OR_THROW(hipMemcpyAsync(out, s->z_st, (size_t)latent_bytes(*s, false), hipMemcpyDeviceToDevice, st));
    } else {
        void* slots[2] = {(void*)x, out};
        s->enc->run(slots, 2, st);
    }
}

// one decoder block: latents or indices -> audio (B, 1, block)
static void stream_dec(Stream* s, const void* in, float* y, const float* noise_u, hipStream_t st) {
    if (!s->has_dec()) fail(RAVE_ERR_STATE, "stream was created RAVE_STREAM_ENCODE_ONLY");
    sync_adain(*s);
    Model* m = s->m;
    const int64_t nu = noise_count(*s);
    const float* u = nullptr;
    if (nu > 0) {
        if (noise_u && !(s->flags & RAVE_STREAM_GRAPH)) {
            u = noise_u;
        } else if (noise_u) {
            RAVE_HIP_OR_THROW(hipMemcpyAsync(s->u_st, noise_u, (size_t)nu * 4, hipMemcpyDeviceToDevice, st));
            u = s->u_st;
        } else {
            check_rc(rave_fill_uniform(s->u_st, nu, 0x13198A2E03707344ull + 0x9E3779B97F4A7C15ull * ++m->noise_calls,
                                       0.f, 1.f, st),
                     "noise draw");
            u = s->u_st;
        }
    }
    if (s->flags & RAVE_STREAM_GRAPH) {
        if (s->dec_in.dst) direct_copy(s->dec_in, in, st);
        else RAVE_HIP_OR_THROW(hipMemcpyAsync(s->zi_st, in, (size_t)latent_bytes(*s, true), hipMemcpyDeviceToDevice, st));
        RAVE_HIP_OR_THROW(hipGraphLaunch(s->dec_exec, st));
        RAVE_HIP_OR_THROW(hipMemcpyAsync(y, s->y_st, (size_t)s->B * s->block * 4, hipMemcpyDeviceToDevice, st));
    } else {
        void* slots[3] = {(void*)in, (void*)y, (void*)(u ? u : y)};
        s->dec->run(slots, 3, st);
    }
}
}  // namespace rave

extern "C" int rave_stream_encode(rave_stream* h, const float* x, float* z, void* stream) {
    return guarded([&] {
        Stream* s = stream_of(h);
        s->m->coop_check();
        if (!x || !z) fail(RAVE_ERR_ARG, "stream encode: null tensor");
        if (s->codes) fail(RAVE_ERR_ARG, "discrete config: stream with rave_stream_encode_codes");
        stream_enc(s, x, z, as_stream(stream));
    });
}

extern "C" int rave_stream_decode(rave_stream* h, const float* z, float* y, const float* noise_u, void* stream) {
    return guarded([&] {
        Stream* s = stream_of(h);
        s->m->coop_check();
        if (!z || !y) fail(RAVE_ERR_ARG, "stream decode: null tensor");
        if (s->codes) fail(RAVE_ERR_ARG, "discrete config: stream with rave_stream_decode_codes");
        stream_dec(s, z, y, noise_u, as_stream(stream));
    });
}

extern "C" int rave_stream_encode_codes(rave_stream* h, const float* x, int64_t* idx, void* stream) {
    return guarded([&] {
        Stream* s = stream_of(h);
        s->m->coop_check();
        if (!x || !idx) fail(RAVE_ERR_ARG, "stream encode_codes: null tensor");
        if (!s->codes) fail(RAVE_ERR_ARG, "encode_codes needs a discrete (RVQ) config");
        stream_enc(s, x, idx, as_stream(stream));
    });
}

extern "C" int rave_stream_decode_codes(rave_stream* h, const int64_t* idx, float* y, const float* noise_u,
                                        void* stream) {
    return guarded([&] {
        Stream* s = stream_of(h);
        s->m->coop_check();
        if (!idx || !y) fail(RAVE_ERR_ARG, "stream decode_codes: null tensor");
        if (!s->codes) fail(RAVE_ERR_ARG, "decode_codes needs a discrete (RVQ) config");
        stream_dec(s, idx, y, noise_u, as_stream(stream));
    });
}

// kernel launches of one block: the kernel nodes of the captured graph (graph
// mode; the two staging copies around a replay are not counted) or the plan's
// ops (eager mode); which 0 = encode, 1 = decode
extern "C" int rave_stream_launches(const rave_stream* h, int which) {
    int n = 0;
    int rc = guarded([&] {
        Stream* s = stream_of(const_cast<rave_stream*>(h));
        if (which != 0 && which != 1) fail(RAVE_ERR_ARG, "which must be 0 (encode) or 1 (decode)");
        if (which == 0 ? !s->has_enc() : !s->has_dec()) fail(RAVE_ERR_STATE, "stream has no such direction");
        hipGraph_t g = which == 0 ? s->enc_graph : s->dec_graph;
        if (!g) {
            // eager: the plan's ops, with a run of history shifts going out as one
            // launch per rave::kShiftBatch (rave_plan_run, capi.cpp)
            const auto& ops = (which == 0 ? s->enc : s->dec)->ops;
            for (size_t i = 0; i < ops.size();) {
                int run = 0;
                while (i + run < ops.size() && run < rave::kShiftBatch && ops[i + run].op.kind == RAVE_OP_SHIFT_HISTORY) ++run;
                ++n;
                i += run > 0 ? run : 1;
            }
            return;
        }
        size_t cnt = 0;
        RAVE_HIP_OR_THROW(hipGraphGetNodes(g, nullptr, &cnt));
        std::vector<hipGraphNode_t> nodes(cnt);
        RAVE_HIP_OR_THROW(hipGraphGetNodes(g, nodes.data(), &cnt));
        for (size_t i = 0; i < cnt; ++i) {
            hipGraphNodeType t;
            RAVE_HIP_OR_THROW(hipGraphNodeGetType(nodes[i], &t));
            n += t == hipGraphNodeTypeKernel ? 1 : 0;
        }
    });
    return rc == RAVE_OK ? n : rc;
}

extern "C" int rave_stream_delay(const rave_stream* h) {
    int d = 0;
    int rc = guarded([&] { d = stream_of(const_cast<rave_stream*>(h))->delay; });
    return rc == RAVE_OK ? d : rc;
}
