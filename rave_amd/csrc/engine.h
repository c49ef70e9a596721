// Model engine internals (include/rave_amd.h "model engine"): the RAVE module
// graph, launch plans with liveness-planned workspaces, the per-op autotuner
// and the streaming state.  Host C++ only; every kernel is reached through the
// C-ABI entry points of the other translation units.
#pragma once

#include <algorithm>
#include <cstring>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <utility>
#include <vector>

#include "common.h"

namespace rave {

// Status carried out of the engine by exception and turned into a return code
// (and rave_last_error text) at the C boundary.
struct EngineError {
    int code;
    std::string msg;
};
[[noreturn]] inline void fail(int code, const std::string& msg) { throw EngineError{code, msg}; }
inline void check_rc(int rc, const std::string& what) {
    if (rc != RAVE_OK) fail(rc, what + ": " + rave_last_error());
}
#define RAVE_HIP_OR_THROW(expr)                                                              \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess) ::rave::fail(RAVE_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

int plan_patch(rave_plan* plan, int op, int offset, const void* data, int n);   // capi.cpp
int plan_run_from(rave_plan* plan, void* const* slots, int n_slots, void* stream, int first, int end = -1,
                  int skip = -1);   // capi.cpp

// ------------------------------------------------------------------ graph
// One convolution (or transposed convolution) of the reference module tree,
// with the activation module before it fused as a prologue and an optional
// Residual add on its output.  `name` is the reference state_dict prefix.
struct Node {
    std::string name;
    int c_in = 0, c_out = 0, kernel = 1, stride = 1, dilation = 1, pad_l = 0, pad_r = 0;
    bool transposed = false, weight_norm = true, bias = true;
    int act = RAVE_ACT_NONE;
    std::string alpha;          // Snake alpha parameter (act == SNAKE)
    std::string src, dst;       // tensor ids
    std::string residual;       // tensor id added to the output ("" = none)
    std::string adain;          // AdaIN module applied to the input first ("" = none)
    // cached (streaming) mode: AlignBranches delay of the residual identity
    // branch (rave/blocks.py:36-41: the unit's cumulative_delay, i.e. its k3
    // conv's right padding; 0 in causal mode)
    int res_delay = 0;
    int out_len(int t_in) const;
    // cached_conv's CachedConv1d crop-pad that makes (r + cd) a multiple of the
    // stride (cd = 0: no conv of these graphs passes cumulative_delay)
    int stride_delay() const { return transposed ? 0 : (stride - (pad_r % stride)) % stride; }
};

struct Graph {
    std::vector<Node> encoder, decoder, noise;
    std::vector<std::pair<std::string, int>> adain_modules;   // (prefix, channels)
    std::vector<const Node*> convs() const;
};

void build_graph(const rave_model_config& c, Graph& g);
// (name, shape) of every parameter the config needs, in graph order; pqmf.hk last
// with an empty shape (its length is the checkpoint's).
std::vector<std::pair<std::string, std::vector<int64_t>>> param_table(const rave_model_config& c);
std::pair<int, int> get_padding(int k, int dilation, bool causal);

// ------------------------------------------------------------------ plans
// A pointer inside an op's argument struct, resolved when the plan is finalised.
struct PRef {
    enum Kind { NONE, WS, ARENA, ABS, SPLITK, IO } kind = NONE;
    int64_t off = 0;   // bytes from the base (WS / ARENA / IO), absolute address (ABS)
    int slot = 0;      // IO slot
};
struct View {
    PRef p;
    int64_t sb = 0, sc = 0;          // batch / channel strides, elements
    View at(int64_t elems, int elem_bytes = 4) const {
        View v = *this;
        v.p.off += elems * elem_bytes;
        return v;
    }
};
inline View ws_view(int64_t off_floats, int64_t sb, int64_t sc) {
    View v;
    v.p.kind = PRef::WS;
    v.p.off = off_floats * 4;
    v.sb = sb;
    v.sc = sc;
    return v;
}
inline View io_view(int slot, int64_t sb, int64_t sc) {
    View v;
    v.p.kind = PRef::IO;
    v.p.slot = slot;
    v.sb = sb;
    v.sc = sc;
    return v;
}
inline View abs_view(const void* p) {
    View v;
    v.p.kind = PRef::ABS;
    v.p.off = (int64_t)(uintptr_t)p;
    return v;
}

// First-fit allocator with liveness reuse (sizes in floats, 256-byte granules).
struct Workspace {
    std::vector<std::pair<int64_t, int64_t>> free_;
    int64_t top = 0;
    static int64_t round(int64_t n) { return (n + 63) / 64 * 64; }
    int64_t alloc(int64_t n);
    void release(int64_t off, int64_t n);
};

struct PlanOp {
    int kind = 0;
    rave_plan_op op{};
    std::vector<std::pair<int, PRef>> ptrs;   // (byte offset of the pointer field in op.u, ref)
    std::string label;
    double flops = 0, bytes = 0;
    int prec = -1;
};

struct Plan {
    std::vector<PlanOp> ops;
    Workspace ws;
    int64_t splitk_max = 0;          // floats
    void* ws_dev = nullptr;
    int64_t ws_floats = 0;
    rave_plan* handle = nullptr;
    ~Plan();
    template <typename A>
    PlanOp& add(int kind, const A& args, const std::string& label) {
        static_assert(sizeof(A) <= RAVE_OP_PAYLOAD, "payload");
        PlanOp o;
        o.kind = kind;
        o.op.kind = kind;
        std::memcpy(o.op.u.raw, &args, sizeof(A));
        o.label = label;
        ops.push_back(o);
        return ops.back();
    }
    // bind pointer field `field` (address inside the args copy `base`) to view v
    template <typename A, typename F>
    void bind(PlanOp& o, const A& base, F* const& field, const View* v) {
        const int off = (int)((const char*)&field - (const char*)&base);
        if (v) o.ptrs.push_back({off, v->p});
        else o.ptrs.push_back({off, PRef{}});
    }
    View splitk(int64_t floats) {
        View v;
        if (floats <= 0) return v;
        splitk_max = std::max(splitk_max, floats);
        v.p.kind = PRef::SPLITK;
        return v;
    }
    // allocate the workspace, resolve pointers, create the executor plan
    void finalize(const void* arena);
    void run(void* const* slots, int n_slots, hipStream_t st);
};

struct Model;

// ------------------------------------------------------------------ streaming
struct StreamBuf {
    View v;          // the whole [history | block] buffer (workspace)
    int h = 0, t = 0, c = 0;
};

struct Stream {
    Model* m = nullptr;
    int B = 1, block = 0, Fz = 0, F = 0, flags = 0;
    bool codes = false;                            // discrete config: the plans end / start with RVQ
    std::unique_ptr<Plan> enc, dec;
    std::map<std::string, StreamBuf> enc_bufs, dec_bufs;
    // graph mode: staging buffers and captured executables
    float* stage = nullptr;
    float *x_st = nullptr, *z_st = nullptr, *zi_st = nullptr, *y_st = nullptr, *u_st = nullptr;
    hipGraphExec_t enc_exec = nullptr, dec_exec = nullptr;
    hipGraph_t enc_graph = nullptr, dec_graph = nullptr;
    hipStream_t cap = nullptr;
    // graph mode: the block's input goes straight into the history buffer's new
    // columns (a 2-D copy by the host call) instead of staging + the plan's copy
    // op, which the captured graph then skips (op 0): rows of `width` floats,
    // `rows` of them at `pitch` floats (RAVE_STREAM_DIRECT=0 keeps the staging)
    struct Direct {
        float* dst = nullptr;
        int64_t pitch = 0, rows = 0, width = 0;
    } enc_in, dec_in;
    // graph mode: the encoder plan's speaker fill (op index, -1: none) writes the
    // constant speaker channels of the staged latents; it runs outside the graph,
    // once per speaker (Model::spk_version)
    int enc_fill = -1, spk_seen = -1;
    int delay = 0;
    int ad_mode = -1;                              // AdaIN mode baked into the plans
    int ad_row0 = 0;                               // AdaIN buffer row baked into the plans
    bool has_enc() const { return enc != nullptr; }
    bool has_dec() const { return dec != nullptr; }
    std::vector<int> enc_adain, dec_adain;         // AdaIN op indices
    ~Stream();
};

}  // namespace rave
