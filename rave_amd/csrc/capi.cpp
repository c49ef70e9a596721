// C-ABI glue: error reporting, ABI self-check, and the plan executor that
// replays a recorded op sequence (the RAVE.encode / decode module graph,
// rave/model.py:594-634) with per-call pointer relocation.
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <vector>

#include "common.h"
#include "shift_batch.h"

namespace rave {
static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
thread_local OpEvents g_op_events;
}  // namespace rave

struct rave_plan {
    std::vector<rave_plan_op> ops;
    std::vector<rave_reloc> relocs;
    std::vector<hipEvent_t> ev;          // 2 per op per armed run when profiling
    int runs_cap = 0;                    // armed runs
    int runs = 0;                        // runs recorded since the last op_times
};

extern "C" const char* rave_last_error(void) { return rave::g_err.c_str(); }

extern "C" int rave_abi_version(void) { return RAVE_ABI_VERSION; }

extern "C" int rave_struct_sizes(int64_t* out, int n) {
    const int64_t sizes[] = {
        (int64_t)sizeof(rave_conv1d_args),       (int64_t)sizeof(rave_pqmf_analysis_args),
        (int64_t)sizeof(rave_pqmf_synthesis_args), (int64_t)sizeof(rave_fill_args),
        (int64_t)sizeof(rave_rvq_args),          (int64_t)sizeof(rave_shift_args),
        (int64_t)sizeof(rave_plan_op),           (int64_t)sizeof(rave_reloc),
        (int64_t)sizeof(rave_copy_args),         (int64_t)sizeof(rave_noise_args),
        (int64_t)sizeof(rave_adain_args),        (int64_t)sizeof(rave_unit_args),
        (int64_t)sizeof(rave_stack_args),        (int64_t)sizeof(rave_model_config),
        (int64_t)sizeof(rave_param),             (int64_t)sizeof(rave_op_info),
        (int64_t)sizeof(rave_fir_args),          (int64_t)sizeof(rave_row_stats_args),
        (int64_t)sizeof(rave_attn_pool_args),    (int64_t)sizeof(rave_linear_args),
        (int64_t)sizeof(rave_maxpool_args),      (int64_t)sizeof(rave_edge_args),
    };
    const int cnt = (int)(sizeof(sizes) / sizeof(sizes[0]));
    if (!out) return cnt;
    for (int i = 0; i < n && i < cnt; ++i) out[i] = sizes[i];
    return cnt;
}

extern "C" int rave_plan_create(const rave_plan_op* ops, int n_ops, const rave_reloc* relocs,
                                int n_relocs, rave_plan** out) {
    if (!out || n_ops < 0 || n_relocs < 0 || (n_ops && !ops) || (n_relocs && !relocs)) {
        rave::set_error("plan_create: bad arguments");
        return RAVE_ERR_ARG;
    }
    for (int i = 0; i < n_relocs; ++i) {
        const rave_reloc& r = relocs[i];
        if (r.op < 0 || r.op >= n_ops || r.field_offset < 0 ||
            r.field_offset + (int)sizeof(void*) > RAVE_OP_PAYLOAD || (r.field_offset % 8) != 0 ||
            r.slot < 0) {
            rave::set_error("plan_create: bad relocation " + std::to_string(i));
            return RAVE_ERR_ARG;
        }
    }
    rave_plan* p = new rave_plan;
    p->ops.assign(ops, ops + n_ops);
    p->relocs.assign(relocs, relocs + n_relocs);
    *out = p;
    return RAVE_OK;
}

extern "C" int rave_plan_profile(rave_plan* plan, int runs) {
    if (!plan || runs < 0) {
        rave::set_error("plan_profile: null plan or negative run count");
        return RAVE_ERR_STATE;
    }
    for (hipEvent_t e : plan->ev) (void)hipEventDestroy(e);
    plan->ev.clear();
    plan->runs_cap = 0;
    plan->runs = 0;
    if (runs > 0) {
        plan->ev.resize(2 * plan->ops.size() * (size_t)runs);
        for (auto& e : plan->ev) {
            hipError_t err = hipEventCreate(&e);
            if (err != hipSuccess) {
                rave::set_error(std::string("plan_profile: ") + hipGetErrorString(err));
                return RAVE_ERR_HIP;
            }
        }
        plan->runs_cap = runs;
    }
    return RAVE_OK;
}

extern "C" int rave_plan_op_times(rave_plan* plan, float* ms, int n) {
    if (!plan || plan->ev.empty()) {
        rave::set_error("plan_op_times: profiling not enabled");
        return RAVE_ERR_STATE;
    }
    const int nops = (int)plan->ops.size();
    const int runs = plan->runs;
    for (int r = 0; r < runs; ++r) {
        hipEvent_t* ev = plan->ev.data() + (size_t)2 * nops * r;
        hipError_t err = hipEventSynchronize(ev[2 * nops - 1]);
        for (int i = 0; i < nops && i < n && err == hipSuccess; ++i) {
            float t = 0.f;
            err = hipEventElapsedTime(&t, ev[2 * i], ev[2 * i + 1]);
            ms[i] += t;
        }
        if (err != hipSuccess) {
            rave::set_error(std::string("plan_op_times: ") + hipGetErrorString(err));
            return RAVE_ERR_HIP;
        }
    }
    plan->runs = 0;
    return runs;
}

extern "C" int rave_plan_destroy(rave_plan* plan) {
    if (plan)
        for (hipEvent_t e : plan->ev) (void)hipEventDestroy(e);
    delete plan;
    return RAVE_OK;
}

extern "C" int rave_plan_size(const rave_plan* plan) { return plan ? (int)plan->ops.size() : -1; }

namespace rave {
// Engine-internal: overwrite `n` bytes of op `op`'s argument payload (e.g. an
// AdaIN op's mode when the learn flags change between streaming blocks).
int plan_patch(rave_plan* plan, int op, int offset, const void* data, int n) {
    if (!plan || op < 0 || op >= (int)plan->ops.size() || offset < 0 || n < 0 || offset + n > RAVE_OP_PAYLOAD) {
        set_error("plan_patch: bad arguments");
        return RAVE_ERR_ARG;
    }
    std::memcpy(plan->ops[op].u.raw + offset, data, (size_t)n);
    return RAVE_OK;
}
}  // namespace rave

namespace rave {
int plan_run_from(rave_plan* plan, void* const* slots, int n_slots, void* stream, int first, int end, int skip);
}

extern "C" int rave_plan_run(rave_plan* plan, void* const* slots, int n_slots, void* stream) {
    return rave::plan_run_from(plan, slots, n_slots, stream, 0, -1, -1);
}

namespace rave {
// Engine-internal: run ops [first, end) of the plan (end < 0: to the last op),
// leaving out op `skip` (< 0: none).  A stream graph whose input copy the host
// does itself is captured from op 1, and its speaker fill runs only when the
// speaker changes.  Unprofiled unless it is the whole plan.
int plan_run_from(rave_plan* plan, void* const* slots, int n_slots, void* stream, int first, int end, int skip) {
    if (!plan) {
        rave::set_error("plan_run: null plan");
        return RAVE_ERR_STATE;
    }
    if (end < 0) end = (int)plan->ops.size();
    if (first < 0 || first > end || end > (int)plan->ops.size()) {
        rave::set_error("plan_run: bad op range");
        return RAVE_ERR_ARG;
    }
    // The relocated op list is per call and per host thread (the plan itself is
    // read-only here), so threads may run one plan concurrently on their own
    // streams as long as the plan's workspace slots differ per call.
    static thread_local std::vector<rave_plan_op> scratch;
    scratch.assign(plan->ops.begin(), plan->ops.end());
    for (const rave_reloc& r : plan->relocs) {
        if (r.slot >= n_slots || !slots || !slots[r.slot]) {
            rave::set_error("plan_run: slot " + std::to_string(r.slot) + " not bound");
            return RAVE_ERR_ARG;
        }
        char* base = static_cast<char*>(slots[r.slot]) + r.byte_offset;
        std::memcpy(scratch[r.op].u.raw + r.field_offset, &base, sizeof(void*));
    }
    const bool prof = first == 0 && end == (int)plan->ops.size() && skip < 0 &&
                      plan->runs < plan->runs_cap;   // armed and not yet full
    hipEvent_t* ev = prof ? plan->ev.data() + (size_t)2 * scratch.size() * plan->runs : nullptr;
    for (size_t i = (size_t)first; i < (size_t)end; ++i) {
        if ((int)i == skip) continue;
        const rave_plan_op& op = scratch[i];
        int rc;
        if (prof) rave::g_op_events = {ev[2 * i], ev[2 * i + 1]};
        switch (op.kind) {
            case RAVE_OP_CONV: rc = rave_conv1d(&op.u.conv, stream); break;
            case RAVE_OP_PQMF_ANALYSIS: rc = rave_pqmf_analysis(&op.u.ana, stream); break;
            case RAVE_OP_PQMF_SYNTHESIS: rc = rave_pqmf_synthesis(&op.u.syn, stream); break;
            case RAVE_OP_FILL: rc = rave_fill_channels(&op.u.fill, stream); break;
            case RAVE_OP_RVQ_ENCODE: rc = rave_rvq_encode(&op.u.rvq, stream); break;
            case RAVE_OP_RVQ_DECODE: rc = rave_rvq_decode(&op.u.rvq, stream); break;
            case RAVE_OP_SHIFT_HISTORY: {
                // consecutive history shifts (one per streaming buffer) go out as
                // one launch, timed on the first op; the rest record empty intervals
                const rave_shift_args* batch[rave::kShiftBatch];
                int n = 0;
                while (n < rave::kShiftBatch && i + n < (size_t)end && (int)(i + n) != skip &&
                       scratch[i + n].kind == RAVE_OP_SHIFT_HISTORY) {
                    batch[n] = &scratch[i + n].u.shift;
                    ++n;
                }
                rc = rave::shift_history_batch(batch, n, static_cast<hipStream_t>(stream));
                if (prof && rave::g_op_events.start) {
                    (void)hipEventRecord(ev[2 * i], static_cast<hipStream_t>(stream));
                    (void)hipEventRecord(ev[2 * i + 1], static_cast<hipStream_t>(stream));
                }
                for (int j = 1; j < n && prof; ++j) {
                    (void)hipEventRecord(ev[2 * (i + j)], static_cast<hipStream_t>(stream));
                    (void)hipEventRecord(ev[2 * (i + j) + 1], static_cast<hipStream_t>(stream));
                }
                i += n - 1;
                if (prof) rave::g_op_events = {};
                break;
            }
            case RAVE_OP_COPY: rc = rave_copy(&op.u.copy, stream); break;
            case RAVE_OP_NOISE: rc = rave_noise_synth(&op.u.noise, stream); break;
            case RAVE_OP_ADAIN: rc = rave_adain(&op.u.adain, stream); break;
            case RAVE_OP_UNIT: rc = rave_residual_unit(&op.u.unit, stream); break;
            case RAVE_OP_STACK: rc = rave_residual_stack(&op.u.stack, stream); break;
            case RAVE_OP_HEAD: rc = rave_encoder_head(&op.u.edge, stream); break;
            case RAVE_OP_TAIL: rc = rave_decoder_tail(&op.u.edge, stream); break;
            default:
                rave::set_error("plan_run: unknown op kind " + std::to_string(op.kind));
                return RAVE_ERR_STATE;
        }
        if (prof) {
            if (rave::g_op_events.start) {   // the op launched nothing: record an empty interval
                (void)hipEventRecord(ev[2 * i], static_cast<hipStream_t>(stream));
                (void)hipEventRecord(ev[2 * i + 1], static_cast<hipStream_t>(stream));
            }
            rave::g_op_events = {};
        }
        if (rc != RAVE_OK) {
            rave::set_error("plan op " + std::to_string(i) + ": " + rave::g_err);
            return rc;
        }
    }
    if (prof) ++plan->runs;
    return RAVE_OK;
}
}  // namespace rave
