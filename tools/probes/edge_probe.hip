// Stage timing of the fused path edges (csrc/edge_split.hip) at the bench
// shape (16 clips x 4096 PQMF frames).  Built once per stage cut:
//   hipcc -O3 --offload-arch=gfx950 -DRAVE_EDGE_STOP=<n> tools/probes/edge_probe.hip -o edge_probe_<n>
// (no -DRAVE_EDGE_STOP: the whole kernels).  Operands are zeros / small
// constants: timing only, no results checked (tests/test_gpu_edges.py checks).
#include "../../rave_amd/csrc/edge_split.hip"

#include <cstdio>
#include <vector>

namespace rave {
void set_error(const std::string& msg) { std::fprintf(stderr, "error: %s\n", msg.c_str()); }
thread_local OpEvents g_op_events;
}  // namespace rave

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            return 1;                                                              \
        }                                                                          \
    } while (0)

template <typename F>
static double time_us(F&& f, int reps = 20) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int i = 0; i < 3; ++i) f();
    (void)hipEventRecord(e0, nullptr);
    for (int i = 0; i < reps; ++i) f();
    (void)hipEventRecord(e1, nullptr);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return 1e3 * ms / reps;
}

int main() {
    const int B = 16, F = 4096, T = 16 * F;
    float *x_audio, *x_feat, *y_feat, *y_audio, *w, *filt, *bias, *alpha, *z, *spk;
    CK(hipMalloc(&x_audio, (size_t)B * T * 4));
    CK(hipMalloc(&x_feat, (size_t)B * 64 * F * 4));
    CK(hipMalloc(&y_feat, (size_t)B * 64 * F * 4));
    CK(hipMalloc(&y_audio, (size_t)B * T * 4));
    CK(hipMalloc(&w, (size_t)4 << 20));
    CK(hipMalloc(&filt, (size_t)16 * 16 * 33 * 4 + 16 * 513 * 4));
    CK(hipMalloc(&bias, 64 * 4));
    CK(hipMalloc(&alpha, 64 * 4));
    CK(hipMalloc(&z, (size_t)B * 320 * 64 * 4));
    CK(hipMalloc(&spk, 256 * 4));
    std::vector<float> ones((size_t)B * 64 * F, 0.25f);
    CK(hipMemcpy(x_feat, ones.data(), ones.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(x_audio, ones.data(), (size_t)B * T * 4, hipMemcpyHostToDevice));
    CK(hipMemset(w, 0, (size_t)4 << 20));
    CK(hipMemcpy(filt, ones.data(), (size_t)16 * 16 * 33 * 4, hipMemcpyHostToDevice));
    CK(hipMemset(bias, 0, 64 * 4));
    CK(hipMemcpy(alpha, ones.data(), 64 * 4, hipMemcpyHostToDevice));

    rave_edge_args h{};
    h.batch = B; h.frames = F; h.conv_c_in = 6; h.conv_c_out = 64; h.conv_kernel = 7; h.conv_pad_left = 3;
    h.pqmf_taps = 513; h.pqmf_pad_left = 256;
    h.x = x_audio; h.x_sb = T; h.y = y_feat; h.y_sb = 64 * F; h.y_sc = F;
    h.weight = w; h.bias = bias; h.filter = filt;
    h.fill_channels = 256; h.fill_t = 64; h.fill_y = z + 64 * 64; h.f_sb = 320 * 64; h.f_sc = 64; h.fill_values = spk;

    rave_edge_args t{};
    t.batch = B; t.frames = F; t.conv_c_in = 64; t.conv_c_out = 32; t.conv_kernel = 7; t.conv_pad_left = 3;
    t.pqmf_taps = 33; t.pqmf_pad_left = 16; t.mode = 1; t.act = RAVE_ACT_LEAKY; t.leaky_slope = 0.2f;
    t.x = x_feat; t.x_sb = 64 * F; t.x_sc = F; t.y = y_audio; t.y_sb = T;
    t.weight = w; t.bias = bias; t.filter = filt;

    int rc = 0;
    const double th = time_us([&] { rc |= rave_encoder_head(&h, nullptr); });
    const double tt = time_us([&] { rc |= rave_decoder_tail(&t, nullptr); });
    CK(hipDeviceSynchronize());
#ifdef RAVE_EDGE_STOP
    const int stop = RAVE_EDGE_STOP;
#else
    const int stop = 0;
#endif
    std::printf("{\"stop\": %d, \"head_us\": %.2f, \"tail_us\": %.2f, \"rc\": %d}\n", stop, th, tt, rc);
    return rc != 0;
}
