"""ctypes binding of librave_amd.so (include/rave_amd.h).

The shared library is built in-tree by ``__graft_entry__.build()`` /
``make -C rave_amd/csrc``.  There is no fallback: if the library is missing
or its ABI does not match these struct mirrors, importing fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "librave_amd.so")
# Kernel-tuning hook only: tools/ may point this at the -DRAVE_STAMPS diagnostic
# build (rave_amd/librave_amd_diag.so).  The product always loads LIB_PATH.
if os.environ.get("RAVE_AMD_DIAG_LIB") == "1":
    LIB_PATH = os.path.join(_HERE, "librave_amd_diag.so")
# ... or at an A/B experiment build (csrc/Makefile: OUT=../librave_amd_<name>.so)
if os.environ.get("RAVE_AMD_LIB_VARIANT"):
    LIB_PATH = os.path.join(_HERE, f"librave_amd_{os.environ['RAVE_AMD_LIB_VARIANT']}.so")

RAVE_OK = 0
RAVE_ERR_ARG = -1
RAVE_ERR_HIP = -2
RAVE_ERR_UNSUPPORTED = -3
RAVE_ERR_STATE = -4
RAVE_ERR_COOP = -5         # a cooperative unit's in-launch hand-off gave up (RuntimeError)

ACT = {"none": 0, "leaky": 1, "snake": 2}

OP_CONV = 1
OP_PQMF_ANALYSIS = 2
OP_PQMF_SYNTHESIS = 3
OP_FILL = 4
OP_RVQ_ENCODE = 5
OP_RVQ_DECODE = 6
OP_SHIFT_HISTORY = 7
OP_COPY = 8
OP_NOISE = 9
OP_ADAIN = 10
OP_UNIT = 11
OP_STACK = 12
OP_HEAD = 13
OP_TAIL = 14
ABI_VERSION = 18
SPLITK_TICKETS = 4096       # RAVE_SPLITK_TICKETS: zeroed int32 counters at the head of a split-K workspace
SPLITK_STATUS_WORD = SPLITK_TICKETS - 1   # RAVE_SPLITK_STATUS_WORD: the cooperative unit's give-up word

# GEMM arithmetic of conv / unit ops (include/rave_amd.h RAVE_PREC_*)
PREC_F32 = 0
PREC_SPLIT16 = 1
PREC_AUTO = 2
PREC_F32_TUNED = 3      # exact fp32, launch choices autotuned (RAVE_PREC_F32_TUNED)
PREC_F32_RING = 4       # exact fp32 on the split16 kernels' staging machinery (RAVE_PREC_F32_RING)
PREC_BF16X3 = 5         # fp32 on the bf16 matrix cores, exact 3-way operand split (RAVE_PREC_BF16X3)
PREC_F32_BF3 = 6        # model mode: per op the fastest of F32 / F32_RING / BF16X3 (RAVE_PREC_F32_BF3)
PRECISION = {"f32": PREC_F32, "split16": PREC_SPLIT16, "f32_ring": PREC_F32_RING, "bf16x3": PREC_BF16X3}
STREAM_GRAPH = 1
STREAM_ENCODE_ONLY = 2
STREAM_DECODE_ONLY = 4

i32, i64, f32, vp = C.c_int32, C.c_int64, C.c_float, C.c_void_p


class ConvArgs(C.Structure):
    _fields_ = [("c_in", i32), ("c_out", i32), ("kernel", i32), ("stride", i32), ("dilation", i32),
                ("pad_left", i32), ("pad_right", i32), ("transposed", i32), ("out_shift", i32),
                ("act", i32), ("leaky_slope", f32), ("batch", i32), ("t_in", i32), ("t_out", i32),
                ("precision", i32),
                ("x", vp), ("x_sb", i64), ("x_sc", i64),
                ("y", vp), ("y_sb", i64), ("y_sc", i64),
                ("residual", vp), ("r_sb", i64), ("r_sc", i64),
                ("weight", vp), ("bias", vp), ("alpha", vp), ("partial", vp), ("stamps", vp),
                ("config", i32), ("_pad1", i32)]


class AnalysisArgs(C.Structure):
    _fields_ = [("n_band", i32), ("taps", i32), ("n_out_bands", i32), ("batch", i32),
                ("t_in", i32), ("pad_left", i32), ("t_out", i32), ("precision", i32),
                ("x", vp), ("x_sb", i64),
                ("y", vp), ("y_sb", i64), ("y_sc", i64),
                ("hkf", vp)]


class SynthesisArgs(C.Structure):
    _fields_ = [("n_band", i32), ("taps", i32), ("batch", i32), ("t_in", i32),
                ("pad_left", i32), ("mode", i32), ("frame0", i32), ("x_len", i32),
                ("x", vp), ("x_sb", i64), ("x_sc", i64),
                ("noise", vp), ("n_sb", i64), ("n_sc", i64),
                ("y", vp), ("y_sb", i64),
                ("hki", vp), ("precision", i32), ("_pad0", i32)]


class FillArgs(C.Structure):
    _fields_ = [("batch", i32), ("channels", i32), ("t_len", i32), ("_pad0", i32),
                ("y", vp), ("y_sb", i64), ("y_sc", i64), ("values", vp)]


class RvqArgs(C.Structure):
    _fields_ = [("n_q", i32), ("codebook_size", i32), ("dim", i32), ("batch", i32),
                ("t_len", i32), ("_pad0", i32),
                ("codebooks", vp),
                ("z", vp), ("z_sb", i64), ("z_sc", i64),
                ("idx", vp), ("i_sb", i64), ("i_sq", i64),
                ("y", vp), ("y_sb", i64), ("y_sc", i64),
                ("work", vp)]


class ShiftArgs(C.Structure):
    _fields_ = [("batch", i32), ("channels", i32), ("hist", i32), ("t_new", i32),
                ("buf", vp), ("sb", i64), ("sc", i64)]


class CopyArgs(C.Structure):
    _fields_ = [("batch", i32), ("channels", i32), ("t_len", i32), ("_pad0", i32),
                ("x", vp), ("x_sb", i64), ("x_sc", i64),
                ("y", vp), ("y_sb", i64), ("y_sc", i64)]


class NoiseArgs(C.Structure):
    _fields_ = [("batch", i32), ("frames", i32), ("n_band", i32), ("noise_bands", i32),
                ("target", i32), ("_pad0", i32),
                ("amp", vp), ("a_sb", i64), ("a_sc", i64),
                ("u", vp), ("u_sb", i64),
                ("y", vp), ("y_sb", i64), ("y_sc", i64)]


class AdainArgs(C.Structure):
    _fields_ = [("batch", i32), ("channels", i32), ("t_len", i32), ("mode", i32),
                ("max_batch", i32), ("row0", i32),
                ("x", vp), ("x_sb", i64), ("x_sc", i64),
                ("y", vp), ("y_sb", i64), ("y_sc", i64),
                ("stats", vp), ("counters", vp), ("ticket", vp)]


class UnitArgs(C.Structure):
    _fields_ = [("channels", i32), ("batch", i32), ("t_len", i32), ("dilation", i32),
                ("pad_left", i32), ("act", i32), ("leaky_slope", f32), ("precision", i32),
                ("x", vp), ("x_sb", i64), ("x_sc", i64),
                ("y", vp), ("y_sb", i64), ("y_sc", i64),
                ("weight", vp), ("bias1", vp), ("bias2", vp), ("alpha0", vp), ("alpha2", vp),
                ("workspace", vp), ("status", vp), ("x_len", i32), ("res_shift", i32),
                ("coop_rb", i32), ("reserved0", i32)]


STACK_UNITS = 3


class StackArgs(C.Structure):
    _fields_ = ([("channels", i32), ("batch", i32), ("t_len", i32), ("act", i32),
                 ("leaky_slope", f32), ("precision", i32)]
                + [(f"dilation{u}", i32) for u in range(STACK_UNITS)]
                + [(f"pad_left{u}", i32) for u in range(STACK_UNITS)]
                + [("x", vp), ("x_sb", i64), ("x_sc", i64), ("y", vp), ("y_sb", i64), ("y_sc", i64)]
                + [(f"{f}{u}", vp) for f in ("weight", "bias1", "bias2", "alpha0", "alpha2")
                   for u in range(STACK_UNITS)])


class FirArgs(C.Structure):
    _fields_ = [("batch", i32), ("t_in", i32), ("t_out", i32), ("phases", i32), ("taps", i32),
                ("stride", i32), ("pad_left", i32), ("_pad0", i32),
                ("x", vp), ("x_sb", i64), ("y", vp), ("y_sb", i64), ("h", vp)]


class RowStatsArgs(C.Structure):
    _fields_ = [("batch", i32), ("channels", i32), ("t_len", i32), ("act", i32),
                ("leaky_slope", f32), ("var_min", f32), ("var_max", f32), ("_pad0", i32),
                ("x", vp), ("x_sb", i64), ("x_sc", i64), ("y", vp), ("y_sb", i64)]


class AttnPoolArgs(C.Structure):
    _fields_ = [("batch", i32), ("channels", i32), ("t_len", i32), ("act", i32),
                ("leaky_slope", f32), ("var_min", f32), ("var_max", f32), ("_pad0", i32),
                ("x", vp), ("x_sb", i64), ("x_sc", i64), ("logits", vp), ("l_sb", i64), ("l_sc", i64),
                ("y", vp), ("y_sb", i64)]


class LinearArgs(C.Structure):
    _fields_ = [("batch", i32), ("n_in", i32), ("n_out", i32), ("_pad0", i32),
                ("x", vp), ("x_sb", i64), ("w", vp), ("bias", vp), ("y", vp), ("y_sb", i64)]


class MaxPoolArgs(C.Structure):
    _fields_ = [("batch", i32), ("channels", i32), ("t_out", i32), ("kernel", i32),
                ("x", vp), ("x_sb", i64), ("x_sc", i64), ("y", vp), ("y_sb", i64), ("y_sc", i64)]


class EdgeArgs(C.Structure):
    _fields_ = [("batch", i32), ("frames", i32), ("conv_c_in", i32), ("conv_c_out", i32), ("conv_kernel", i32),
                ("conv_pad_left", i32), ("pqmf_taps", i32), ("pqmf_pad_left", i32), ("mode", i32), ("act", i32),
                ("leaky_slope", f32), ("fill_channels", i32), ("fill_t", i32), ("precision", i32),
                ("x", vp), ("x_sb", i64), ("x_sc", i64), ("y", vp), ("y_sb", i64), ("y_sc", i64),
                ("weight", vp), ("bias", vp), ("alpha", vp), ("filter", vp),
                ("noise", vp), ("n_sb", i64), ("n_sc", i64),
                ("fill_y", vp), ("f_sb", i64), ("f_sc", i64), ("fill_values", vp)]


MAX_RATIOS = 8
MAX_DILATIONS = 8


class ModelConfig(C.Structure):
    _fields_ = [("n_band", i32), ("enc_bands", i32), ("capacity", i32), ("latent_size", i32),
                ("kernel_size", i32), ("speaker_size", i32), ("n_ratios", i32),
                ("ratios", i32 * MAX_RATIOS), ("n_dilations", i32 * MAX_RATIOS),
                ("dilations", (i32 * MAX_DILATIONS) * MAX_RATIOS),
                ("amplitude_modulation", i32), ("causal", i32), ("activation", i32), ("adain", i32),
                ("leaky_slope", f32), ("conv_bias", i32), ("convt_bias", i32),
                ("noise", i32), ("noise_hidden", i32), ("noise_bands", i32), ("n_noise_ratios", i32),
                ("noise_ratios", i32 * MAX_RATIOS), ("rvq_quantizers", i32), ("rvq_codebook_size", i32),
                ("fuse_units", i32)]


class Param(C.Structure):
    _fields_ = [("name", C.c_char_p), ("data", vp), ("numel", i64)]


class OpInfo(C.Structure):
    _fields_ = [("kind", i32), ("precision", i32), ("flops", C.c_double), ("bytes", C.c_double),
                ("label", C.c_char * 96)]


PAYLOAD = 240


class PlanOp(C.Structure):
    _fields_ = [("kind", i32), ("_pad0", i32), ("raw", C.c_ubyte * PAYLOAD)]


class Reloc(C.Structure):
    _fields_ = [("op", i32), ("field_offset", i32), ("slot", i32), ("_pad0", i32),
                ("byte_offset", i64)]


STRUCTS = [ConvArgs, AnalysisArgs, SynthesisArgs, FillArgs, RvqArgs, ShiftArgs, PlanOp, Reloc,
           CopyArgs, NoiseArgs, AdainArgs, UnitArgs, StackArgs, ModelConfig, Param, OpInfo,
           FirArgs, RowStatsArgs, AttnPoolArgs, LinearArgs, MaxPoolArgs, EdgeArgs]

# every exported symbol of include/rave_amd.h
EXPORTS = [
    "rave_last_error", "rave_abi_version", "rave_struct_sizes",
    "rave_conv1d_chunk", "rave_conv1d_packed_size", "rave_conv1d_pack_weight", "rave_conv1d",
    "rave_conv1d_workspace", "rave_conv1d_configs", "rave_conv1d_split_packed_size", "rave_conv1d_split_pack_weight",
    "rave_conv1d_ring_pack_weight", "rave_conv1d_bf3_packed_size", "rave_conv1d_bf3_pack_weight",
    "rave_pqmf_analysis", "rave_pqmf_synthesis", "rave_fill_channels", "rave_copy",
    "rave_rvq_workspace", "rave_rvq_encode", "rave_rvq_decode", "rave_shift_history", "rave_noise_synth", "rave_adain",
    "rave_unit_packed_size", "rave_unit_pack_weight", "rave_residual_unit",
    "rave_unit_split_packed_size", "rave_unit_split_pack_weight", "rave_unit_ring_pack_weight",
    "rave_unit_bf3_packed_size", "rave_unit_bf3_pack_weight",
    "rave_unit_workspace", "rave_debug_coop", "rave_model_check",
    "rave_stack_supported", "rave_residual_stack",
    "rave_plan_create", "rave_plan_run", "rave_plan_destroy", "rave_plan_size",
    "rave_plan_profile", "rave_plan_op_times", "rave_fill_uniform",
    "rave_model_param_count", "rave_model_param_info", "rave_model_create", "rave_model_destroy",
    "rave_model_encode", "rave_model_decode", "rave_model_forward", "rave_model_encode_codes",
    "rave_model_decode_codes", "rave_model_noise_shape", "rave_model_adain_control", "rave_model_set_row0",
    "rave_model_set_speaker",
    "rave_model_adain_count", "rave_model_adain_info", "rave_model_adain_get", "rave_model_adain_set",
    "rave_model_tuning_get", "rave_model_tuning_set", "rave_model_plan_ops", "rave_model_profile",
    "rave_model_op_times", "rave_stream_create", "rave_stream_destroy", "rave_stream_reset",
    "rave_stream_encode", "rave_stream_decode", "rave_stream_encode_codes", "rave_stream_decode_codes",
    "rave_stream_delay",
    "rave_stream_launches",
    "rave_fir", "rave_row_stats", "rave_attn_pool", "rave_linear", "rave_maxpool",
    "rave_encoder_head", "rave_decoder_tail", "rave_encoder_head_pack_filter", "rave_decoder_tail_pack_filter",
    "rave_encoder_head_pack_filter_f32", "rave_decoder_tail_pack_filter_f32",
]
EDGE_FILTER_FLOATS = 8836   # RAVE_EDGE_FILTER_FLOATS


class NativeError(RuntimeError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"rave_amd native library not built: {LIB_PATH} is missing "
                          "(run `python -c 'import __graft_entry__ as g; g.build()'` or "
                          "`make -C rave_amd/csrc`)")
    lib = C.CDLL(LIB_PATH)
    lib.rave_last_error.restype = C.c_char_p
    lib.rave_abi_version.restype = C.c_int
    lib.rave_struct_sizes.argtypes = [C.POINTER(i64), C.c_int]
    lib.rave_conv1d_chunk.argtypes = [C.c_int] * 5
    lib.rave_conv1d_packed_size.argtypes = [C.c_int] * 6
    lib.rave_conv1d_packed_size.restype = i64
    lib.rave_conv1d_pack_weight.argtypes = [vp] + [C.c_int] * 7 + [vp]
    lib.rave_conv1d_workspace.argtypes = [C.POINTER(ConvArgs)]
    lib.rave_conv1d_configs.argtypes = [C.POINTER(ConvArgs), C.POINTER(i32), C.c_int]
    lib.rave_conv1d_split_packed_size.argtypes = [C.c_int] * 6
    lib.rave_conv1d_split_packed_size.restype = i64
    lib.rave_conv1d_split_pack_weight.argtypes = [vp] + [C.c_int] * 7 + [vp]
    lib.rave_conv1d_ring_pack_weight.argtypes = [vp] + [C.c_int] * 7 + [vp]
    lib.rave_conv1d_bf3_packed_size.argtypes = [C.c_int] * 6
    lib.rave_conv1d_bf3_packed_size.restype = i64
    lib.rave_conv1d_bf3_pack_weight.argtypes = [vp] + [C.c_int] * 7 + [vp]
    lib.rave_encoder_head_pack_filter.argtypes = [vp, C.c_int, C.c_int, C.c_int, vp]
    lib.rave_encoder_head_pack_filter_f32.argtypes = [vp, C.c_int, C.c_int, C.c_int, vp]
    lib.rave_decoder_tail_pack_filter_f32.argtypes = [vp, C.c_int, C.c_int, vp]
    lib.rave_decoder_tail_pack_filter.argtypes = [vp, C.c_int, C.c_int, vp]
    lib.rave_unit_packed_size.argtypes = [C.c_int]
    lib.rave_unit_packed_size.restype = i64
    lib.rave_unit_pack_weight.argtypes = [vp, vp, C.c_int, vp]
    lib.rave_unit_workspace.argtypes = [C.c_void_p]
    lib.rave_unit_workspace.restype = i64
    lib.rave_debug_coop.argtypes = [i64, C.c_int]
    lib.rave_unit_split_packed_size.argtypes = [C.c_int]
    lib.rave_stack_supported.argtypes = [C.c_int]
    lib.rave_unit_split_packed_size.restype = i64
    lib.rave_unit_split_pack_weight.argtypes = [vp, vp, C.c_int, vp]
    lib.rave_unit_ring_pack_weight.argtypes = [vp, vp, C.c_int, vp]
    lib.rave_unit_bf3_packed_size.argtypes = [C.c_int]
    lib.rave_unit_bf3_packed_size.restype = i64
    lib.rave_unit_bf3_pack_weight.argtypes = [vp, vp, C.c_int, vp]
    lib.rave_conv1d_workspace.restype = i64
    lib.rave_rvq_workspace.argtypes = [C.POINTER(RvqArgs)]
    lib.rave_rvq_workspace.restype = i64
    for name, st in [("rave_conv1d", ConvArgs), ("rave_pqmf_analysis", AnalysisArgs),
                     ("rave_pqmf_synthesis", SynthesisArgs), ("rave_fill_channels", FillArgs),
                     ("rave_rvq_encode", RvqArgs), ("rave_rvq_decode", RvqArgs),
                     ("rave_shift_history", ShiftArgs), ("rave_copy", CopyArgs),
                     ("rave_noise_synth", NoiseArgs), ("rave_adain", AdainArgs),
                     ("rave_residual_unit", UnitArgs), ("rave_residual_stack", StackArgs),
                     ("rave_fir", FirArgs), ("rave_row_stats", RowStatsArgs), ("rave_attn_pool", AttnPoolArgs),
                     ("rave_linear", LinearArgs), ("rave_maxpool", MaxPoolArgs),
                     ("rave_encoder_head", EdgeArgs), ("rave_decoder_tail", EdgeArgs)]:
        getattr(lib, name).argtypes = [C.POINTER(st), vp]
    lib.rave_plan_create.argtypes = [C.POINTER(PlanOp), C.c_int, C.POINTER(Reloc), C.c_int,
                                     C.POINTER(vp)]
    lib.rave_plan_run.argtypes = [vp, C.POINTER(vp), C.c_int, vp]
    lib.rave_plan_destroy.argtypes = [vp]
    lib.rave_plan_size.argtypes = [vp]
    lib.rave_plan_profile.argtypes = [vp, C.c_int]
    lib.rave_plan_op_times.argtypes = [vp, C.POINTER(C.c_float), C.c_int]
    lib.rave_fill_uniform.argtypes = [vp, i64, C.c_uint64, f32, f32, vp]
    # model engine
    cfgp = C.POINTER(ModelConfig)
    lib.rave_model_param_count.argtypes = [cfgp]
    lib.rave_model_param_info.argtypes = [cfgp, C.c_int, C.c_char_p, C.c_int, C.POINTER(i64)]
    lib.rave_model_create.argtypes = [cfgp, C.POINTER(Param), C.c_int, vp, C.c_int, C.POINTER(vp)]
    lib.rave_model_destroy.argtypes = [vp]
    lib.rave_model_encode.argtypes = [vp, vp, C.c_int, C.c_int, vp, vp]
    lib.rave_model_decode.argtypes = [vp, vp, C.c_int, C.c_int, vp, vp, vp]
    lib.rave_model_forward.argtypes = [vp, vp, C.c_int, C.c_int, vp, vp, vp]
    lib.rave_model_encode_codes.argtypes = [vp, vp, C.c_int, C.c_int, vp, vp]
    lib.rave_model_decode_codes.argtypes = [vp, vp, C.c_int, C.c_int, vp, vp, vp]
    lib.rave_model_check.argtypes = [vp, C.c_int, vp]
    lib.rave_model_noise_shape.argtypes = [vp, C.c_int, C.c_int, C.POINTER(i64)]
    lib.rave_model_adain_control.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, vp]
    lib.rave_model_set_row0.argtypes = [vp, C.c_int]
    lib.rave_model_set_speaker.argtypes = [vp, vp, vp]
    lib.rave_model_adain_count.argtypes = [vp]
    lib.rave_model_adain_info.argtypes = [vp, C.c_int, C.c_char_p, C.c_int, C.POINTER(C.c_int),
                                          C.POINTER(C.c_int)]
    lib.rave_model_adain_get.argtypes = [vp, C.c_int, vp, vp]
    lib.rave_model_adain_set.argtypes = [vp, C.c_int, vp, vp]
    lib.rave_model_tuning_get.argtypes = [vp, C.c_char_p, C.c_int]
    lib.rave_model_tuning_set.argtypes = [vp, C.c_char_p]
    lib.rave_model_plan_ops.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.POINTER(OpInfo), C.c_int]
    lib.rave_model_profile.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int]
    lib.rave_model_op_times.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_float), C.c_int]
    lib.rave_stream_create.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.POINTER(vp)]
    lib.rave_stream_destroy.argtypes = [vp]
    lib.rave_stream_reset.argtypes = [vp, vp]
    lib.rave_stream_encode.argtypes = [vp, vp, vp, vp]
    lib.rave_stream_decode.argtypes = [vp, vp, vp, vp, vp]
    lib.rave_stream_encode_codes.argtypes = [vp, vp, vp, vp]
    lib.rave_stream_decode_codes.argtypes = [vp, vp, vp, vp, vp]
    lib.rave_stream_delay.argtypes = [vp]
    lib.rave_stream_launches.argtypes = [vp, C.c_int]
    # ABI self-check
    n = lib.rave_struct_sizes(None, 0)
    buf = (i64 * n)()
    lib.rave_struct_sizes(buf, n)
    native = list(buf)
    mine = [C.sizeof(s) for s in STRUCTS]
    if native != mine:
        raise ImportError(f"rave_amd ABI mismatch: native struct sizes {native} != ctypes {mine}")
    if lib.rave_abi_version() != ABI_VERSION:
        raise ImportError("rave_amd ABI version mismatch")
    return lib


lib = _load()


def model_config(cfg) -> ModelConfig:
    """rave_amd.config.RaveConfig -> the engine's rave_model_config."""
    c = ModelConfig()
    c.n_band, c.enc_bands, c.capacity = cfg.n_band, cfg.enc_bands, cfg.capacity
    c.latent_size, c.kernel_size, c.speaker_size = cfg.latent_size, cfg.kernel_size, cfg.speaker_size
    if len(cfg.ratios) > MAX_RATIOS or len(cfg.dilations) != len(cfg.ratios):
        raise ValueError("ratios / dilations do not fit the engine's limits")
    c.n_ratios = len(cfg.ratios)
    for i, (r, ds) in enumerate(zip(cfg.ratios, cfg.dilations)):
        if len(ds) > MAX_DILATIONS:
            raise ValueError("too many dilations per stage")
        c.ratios[i] = r
        c.n_dilations[i] = len(ds)
        for j, d in enumerate(ds):
            c.dilations[i][j] = d
    c.amplitude_modulation = int(cfg.amplitude_modulation)
    c.causal = int(cfg.causal)
    c.activation = ACT[cfg.activation]
    c.adain = int(cfg.adain)
    c.leaky_slope = cfg.leaky_slope
    c.conv_bias, c.convt_bias = int(cfg.conv_bias), int(cfg.convt_bias)
    if cfg.noise is not None:
        c.noise = 1
        c.noise_hidden, c.noise_bands = cfg.noise.hidden_size, cfg.noise.noise_bands
        c.n_noise_ratios = len(cfg.noise.ratios)
        for i, r in enumerate(cfg.noise.ratios):
            c.noise_ratios[i] = r
    if cfg.rvq is not None:
        c.rvq_quantizers, c.rvq_codebook_size = cfg.rvq.num_quantizers, cfg.rvq.codebook_size
    c.fuse_units = 1
    return c


def check(rc: int, what: str = "") -> None:
    if rc == RAVE_OK:
        return
    msg = lib.rave_last_error().decode(errors="replace")
    text = f"{what}: {msg}" if what else msg
    if rc in (RAVE_ERR_ARG,):
        raise ValueError(text)
    if rc == RAVE_ERR_UNSUPPORTED:
        raise NotImplementedError(text)
    raise NativeError(f"{text} (status {rc})")


def conv_configs(args: "ConvArgs") -> list:
    """Launch configurations valid for ``args`` (rave_conv1d_configs), without 0."""
    buf = (i32 * 1024)()
    n = int(lib.rave_conv1d_configs(C.byref(args), buf, 1024))
    if n < 0:
        check(n, "conv1d_configs")
    return [int(buf[i]) for i in range(min(n, 1024))]


def conv_chunk(c_in, kernel, stride, dilation, transposed) -> int:
    return int(lib.rave_conv1d_chunk(c_in, kernel, stride, dilation, int(transposed)))


def pack_conv_weight(w, c_in, c_out, kernel, stride, dilation, transposed, out_shift=None,
                     precision=PREC_F32):
    """Host repack (numpy float32, torch layout) -> packed numpy float32 (for
    PREC_SPLIT16 a byte image of f16 fragments + row scales, in 4-byte units).
    ``out_shift`` (ConvTranspose only): stride//2 for torch padding r//2 (default),
    0 for the cached streaming form."""
    if out_shift is None:
        out_shift = stride // 2 if transposed else 0
    import numpy as np
    w = np.ascontiguousarray(w, dtype=np.float32)
    size_fn, pack_fn = ((lib.rave_conv1d_packed_size, lib.rave_conv1d_pack_weight)
                        if precision == PREC_F32 else
                        (lib.rave_conv1d_split_packed_size, lib.rave_conv1d_ring_pack_weight)
                        if precision == PREC_F32_RING else
                        (lib.rave_conv1d_bf3_packed_size, lib.rave_conv1d_bf3_pack_weight)
                        if precision == PREC_BF16X3 else
                        (lib.rave_conv1d_split_packed_size, lib.rave_conv1d_split_pack_weight))
    n = int(size_fn(c_in, c_out, kernel, stride, dilation, int(transposed)))
    if n <= 0:
        raise NotImplementedError(f"unsupported conv shape c_in={c_in} k={kernel} s={stride} d={dilation}")
    out = np.zeros(n, np.float32)
    check(pack_fn(w.ctypes.data, c_in, c_out, kernel, stride, dilation,
                  int(transposed), int(out_shift), out.ctypes.data), "pack_weight")
    return out


def pack_edge_filter(filt, head: bool, n_out_bands: int = 6, f32: bool = False):
    """PQMF filter -> the fused edges' pre-split image (numpy float32):
    head: hkf (16, taps) analysis rows; tail: hki (16, 16, taps).  f32: the
    exact-fp32 image (edges run with precision RAVE_PREC_F32_RING)."""
    import numpy as np
    f = np.ascontiguousarray(filt, dtype=np.float32)
    out = np.zeros(EDGE_FILTER_FLOATS, np.float32)
    if head:
        fn = lib.rave_encoder_head_pack_filter_f32 if f32 else lib.rave_encoder_head_pack_filter
        check(fn(f.ctypes.data, f.shape[0], f.shape[-1], int(n_out_bands), out.ctypes.data), "encoder_head_pack_filter")
    else:
        fn = lib.rave_decoder_tail_pack_filter_f32 if f32 else lib.rave_decoder_tail_pack_filter
        check(fn(f.ctypes.data, f.shape[0], f.shape[-1], out.ctypes.data), "decoder_tail_pack_filter")
    return out


def stack_supported(channels: int) -> bool:
    """Fused split-f16 residual stack (rave_residual_stack) available at this width."""
    return bool(lib.rave_stack_supported(int(channels)))


def unit_supported(channels: int, precision: int = PREC_F32) -> bool:
    size_fn = (lib.rave_unit_packed_size if precision == PREC_F32 else lib.rave_unit_bf3_packed_size
               if precision == PREC_BF16X3 else lib.rave_unit_split_packed_size)
    return int(size_fn(int(channels))) > 0


def pack_unit_weight(w1, w2, channels, precision=PREC_F32):
    """Fused residual unit weights: W1 (C, C, 3) and W2 (C, C, 1) -> packed float32
    (PREC_SPLIT16: f16 fragment image + row scales, in 4-byte units; PREC_BF16X3:
    bf16 (hi, lo, mid) fragment image)."""
    import numpy as np
    size_fn, pack_fn = ((lib.rave_unit_packed_size, lib.rave_unit_pack_weight) if precision == PREC_F32
                        else (lib.rave_unit_split_packed_size, lib.rave_unit_ring_pack_weight)
                        if precision == PREC_F32_RING
                        else (lib.rave_unit_bf3_packed_size, lib.rave_unit_bf3_pack_weight)
                        if precision == PREC_BF16X3
                        else (lib.rave_unit_split_packed_size, lib.rave_unit_split_pack_weight))
    n = int(size_fn(int(channels)))
    if n <= 0:
        raise NotImplementedError(f"fused residual unit does not support C={channels}")
    w1 = np.ascontiguousarray(w1, dtype=np.float32)
    w2 = np.ascontiguousarray(w2, dtype=np.float32)
    if w1.shape != (channels, channels, 3) or w2.reshape(channels, channels).shape != (channels, channels):
        raise ValueError("unit weights must be (C, C, 3) and (C, C, 1)")
    out = np.zeros(n, np.float32)
    check(pack_fn(w1.ctypes.data, w2.ctypes.data, int(channels), out.ctypes.data), "unit_pack_weight")
    return out


def struct_payload(args: C.Structure):
    return bytes(C.string_at(C.addressof(args), C.sizeof(args)))
