"""ctypes binding of lib/libmerlin_hip.so (the C ABI in include/merlin_hip.h).

There is no CPU or PyTorch fallback: if the HIP library is missing or fails to
load, importing anything that needs it raises ``MerlinNativeError`` with the
build command.  All device-pointer arguments are torch CUDA(HIP) tensors; every
call is ordered on torch's current stream of the tensor's device.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import gc
import os

import torch  # loads the HIP runtime that libmerlin_hip.so links against (same soname)

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("MERLIN_HIP_LIB", os.path.join(PKG_ROOT, "lib", "libmerlin_hip.so"))

MERLIN_OK = 0
LAYOUT_NCHW = 0
LAYOUT_NHWC = 1
OBS_WORDS = 8
DEVERR_BAD_ACTION = 1
DEVERR_PLACE_OBJ = 2
DEVERR_BAD_TILE = 4  # merlin_tower_codes_conv3 saw a frame that is no observation (merlin_tower_errors)
DEVERR_SLOT_EMPTY = 8  # a reset met an empty look-ahead slot with the step fallback off (merlin_env_set_step_fallback)

DIFFICULTY_IDS = {"easy": 0, "medium": 1, "mediumhard": 2, "hard": 3, "hardest": 4}


class MerlinNativeError(RuntimeError):
    pass


class EnvConfig(C.Structure):
    _fields_ = [
        ("num_envs", C.c_int32),
        ("size", C.c_int32),
        ("difficulty", C.c_int32),
        ("max_steps", C.c_int32),
        ("stuck_penalty", C.c_int32),
        ("max_stay", C.c_int32),
        ("penalty", C.c_double),
        ("exploration_bonus", C.c_int32),
        ("bonus", C.c_double),
        ("reseed_each_reset", C.c_int32),
    ]


_lib = None
# MERLIN_ABI_VERSION of include/merlin_hip.h this binding is written against (3: the compact 4^9 + 3 4^8 acting-table
# keys of merlin_tower_codes_conv3 / merlin_tower_all_windows, the plane-operand GEMM entry points)
ABI_VERSION = 3


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MerlinNativeError(
            f"HIP library not found at {LIB_PATH}; build it with "
            f"`make -C {PKG_ROOT}` (hipcc --offload-arch=gfx950)")
    try:
        L = C.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover - depends on the runtime image
        raise MerlinNativeError(f"failed to load {LIB_PATH}: {e}") from e
    vp, i32, i64, u64p = C.c_void_p, C.c_int32, C.c_int64, C.POINTER(C.c_uint64)
    L.merlin_version.restype = C.c_int
    if L.merlin_version() != ABI_VERSION:  # a library built from another header: its tables / layouts differ
        raise MerlinNativeError(f"{LIB_PATH} has ABI version {L.merlin_version()}, this package binds version "
                                f"{ABI_VERSION} (include/merlin_hip.h MERLIN_ABI_VERSION); rebuild it")
    L.merlin_last_error.restype = C.c_char_p
    L.merlin_tile_atlas.argtypes = [vp]
    L.merlin_env_config_layout.argtypes = [C.POINTER(C.c_int64), i32]
    L.merlin_env_config_layout.restype = i64
    L.merlin_env_create.argtypes = [C.POINTER(EnvConfig), C.POINTER(vp)]
    L.merlin_env_destroy.argtypes = [vp]
    L.merlin_env_seed.argtypes = [vp, u64p, i32, vp]
    L.merlin_env_reset.argtypes = [vp, vp, vp, vp]
    L.merlin_env_step.argtypes = [vp, vp, i32, i64, vp, vp, vp, vp, vp, vp, vp, i32, vp]
    L.merlin_group_act.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, vp, vp, i32, vp]
    L.merlin_env_act_step.argtypes = [vp, vp, i32, vp, vp, i32, i32, C.c_uint64, vp, i64, i64, vp, vp, vp, vp, vp,
                                      vp, vp, vp, vp, vp, vp]
    L.merlin_env_set_refill_interval.argtypes = [vp, i32]
    L.merlin_env_set_step_fallback.argtypes = [vp, i32]
    L.merlin_env_refill.argtypes = [vp, vp]
    L.merlin_env_get_state.argtypes = [vp, vp, vp, vp, vp]
    L.merlin_env_full_obs.argtypes = [vp, vp, vp]
    L.merlin_env_errors.argtypes = [vp, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), vp]
    L.merlin_obs_expand_f32.argtypes = [vp, vp, i64, vp, C.c_float, i32, vp]
    L.merlin_obs_expand_u8.argtypes = [vp, vp, i64, vp, vp]
    L.merlin_gae.argtypes = [vp, vp, vp, vp, vp, vp, i32, i32, C.c_double, C.c_double, vp, vp]
    L.merlin_adv_normalize.argtypes = [vp, i64, vp, vp, vp]
    L.merlin_conv1_lut_fwd.argtypes = [vp, vp, i64, vp, vp, i32, vp, vp]
    L.merlin_conv1_lut_bwd.argtypes = [vp, vp, i64, vp, vp, i32, vp, vp, vp]
    L.merlin_tower_conv2_im2col_fwd.argtypes = [vp, vp, i64, vp, vp, i32, vp, vp]
    L.merlin_tower_conv2_im2col_bwd.argtypes = [vp, vp, i64, vp, vp, vp, i32, vp, vp, vp]
    L.merlin_tower_conv3_im2col_fwd.argtypes = [vp, vp, i64, i32, vp, vp]
    L.merlin_tower_conv3_col2im_bwd.argtypes = [vp, vp, vp, i64, i32, vp, vp]
    L.merlin_tower_conv3_col2im_bwd_chunked.argtypes = [vp, vp, vp, i64, i32, vp, vp, vp]
    L.merlin_tower_conv2_lut_rows.restype = C.c_int
    L.merlin_tower_conv2_lut_fwd.argtypes = [vp, vp, i64, vp, i32, vp, vp]
    L.merlin_tower_conv2_lut_bwd.argtypes = [vp, i64, vp, vp, i32, vp, vp]
    L.merlin_tower_conv2_lut_fwd_grouped.argtypes = [vp, i64, i64, vp, i32, vp, vp]
    L.merlin_tower_conv2_lut_slab_bytes.argtypes = [i32, i64]
    L.merlin_tower_conv2_lut_slab_bytes.restype = i64
    L.merlin_tower_conv2_lut_bwd_grouped.argtypes = [vp, i64, vp, vp, i32, vp, vp, vp]
    L.merlin_tower_window_lut.argtypes = [vp, i64, vp, i32, vp, vp]
    L.merlin_tower_window_conv3.argtypes = [vp, i64, vp, vp, i64, vp, i32, vp, vp]
    L.merlin_tower_window_lut_bias_relu.argtypes = [vp, i64, vp, i32, vp, vp, vp]
    L.merlin_minibatch_patch_maps.argtypes = [vp, vp, i64, i64, vp, i32, vp, vp, vp, vp]
    L.merlin_tower_window_conv3_bits.argtypes = [vp, i64, vp, vp, i64, vp, i32, vp, vp, vp, vp]
    L.merlin_tower_window_conv3_reuse.argtypes = [vp, i64, vp, vp, i64, vp, i32, vp, vp, vp, vp, i32, vp]
    L.merlin_tower_all_windows.restype = i64
    L.merlin_tower_codes_conv3.argtypes = [vp, i64, vp, vp, i32, vp, vp]
    L.merlin_tower_codes_conv3_amax.argtypes = [vp, i64, vp, vp, i32, vp, vp, vp]
    L.merlin_tower_errors.argtypes = [C.POINTER(C.c_uint32), vp]
    L.merlin_segment_sum.argtypes = [vp, i64, vp, vp, i64, vp, i32, i64, vp, i64, i32, vp, i64, vp, i32, vp]
    L.merlin_segment_sum_masked.argtypes = [vp, vp, i64, vp, vp, i64, vp, i32, i64, vp, i64, i32, vp, i64, vp, i32,
                                            vp]
    L.merlin_tower_heads_fwd.argtypes = [vp, i64, i32, vp, i32, vp, vp, vp, vp, vp, vp]
    L.merlin_segment_sum_marked.argtypes = [vp, vp, i64, vp, vp, i64, vp, i32, i64, vp, i64, i32, vp, i64, vp, i32,
                                            vp, vp]
    L.merlin_segment_sum_fused.argtypes = [vp, vp, i64, vp, vp, i64, vp, i32, i64, vp, i64, i32, vp, i64, vp, i32,
                                           vp, vp, vp, vp]
    L.merlin_segment_sum_mask_rows.argtypes = [vp, vp, i64, vp, vp, i64, vp, i32, i64, vp, i64, i32, vp, i64, vp, i32,
                                               vp, vp, vp, vp, vp]
    L.merlin_tower_bias_relu.argtypes = [vp, vp, i64, i32, i32, vp]
    L.merlin_tower_relu_bwd.argtypes = [vp, vp, vp, i64, i32, i32, vp, vp]
    L.merlin_tower_colsum.argtypes = [vp, i64, i32, i64, i64, i32, vp, vp]
    L.merlin_tower_head_bwd.argtypes = [vp, vp, vp, vp, vp, i64, i32, i32, vp, vp, vp, vp, vp, vp]
    L.merlin_tower_head_bwd_planes.argtypes = [vp, vp, vp, vp, vp, i64, i32, i32, vp, vp, vp, vp, vp, vp, vp]
    L.merlin_act_heads.argtypes = [vp, vp, i64, i32, vp, vp, vp, vp, i32, i32, C.c_uint64, vp, i64, i64, vp, vp, vp,
                                   vp]
    L.merlin_ppo_loss_workspace.argtypes = [i64]
    L.merlin_ppo_loss_workspace.restype = i64
    L.merlin_clip_adam_workspace.argtypes = [i32, vp]
    L.merlin_clip_adam_workspace.restype = i64
    L.merlin_clip_adam.argtypes = [i32, vp, vp, vp, vp, vp, vp, C.c_double, C.c_double, C.c_double, C.c_double, C.c_float,
                                   vp, vp, vp]
    L.merlin_ppo_loss.argtypes = [vp, vp, vp, vp, i64, i32, vp, vp, vp, i64, vp, vp, vp, vp, vp, C.c_double,
                                  C.c_double, C.c_double, vp, vp, vp, vp, vp, vp, vp, vp]
    L.merlin_ppo_loss_absmax.argtypes = [vp, vp, vp, vp, i64, i32, vp, vp, vp, i64, vp, vp, vp, vp, vp, C.c_double,
                                         C.c_double, C.c_double, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.merlin_x6_split.argtypes = [vp, i64, vp, vp]
    L.merlin_x6_join.argtypes = [vp, i64, vp, vp]
    L.merlin_x6_gemm_nt.argtypes = [vp, vp, i64, i32, i32, i32, i64, i64, vp, vp, i64, i32, vp]
    L.merlin_x6_tn_slab_floats.argtypes = [i32, i32, i32, i32]
    L.merlin_x6_tn_slab_floats.restype = i64
    L.merlin_x6_gemm_tn.argtypes = [vp, vp, i64, i32, i32, i32, i64, i64, i32, vp, vp, i32, vp]
    L.merlin_h3_amax.argtypes = [vp, i64, i32, i64, vp, vp]
    L.merlin_h3_split.argtypes = [vp, i64, i32, vp, vp, vp]
    L.merlin_h3_gemm_nt.argtypes = [vp, vp, vp, vp, i64, i32, i32, i32, i64, i64, vp, vp, i64, vp, i32, vp]
    L.merlin_h3_gemm_tn.argtypes = [vp, vp, vp, vp, i64, i32, i32, i32, i64, i64, i32, vp, vp, i32, vp]
    L.merlin_h3_gemm_tn_planes.argtypes = [vp, vp, vp, vp, i64, i32, i32, i32, i64, i64, i32, vp, vp, i32, vp]
    L.merlin_h3_gemm_nt_gather.argtypes = [vp, vp, vp, vp, i64, i32, i32, i32, i64, i64, vp, vp, i64, vp, i32, vp]
    L.merlin_h3_gemm_tn_gather.argtypes = [vp, vp, vp, vp, i64, i32, i32, i32, i64, i64, i32, vp, vp, vp, i32, vp]
    L.merlin_h3_gemm_tn_gather_planes_a.argtypes = [vp, vp, vp, vp, i64, i32, i32, i32, i64, i64, i32, vp, vp, vp, i32,
                                                    vp]
    L.merlin_h3_gemm_nt_planes.argtypes = [vp, vp, vp, vp, i64, i32, i32, i32, i64, i64, vp, vp, i64, i32, vp]
    L.merlin_h3_gemm_nt_heads_planes.argtypes = [vp, vp, vp, vp, i64, i32, i32, i64, i64, vp, vp, i64, vp, vp, i32,
                                                 vp, vp, i32, vp]
    L.merlin_h3_gemm_tn_gather_planes.argtypes = [vp, vp, vp, vp, i64, i32, i32, i32, i64, i64, i32, vp, vp, vp, i32,
                                                  vp]
    L.merlin_tower_window_conv3_planes.argtypes = [vp, i64, vp, vp, i64, vp, i32, vp, vp, vp, vp, vp, vp]
    L.merlin_h3_gemm_nt_heads.argtypes = [vp, vp, vp, vp, i64, i32, i32, i64, i64, vp, vp, i64, vp, vp, i32, vp, vp,
                                          i32, vp]
    L.merlin_h3_heads_parts.argtypes = [i32, i32]
    L.merlin_h3_heads_parts.restype = i32
    L.merlin_heads_combine.argtypes = [vp, i32, i64, i32, vp, vp, vp]
    L.merlin_act_draw.argtypes = [vp, i32, i64, vp, vp, i32, i32, C.c_uint64, vp, i64, i64, vp, vp, vp, vp]
    L.merlin_stage_tables_fwd.argtypes = [vp, vp, vp, vp, vp, i32, vp, vp, vp]
    L.merlin_stage_tables_bwd.argtypes = [vp, vp, vp, vp, vp, vp, i32, vp, vp, vp, vp, vp]
    L.merlin_window_gemm_fwd.argtypes = [vp, vp, i32, i64, vp, vp]
    L.merlin_window_gemm_bwd_work.argtypes = [i32, i64]
    L.merlin_window_gemm_bwd_work.restype = i64
    L.merlin_window_gemm_bwd.argtypes = [vp, vp, vp, i32, i64, vp, vp, vp, vp, vp, i64, vp]
    check_env_config_layout(L)
    _lib = L
    return L


def env_config_layout(L=None):
    """(sizeof, field offsets) of the C merlin_env_config, from the library itself."""
    L = L or lib()
    nf = len(EnvConfig._fields_)
    offs = (C.c_int64 * nf)()
    size = int(L.merlin_env_config_layout(offs, nf))
    return size, [int(o) for o in offs]


def check_env_config_layout(L) -> None:
    """The ctypes EnvConfig must be byte-identical to include/merlin_hip.h's merlin_env_config:
    merlin_env_create reads every field, so a shorter binding would be read past its end."""
    size, offs = env_config_layout(L)
    mine = [getattr(EnvConfig, f).offset for f, _ in EnvConfig._fields_]
    if size != C.sizeof(EnvConfig) or offs != mine:
        raise MerlinNativeError(f"EnvConfig layout mismatch: C sizeof {size} offsets {offs}, "
                                f"ctypes sizeof {C.sizeof(EnvConfig)} offsets {mine}")


EXPORTED_SYMBOLS = (
    "merlin_version", "merlin_last_error", "merlin_tile_atlas", "merlin_env_config_layout", "merlin_env_create",
    "merlin_env_destroy", "merlin_env_seed", "merlin_env_reset", "merlin_env_step", "merlin_env_act_step", "merlin_group_act",
    "merlin_env_set_refill_interval", "merlin_env_refill",
    "merlin_env_get_state", "merlin_env_full_obs", "merlin_env_errors", "merlin_env_set_step_fallback", "merlin_env_num_envs", "merlin_env_size",
    "merlin_obs_expand_f32", "merlin_obs_expand_u8", "merlin_gae", "merlin_adv_normalize",
    "merlin_conv1_lut_fwd", "merlin_conv1_lut_bwd", "merlin_tower_conv2_im2col_fwd",
    "merlin_tower_conv2_im2col_bwd", "merlin_tower_conv3_im2col_fwd", "merlin_tower_conv3_col2im_bwd",
    "merlin_tower_conv3_col2im_bwd_chunked", "merlin_tower_conv2_lut_rows", "merlin_tower_conv2_lut_fwd",
    "merlin_tower_conv2_lut_bwd", "merlin_tower_conv2_lut_fwd_grouped", "merlin_tower_conv2_lut_slab_bytes",
    "merlin_tower_conv2_lut_bwd_grouped", "merlin_tower_window_lut", "merlin_tower_window_lut_bias_relu", "merlin_minibatch_patch_maps", "merlin_segment_sum_mask_rows", "merlin_tower_window_conv3",
    "merlin_tower_window_conv3_bits", "merlin_tower_window_conv3_reuse", "merlin_tower_all_windows", "merlin_tower_codes_conv3",
    "merlin_tower_codes_conv3_amax", "merlin_tower_errors",
    "merlin_segment_sum", "merlin_segment_sum_masked", "merlin_segment_sum_marked", "merlin_segment_sum_fused", "merlin_tower_heads_fwd", "merlin_tower_bias_relu", "merlin_tower_relu_bwd", "merlin_tower_head_bwd",
    "merlin_tower_colsum",
    "merlin_ppo_loss_workspace", "merlin_ppo_loss", "merlin_act_heads",
    "merlin_x6_split", "merlin_x6_join", "merlin_x6_gemm_nt", "merlin_x6_tn_slab_floats", "merlin_x6_gemm_tn",
    "merlin_clip_adam_workspace", "merlin_clip_adam",
    "merlin_h3_amax", "merlin_h3_split", "merlin_h3_gemm_nt", "merlin_h3_gemm_tn",
    "merlin_h3_gemm_tn_planes", "merlin_h3_gemm_nt_gather", "merlin_h3_gemm_tn_gather",
    "merlin_h3_gemm_nt_heads", "merlin_h3_heads_parts", "merlin_heads_combine", "merlin_act_draw",
    "merlin_ppo_loss_absmax", "merlin_tower_head_bwd_planes", "merlin_h3_gemm_nt_planes",
    "merlin_h3_gemm_tn_gather_planes_a", "merlin_h3_gemm_nt_heads_planes", "merlin_h3_gemm_tn_gather_planes",
    "merlin_tower_window_conv3_planes", "merlin_window_gemm_bwd_work", "merlin_window_gemm_bwd",
    "merlin_window_gemm_fwd",
)


_CAPTURE_DEPTH = 0
_DEFERRED: list = []

_hip_rt = None
_cu_streams = []  # raw handles of the CU-masked streams (kept for the process's lifetime)


def cu_masked_stream(device, keep) -> torch.cuda.ExternalStream:
    """A stream whose kernels run only on the compute units i with keep(i) true (hipExtStreamCreateWithCUMask;
    bit i of the mask = CU i).  The fast step's weight gradient on such a stream leaves the other CUs to conv3's
    backward sums queued beside it on the main stream (merlin/fast_step.py SIDE_CU_GROUPS)."""
    global _hip_rt
    if _hip_rt is None:
        _hip_rt = C.CDLL("libamdhip64.so")
        _hip_rt.hipExtStreamCreateWithCUMask.argtypes = [C.POINTER(C.c_void_p), C.c_uint32, C.POINTER(C.c_uint32)]
    dev = torch.device(device)
    n = torch.cuda.get_device_properties(dev).multi_processor_count
    words = (n + 31) // 32
    mask = (C.c_uint32 * words)()
    for i in range(n):
        if keep(i):
            mask[i // 32] |= 1 << (i % 32)
    if not any(mask):
        raise MerlinNativeError("cu_masked_stream: empty CU mask")
    h = C.c_void_p()
    with torch.cuda.device(dev):
        err = _hip_rt.hipExtStreamCreateWithCUMask(C.byref(h), words, mask)
    if err != 0:
        raise MerlinNativeError(f"hipExtStreamCreateWithCUMask failed ({err})")
    _cu_streams.append(h.value)
    return torch.cuda.ExternalStream(h.value, device=dev)



@contextlib.contextmanager
def capture_guard():
    """Wrap every HIP-graph capture (the rollout graph, FOMAML's rollout graphs, the fast step's weight stage).
    Python's cyclic GC can run in the middle of a capture, triggered by any allocation, and finalise garbage
    from earlier agents: a MerlinVecEnv's merlin_env_destroy (hipFree) or an old torch.cuda.CUDAGraph destroyed
    mid-capture invalidates it or aborts the process (gpurun_out/t_w.log, round 3).  So: collect first, keep
    the collector off until the capture ends, and have native handles released while a capture is open
    (merlin.envs.MerlinVecEnv.close) queue their release until it has ended."""
    global _CAPTURE_DEPTH
    drain_deferred()
    gc.collect()
    was_enabled = gc.isenabled()
    gc.disable()
    _CAPTURE_DEPTH += 1
    try:
        yield
    finally:
        _CAPTURE_DEPTH -= 1
        if _CAPTURE_DEPTH == 0:
            if was_enabled:
                gc.enable()
            run_deferred()


def capturing() -> bool:
    """A capture is open in this process (capture_guard) or on the current stream."""
    if _CAPTURE_DEPTH > 0:
        return True
    try:
        return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
    except Exception:
        return False


def defer_release(fn) -> None:
    """Run `fn` (a native release: hipFree underneath) now, or after the open capture ends.  Releases queued during a
    capture outside capture_guard (a user's own torch.cuda.graph) run at the next call here, at the next env creation
    or capture_guard entry -- whichever comes first with no capture open."""
    if capturing():
        _DEFERRED.append(fn)
    else:
        run_deferred()
        fn()


def run_deferred() -> None:
    while _DEFERRED:
        _DEFERRED.pop(0)()


def drain_deferred() -> None:
    """Run the queued releases if no capture is open now."""
    if _DEFERRED and not capturing():
        run_deferred()


# span names of the GEMMs timed through the plane-form wrappers (h3 / x6): bench.py prices them against the 16-bit
# MFMA peak with their plane products counted, every other GEMM span against the f32 MFMA peak
H3_SPANS: set = set()
X6_SPANS: set = set()


class KernelTimer:
    """Opt-in HIP-event timing of the library's launches on the current stream (bench.py).
    Each record keeps (name, start event, end event, algorithmic bytes, algorithmic flops); the
    hipBLASLt GEMMs of the towers are timed the same way (flops only)."""

    records: list | None = None
    every = 1
    counts: dict = {}

    @classmethod
    def start(cls, every: int = 1):
        """every: time only each every-th launch of each kernel name (the event records are not free: two
        marker packets per timed launch)."""
        cls.records, cls.every, cls.counts = [], max(1, int(every)), {}

    @classmethod
    def stop(cls):
        """The records, with byte counts given as callables (known on the device only, e.g. conv3's representative
        rows per minibatch) resolved now, after the timed region."""
        recs, cls.records = cls.records, None
        return [(n, e0, e1, nb() if callable(nb) else nb, fl) for n, e0, e1, nb, fl in (recs or [])]

    @classmethod
    def active(cls) -> bool:
        return cls.records is not None

    @classmethod
    def span(cls, name: str, nbytes: int, flops: int = 0):
        # no events inside a HIP-graph capture (the captured rollout, merlin/ppo.py)
        if cls.records is None or torch.cuda.is_current_stream_capturing():
            return _NULL_SPAN
        c = cls.counts.get(name, 0)
        cls.counts[name] = c + 1
        if c % cls.every:
            return _NULL_SPAN
        return _Span(name, nbytes, flops)


class _Span:
    def __init__(self, name, nbytes, flops=0):
        self.name, self.nbytes, self.flops = name, nbytes, flops

    def __enter__(self):
        self.e0 = torch.cuda.Event(enable_timing=True)
        self.e0.record()
        return self

    def __exit__(self, *exc):
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        KernelTimer.records.append((self.name, self.e0, e1, self.nbytes, self.flops))
        return False


class _NullSpan:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


_NULL_SPAN = _NullSpan()


def check(rc: int, what: str = "") -> None:
    if rc != MERLIN_OK:
        msg = lib().merlin_last_error().decode(errors="replace")
        raise MerlinNativeError(f"{what or 'merlin call'} failed (code {rc}): {msg}")


def ptr(t: torch.Tensor | None):
    if t is None:
        return None
    if not t.is_cuda:
        raise MerlinNativeError("merlin HIP kernels need device (cuda/hip) tensors; got a CPU tensor")
    if not t.is_contiguous():
        raise MerlinNativeError("merlin HIP kernels need contiguous tensors")
    return C.c_void_p(t.data_ptr())


def stream_of(t: torch.Tensor):
    return C.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def tile_atlas():
    """uint8[5, 8, 8, 3]: the library's own render of minigrid's 5 reachable tiles."""
    import numpy as np

    a = np.zeros((5, 8, 8, 3), dtype=np.uint8)
    check(lib().merlin_tile_atlas(a.ctypes.data_as(C.c_void_p)), "merlin_tile_atlas")
    return a


# ---------------------------------------------------------------------------
# observation expansion / GAE wrappers (device tensors)

def expand_obs(codes: torch.Tensor, index: torch.Tensor | None = None, out: torch.Tensor | None = None,
               scale: float = 1.0, layout: str = "nchw") -> torch.Tensor:
    """codes int32[*, 8] -> float32 [n, 3, 56, 56] (nchw) or [n, 56, 56, 3] (nhwc)."""
    n = int(index.numel()) if index is not None else int(codes.shape[0])
    lay = LAYOUT_NCHW if layout == "nchw" else LAYOUT_NHWC
    shape = (n, 3, 56, 56) if lay == LAYOUT_NCHW else (n, 56, 56, 3)
    if out is None:
        out = torch.empty(shape, dtype=torch.float32, device=codes.device)
    assert out.shape == shape and out.dtype == torch.float32
    assert codes.dtype == torch.int32 and codes.shape[-1] == OBS_WORDS
    if index is not None:
        assert index.dtype == torch.int64
    check(lib().merlin_obs_expand_f32(ptr(codes), ptr(index), n, ptr(out), float(scale), lay,
                                      stream_of(codes)), "merlin_obs_expand_f32")
    return out


def expand_obs_u8(codes: torch.Tensor, index: torch.Tensor | None = None) -> torch.Tensor:
    """codes int32[*, 8] -> uint8 [n, 56, 56, 3]: the RGBImgPartialObsWrapper frame."""
    n = int(index.numel()) if index is not None else int(codes.shape[0])
    out = torch.empty((n, 56, 56, 3), dtype=torch.uint8, device=codes.device)
    check(lib().merlin_obs_expand_u8(ptr(codes), ptr(index), n, ptr(out), stream_of(codes)),
          "merlin_obs_expand_u8")
    return out


def gae(rewards, values, dones, last_value, gamma, lam, adv=None, ret=None, stats=None):
    """[T, N] (or [T]) f32 device tensors -> (adv, returns); stats (f64[3]) receives
    (count, sum, sum of squares) of adv when given."""
    T = int(rewards.shape[0])
    N = int(rewards.numel() // T)
    adv = torch.empty_like(rewards) if adv is None else adv
    ret = torch.empty_like(rewards) if ret is None else ret
    last = last_value.reshape(-1).to(torch.float32).contiguous()
    assert last.numel() == N
    for t in (rewards, values, dones):
        assert t.dtype == torch.float32 and t.numel() == T * N
    check(lib().merlin_gae(ptr(rewards), ptr(values), ptr(dones), ptr(last), ptr(adv), ptr(ret), T, N,
                           float(gamma), float(lam), ptr(stats), stream_of(rewards)), "merlin_gae")
    return adv, ret


def adv_normalize(adv: torch.Tensor, stats: torch.Tensor, out: torch.Tensor | None = None):
    out = torch.empty_like(adv) if out is None else out
    check(lib().merlin_adv_normalize(ptr(adv), int(adv.numel()), ptr(stats), ptr(out), stream_of(adv)),
          "merlin_adv_normalize")
    return out


def conv1_lut_fwd(codes: torch.Tensor, index: torch.Tensor | None, tables: torch.Tensor, bias: torch.Tensor,
                  out: torch.Tensor | None = None) -> torch.Tensor:
    """relu(conv1(frame)) of each tower from tile codes: tables f32[T, 32, 4, 20], bias f32[T, 32]
    -> f32[T, n, 32, 13, 13]."""
    T = int(tables.shape[0])
    n = int(index.numel()) if index is not None else int(codes.shape[0])
    if out is None:
        out = torch.empty((T, n, 32, 13, 13), dtype=torch.float32, device=codes.device)
    assert tables.shape == (T, 32, 4, 20) and bias.shape == (T, 32) and out.shape == (T, n, 32, 13, 13)
    check(lib().merlin_conv1_lut_fwd(ptr(codes), ptr(index), n, ptr(tables), ptr(bias), T, ptr(out),
                                     stream_of(codes)), "merlin_conv1_lut_fwd")
    return out


def conv1_lut_bwd(codes: torch.Tensor, index: torch.Tensor | None, act: torch.Tensor, grad: torch.Tensor):
    """(dtables f32[T, 32, 4, 20], dbias f32[T, 32]) for dz = grad * (act > 0)."""
    T = int(act.shape[0])
    n = int(act.shape[1])
    dt = torch.empty((T, 32, 4, 20), dtype=torch.float32, device=act.device)
    db = torch.empty((T, 32), dtype=torch.float32, device=act.device)
    check(lib().merlin_conv1_lut_bwd(ptr(codes), ptr(index), n, ptr(act), ptr(grad), T, ptr(dt), ptr(db),
                                     stream_of(act)), "merlin_conv1_lut_bwd")
    return dt, db


# -- tower stages around the conv2 / conv3 GEMMs -------------------------------------------
def conv2_im2col_fwd(codes, index, tables, bias):
    """-> A2 f32[T, n*25, 512]: conv2's im2col rows of relu(conv1) built from tile codes."""
    T = int(tables.shape[0])
    n = int(index.numel()) if index is not None else int(codes.shape[0])
    out = torch.empty((T, n * 25, 512), dtype=torch.float32, device=codes.device)
    # algorithmic bytes: A2 written (T*25*512*4 per frame) + codes (32) + index (8) per frame
    with KernelTimer.span("k_conv1_im2col_fwd", n * (T * 25 * 512 * 4 + 32 + (8 if index is not None else 0))):
        check(lib().merlin_tower_conv2_im2col_fwd(ptr(codes), ptr(index), n, ptr(tables), ptr(bias), T,
                                                  ptr(out), stream_of(codes)), "merlin_tower_conv2_im2col_fwd")
    return out


def conv2_im2col_bwd(codes, index, tables, bias, dA2):
    T = int(tables.shape[0])
    n = int(dA2.shape[1]) // 25
    dt = torch.empty((T, 32, 4, 20), dtype=torch.float32, device=dA2.device)
    db = torch.empty((T, 32), dtype=torch.float32, device=dA2.device)
    with KernelTimer.span("k_conv1_im2col_bwd", n * (T * 25 * 512 * 4 + 32 + (8 if index is not None else 0))):
        check(lib().merlin_tower_conv2_im2col_bwd(ptr(codes), ptr(index), n, ptr(tables), ptr(bias), ptr(dA2),
                                                  T, ptr(dt), ptr(db), stream_of(dA2)),
              "merlin_tower_conv2_im2col_bwd")
    return dt, db


def conv3_im2col_fwd(Z2, b2):
    """Z2 f32[T, n*25, 64], b2 f32[T, 64] -> A3 f32[T, n*9, 576] (bias + ReLU fused)."""
    T = int(Z2.shape[0])
    n = int(Z2.shape[1]) // 25
    out = torch.empty((T, n * 9, 576), dtype=torch.float32, device=Z2.device)
    with KernelTimer.span("k_im2col3_fwd", n * T * (25 * 64 + 9 * 576) * 4):
        check(lib().merlin_tower_conv3_im2col_fwd(ptr(Z2), ptr(b2), n, T, ptr(out), stream_of(Z2)),
              "merlin_tower_conv3_im2col_fwd")
    return out


def conv3_col2im_bwd(dA3, Z2, b2):
    T = int(Z2.shape[0])
    n = int(Z2.shape[1]) // 25
    out = torch.empty_like(Z2)
    with KernelTimer.span("k_col2im3_bwd", n * T * (9 * 576 + 2 * 25 * 64) * 4):
        check(lib().merlin_tower_conv3_col2im_bwd(ptr(dA3), ptr(Z2), ptr(b2), n, T, ptr(out), stream_of(Z2)),
              "merlin_tower_conv3_col2im_bwd")
    return out


def conv3_col2im_bwd_chunked(dA3, Z2, b2):
    """(dZ2c, absmax): dZ2 = [Z2 + b2 > 0] * col2im(dA3) chunk-major f32[T, 16, n*25, 4] (conv2_lut_bwd's
    input) and int32[1] = float bits of max |dZ2| (the histogram's fixed-point scale)."""
    T = int(Z2.shape[0])
    n = int(Z2.shape[1]) // 25
    out = torch.empty((T, 16, n * 25, 4), dtype=torch.float32, device=Z2.device)
    absmax = torch.empty(1, dtype=torch.int32, device=Z2.device)
    with KernelTimer.span("k_col2im3_bwd", n * T * (9 * 576 + 2 * 25 * 64) * 4):
        check(lib().merlin_tower_conv3_col2im_bwd_chunked(ptr(dA3), ptr(Z2), ptr(b2), n, T, ptr(out), ptr(absmax),
                                                          stream_of(Z2)), "merlin_tower_conv3_col2im_bwd_chunked")
    return out, absmax


LUT2_ROWS = 2720


def conv2_lut_fwd(codes, index, tables):
    """Z2 f32[T, n*25, 64] = conv2(relu(conv1(frame))) (no conv2 bias) by table lookups;
    tables f32[T, 2720, 64] (merlin.actor_critic.conv2_tables)."""
    T = int(tables.shape[0])
    n = int(index.numel()) if index is not None else int(codes.shape[0])
    assert tables.shape == (T, LUT2_ROWS, 64) and tables.dtype == torch.float32
    assert codes.dtype == torch.int32 and codes.shape[-1] == OBS_WORDS
    if index is not None:
        assert index.dtype == torch.int64
    out = torch.empty((T, n * 25, 64), dtype=torch.float32, device=codes.device)
    # algorithmic bytes per frame: codes 32 (+ index 8) + Z2 written T*25*64*4; the
    # 16 table rows per output position are L2-resident gathers (reported separately)
    with KernelTimer.span("k_conv2_lut_fwd", n * (T * 25 * 64 * 4 + 32 + (8 if index is not None else 0))):
        check(lib().merlin_tower_conv2_lut_fwd(ptr(codes), ptr(index), n, ptr(tables), T, ptr(out),
                                               stream_of(codes)), "merlin_tower_conv2_lut_fwd")
    return out


def conv2_lut_fwd_grouped(codes, tables, group_frames: int):
    """Grouped conv2_lut_fwd: codes int32 [G * group_frames, 8] (group g's frames contiguous), tables
    f32 [2G, 2720, 64] (towers 2g / 2g+1 = group g's actor / critic) -> Z2 f32 [2G, group_frames*25, 64]."""
    T = int(tables.shape[0])
    n = int(codes.shape[0])
    assert T % 2 == 0 and n == (T // 2) * group_frames, (T, n, group_frames)
    assert tables.shape == (T, LUT2_ROWS, 64) and tables.dtype == torch.float32 and tables.is_contiguous()
    assert codes.dtype == torch.int32 and codes.shape[-1] == OBS_WORDS and codes.is_contiguous()
    out = torch.empty((T, group_frames * 25, 64), dtype=torch.float32, device=codes.device)
    with KernelTimer.span("k_conv2_lut_fwd", n * (2 * 25 * 64 * 4 + 32)):
        check(lib().merlin_tower_conv2_lut_fwd_grouped(ptr(codes), n, int(group_frames), ptr(tables), T, ptr(out),
                                                       stream_of(codes)), "merlin_tower_conv2_lut_fwd_grouped")
    return out


_SLABS = {}


def conv2_lut_bwd_grouped(codes, dZ2c, absmax):
    """Grouped conv2_lut_bwd: dtables f32 [2G, 2720, 64] from chunk-major dZ2c f32 [2G, 16, F*25, 4]
    (F = frames per group) of frames codes [G * F, 8] (group g's rows contiguous)."""
    T = int(dZ2c.shape[0])
    F = int(dZ2c.shape[2]) // 25
    assert codes.dtype == torch.int32 and codes.shape == ((T // 2) * F, OBS_WORDS) and codes.is_contiguous()
    nbytes = int(lib().merlin_tower_conv2_lut_slab_bytes(T, F))
    key = dZ2c.device
    slabs = _SLABS.get(key)
    if slabs is None or slabs.numel() < nbytes:
        slabs = _SLABS[key] = torch.empty(nbytes, dtype=torch.uint8, device=dZ2c.device)
    dt = torch.empty((T, LUT2_ROWS, 64), dtype=torch.float32, device=dZ2c.device)
    with KernelTimer.span("k_conv2_lut_hist", F * (T * 25 * 64 * 4 + 16 * T * 32)):
        check(lib().merlin_tower_conv2_lut_bwd_grouped(ptr(codes), F, ptr(dZ2c), ptr(absmax), T, ptr(dt), ptr(slabs),
                                                       stream_of(dZ2c)), "merlin_tower_conv2_lut_bwd_grouped")
    return dt


def conv2_lut_bwd(codes, dZ2c, absmax=None):
    """dtables f32[T, 2720, 64] from chunk-major dZ2c f32[T, 16, n*25, 4] of frames codes[0:n]
    (the minibatch's own code rows); absmax int32[1] = float bits of an upper bound on
    max |dZ2c| (computed here when not given)."""
    T = int(dZ2c.shape[0])
    n = int(dZ2c.shape[2]) // 25
    assert codes.dtype == torch.int32 and codes.shape[-1] == OBS_WORDS and codes.shape[0] >= n
    if absmax is None:
        absmax = dZ2c.abs().amax().reshape(1).view(torch.int32) if dZ2c.numel() else \
            torch.zeros(1, dtype=torch.int32, device=dZ2c.device)
    dt = torch.empty((T, LUT2_ROWS, 64), dtype=torch.float32, device=dZ2c.device)
    # algorithmic bytes per frame: dZ2 read once (T*25*64*4) + its code row per 4-channel slice block
    with KernelTimer.span("k_conv2_lut_hist", n * (T * 25 * 64 * 4 + 16 * T * 32)):
        check(lib().merlin_tower_conv2_lut_bwd(ptr(codes), n, ptr(dZ2c), ptr(absmax), T, ptr(dt),
                                               stream_of(dZ2c)), "merlin_tower_conv2_lut_bwd")
    return dt


# -- receptive-field windows (merlin/windows.py, csrc/merlin_window.hip) -----------------------
def window_lut(rows, tables, bias=None):
    """Z2w f32[T, nw, 64]: the sum of the 16 conv2-table rows rows[w] (int32 [nw, 16]) of
    tables f32[T, 2720, 64] for every window w; with bias f32[T, 64]: relu(Z2w + bias) instead (bias_relu_ fused,
    merlin_tower_window_lut_bias_relu)."""
    T, nw = int(tables.shape[0]), int(rows.shape[0])
    assert tables.shape == (T, LUT2_ROWS, 64) and tables.dtype == torch.float32
    assert rows.dtype == torch.int32 and rows.shape == (nw, 16)
    out = torch.empty((T, nw, 64), dtype=torch.float32, device=tables.device)
    # algorithmic bytes: row indices + Z2w written (table rows are L2-resident gathers)
    # the rollout's all-windows table (5^9 rows) is its own kernel instantiation and span (k_window_lut<1>)
    with KernelTimer.span("k_window_lut_all" if nw == ALL_WINDOWS else "k_window_lut", nw * (64 + T * 256)):
        if bias is not None:
            assert bias.shape == (T, 64) and bias.dtype == torch.float32 and bias.is_contiguous()
            check(lib().merlin_tower_window_lut_bias_relu(ptr(rows), nw, ptr(tables), T, ptr(bias), ptr(out),
                                                          stream_of(tables)), "merlin_tower_window_lut_bias_relu")
        else:
            check(lib().merlin_tower_window_lut(ptr(rows), nw, ptr(tables), T, ptr(out), stream_of(tables)),
                  "merlin_tower_window_lut")
    return out


_COLMAX_WS: dict = {}


def window_conv3_planes(Q, wid, groups, b3, rep_row, bound, n_reps=None):
    """(Y3 planes int16[T, n*9, 128], mask int64[T, n*9]): window_conv3(bits=True, rep_row=..., copy=0) with the
    representatives' rows written as h3 planes (merlin_tower_window_conv3_planes), scaled by bound int32[T] (written:
    float bits of relu(b3 + sum over taps of Q's column maxima) per tower, >= every Y3 value).  Only the
    representatives' rows hold data (read through rep_row, as with copy=0)."""
    T, nw = int(Q.shape[0]), int(Q.shape[1])
    n = int(groups.numel())
    assert Q.shape[2] == 576 and Q.dtype == torch.float32 and Q.is_contiguous() and b3.shape == (T, 64) and T <= 2
    assert wid.dtype == torch.int32 and wid.shape[1] == 25 and groups.dtype == torch.int64
    assert rep_row.dtype == torch.int32 and rep_row.is_contiguous() and rep_row.numel() == n * 9
    assert bound.dtype == torch.int32 and bound.numel() >= T
    dev = Q.device
    ws = _COLMAX_WS.get(dev)
    if ws is None:
        ws = _COLMAX_WS[dev] = torch.empty(2 * 64 * 576, dtype=torch.int32, device=dev)  # per-block column maxima
    out = torch.empty((T, n * 9, 128), dtype=torch.int16, device=dev)
    mask = torch.empty((T, n * 9), dtype=torch.int64, device=dev)
    if POISON_PARTIAL:
        out.fill_(-1)
        mask.fill_(-1)
    fixed = n * 144 + 2 * T * nw * 576 * 4  # ids + Q read twice (column maxima, then the gathers' first touch)
    nb = (lambda: T * int(n_reps) * 264 + fixed) if n_reps is not None else T * n * 9 * 264 + fixed
    with KernelTimer.span("k_window_conv3", nb):
        check(lib().merlin_tower_window_conv3_planes(ptr(Q), nw, ptr(wid), ptr(groups), n, ptr(b3), T, ptr(out),
                                                     ptr(mask), ptr(rep_row), ptr(ws), ptr(bound), stream_of(Q)),
              "merlin_tower_window_conv3_planes")
    return out, mask


def window_conv3(Q, wid, groups, b3, bits: bool = False, rows: int | None = None, amax=None, rep_row=None,
                 copy: int = 3, n_reps=None):
    """Y3 f32[T, n*9, 64] = relu(conv3) rows (k, p3) of frames groups[k] from
    Q f32[T, nw, 576], the per-window, per-tap conv3 partial sums (merlin/windows.py).
    bits: also return the rows' ReLU masks, int64[T, n*9] (bit co = Y3 > 0).  rows >= n: the
    outputs hold `rows` frames, those past n zero (Y3) / unwritten (bits).  amax (with bits): int32[T],
    zeroed by the caller, receives max |Y3| per tower as float bits (h3_amax's format).
    rep_row (int32 [n*9], MinibatchWindows.rep_row: per row, a row holding the same 5x5-tile patch): each distinct
    patch of the rows computed once and copied to the rows sharing it (merlin_tower_window_conv3_reuse; same
    outputs); copy (bit 0 Y3 rows, bit 1 mask words) < 3 leaves the other rows' Y3 / masks unwritten: THE RETURNED
    Y3 / MASK THEN HOLD VALID DATA ONLY IN THE REPRESENTATIVE ROWS (rep_row[r] == r) -- read row r as
    Y3[:, rep_row[r]] (the gathered-row GEMMs and merlin_segment_sum_mask_rows do); with POISON_PARTIAL set, the
    unwritten rows are filled with NaN / all-ones words first, so a direct reader shows up in tests.
    n_reps (int32/int64 0-dim device tensor, MinibatchWindows.n_reps, bench timing only): the number of
    representative rows, for the span's algorithmic bytes (256 + 8 B per representative row and tower)."""
    T, nw = int(Q.shape[0]), int(Q.shape[1])
    n = int(groups.numel())
    R = n if rows is None else int(rows)
    assert Q.shape[2] == 576 and Q.dtype == torch.float32 and b3.shape == (T, 64) and R >= n
    assert wid.dtype == torch.int32 and wid.shape[1] == 25 and groups.dtype == torch.int64
    out = torch.empty((T, R * 9, 64), dtype=torch.float32, device=Q.device)
    if R > n:
        out[:, n * 9:].zero_()
    # algorithmic bytes: Y3 written, the frames' ids and window ids, Q read once (its 81 row
    # gathers per frame and tower are L2 / Infinity-Cache hits)
    if rep_row is not None:
        assert bits and R == n and T <= 2
        assert rep_row.dtype == torch.int32 and rep_row.is_contiguous() and rep_row.numel() == n * 9
        mask = torch.empty((T, R * 9), dtype=torch.int64, device=Q.device)
        if POISON_PARTIAL and copy < 3:
            out.fill_(float("nan"))
            mask.fill_(-1)
        fixed = n * 144 + T * nw * 576 * 4  # ids (window ids, group, rep_row) + Q read once
        if copy < 3 and n_reps is not None:  # only the representatives' rows are computed and written
            nb = (lambda: T * int(n_reps) * 264 + fixed)
        else:
            nb = T * n * 9 * 264 + fixed
        with KernelTimer.span("k_window_conv3", nb):
            check(lib().merlin_tower_window_conv3_reuse(ptr(Q), nw, ptr(wid), ptr(groups), n, ptr(b3), T, ptr(out),
                                                        ptr(mask), ptr(amax), ptr(rep_row), int(copy),
                                                        stream_of(Q)),
                  "merlin_tower_window_conv3_reuse")
        return out, mask
    if bits:
        mask = torch.empty((T, R * 9), dtype=torch.int64, device=Q.device)
        with KernelTimer.span("k_window_conv3", T * n * 9 * 264 + n * 108 + T * nw * 576 * 4):
            check(lib().merlin_tower_window_conv3_bits(ptr(Q), nw, ptr(wid), ptr(groups), n, ptr(b3), T, ptr(out),
                                                       ptr(mask), ptr(amax), stream_of(Q)),
                  "merlin_tower_window_conv3_bits")
        return out, mask
    with KernelTimer.span("k_window_conv3", T * n * 9 * 256 + n * 108 + T * nw * 576 * 4):
        check(lib().merlin_tower_window_conv3(ptr(Q), nw, ptr(wid), ptr(groups), n, ptr(b3), T, ptr(out),
                                              stream_of(Q)), "merlin_tower_window_conv3")
    return out


ALL_WINDOWS = 4 ** 9 + 3 * 4 ** 8  # merlin_tower_all_windows(): the acting table's compact keys
# debug: window_conv3 fills the rows it leaves unwritten (copy < 3) with NaN / all-ones mask words
POISON_PARTIAL = os.environ.get("MERLIN_POISON_PARTIAL", "0") == "1"


def minibatch_patch_maps(kid, group_keys, num_frames, group_offsets, nmb, num_patches):
    """(kmap int32 [nmb, K], rep_row int32 [G * 9]) of WindowPlan._bulk_minibatches in two launches
    (merlin_minibatch_patch_maps): kid int32 [F, 9], group_keys int64 [G] (minibatch * F + frame), group_offsets
    int64 [nmb] (first group of each minibatch)."""
    G, K = int(group_keys.numel()), int(num_patches)
    dev = group_keys.device
    assert kid.dtype == torch.int32 and kid.is_contiguous() and group_keys.dtype == torch.int64
    assert group_offsets.dtype == torch.int64 and group_offsets.numel() >= nmb
    kmap = torch.full((nmb, K), -1, dtype=torch.int32, device=dev)
    rmap = torch.empty((nmb, K), dtype=torch.int32, device=dev)
    rep_row = torch.empty(G * 9, dtype=torch.int32, device=dev)
    check(lib().merlin_minibatch_patch_maps(ptr(kid), ptr(group_keys), G, int(num_frames), ptr(group_offsets), K,
                                            ptr(kmap), ptr(rmap), ptr(rep_row), stream_of(group_keys)),
          "merlin_minibatch_patch_maps")
    return kmap, rep_row


def window_conv3_copy_masks(Y3, bits, rep_row):
    """The mask words of the rows that are not their patch's representative, copied from it (the second half of
    window_conv3(rep_row=..., copy=2), for a launch on another stream after the representatives' one)."""
    T, rows = int(bits.shape[0]), int(bits.shape[1])
    n = rows // 9
    assert bits.dtype == torch.int64 and rep_row.dtype == torch.int32 and rep_row.numel() == rows
    with KernelTimer.span("k_window_conv3_copy", T * rows * 12):
        check(lib().merlin_tower_window_conv3_reuse(None, 0, None, None, n, None, T, ptr(Y3), ptr(bits), None,
                                                    ptr(rep_row), 6, stream_of(bits)),
              "merlin_tower_window_conv3_reuse")
    return bits


def codes_conv3(codes, Qall, b3, amax=None):
    """Y3 f32[T, n*9, 64]: relu(conv3) rows (k, p3) of frames codes[k] (int32 [n, 8]) from Qall
    f32[T, ALL_WINDOWS, 576], the per-window, per-tap conv3 partial sums of every window an observation can hold
    (compact keys: merlin/windows.py compact_window_keys)
    (merlin_tower_codes_conv3).  amax (int32 [T], zeroed by the caller): receives max |Y3| per tower as float
    bits (h3_amax's format)."""
    T, n = int(Qall.shape[0]), int(codes.shape[0])
    assert Qall.shape == (T, ALL_WINDOWS, 576) and Qall.dtype == torch.float32 and Qall.is_contiguous()
    assert codes.dtype == torch.int32 and codes.shape[1] == 8 and codes.is_contiguous() and b3.shape == (T, 64)
    if amax is not None:
        assert amax.dtype == torch.int32 and amax.numel() >= T
    out = torch.empty((T, n * 9, 64), dtype=torch.float32, device=Qall.device)
    # algorithmic bytes: codes read + Y3 written (the 81 Qall rows per frame and tower come from the
    # few thousand windows a rollout holds: cache-resident gathers, rocprofv3 PMC ~38 MB per launch)
    with KernelTimer.span("k_codes_conv3", n * 32 + T * n * 9 * 256):
        check(lib().merlin_tower_codes_conv3_amax(ptr(codes), n, ptr(Qall), ptr(b3), T, ptr(out), ptr(amax),
                                                  stream_of(Qall)), "merlin_tower_codes_conv3_amax")
    return out


SEG_ACCUMULATE, SEG_NO_FILL, SEG_MASK_BITS = 1, 2, 4  # include/merlin_hip.h
SEG_ROLE_SHIFT = 8
# the conv3-backward passes get their own kernel instantiations (names in rocprofv3 profiles)
SEG_ROLES = {"k_seg_sum_R": 1, "k_seg_sum_S": 2, "k_seg_sum_dQ": 3, "k_seg_sum_dT2": 4}


# the destinations that span items finished inside the segmented-sum launch (merlin_segment_sum_fused: write-through
# carries and an arrival counter per row), not by a second k_seg_fix launch; the same bits either way
SEG_FUSED = True



def tower_errors(device=None, raise_on_error: bool = True) -> int:
    """The device error flags of the tower kernels since the last call (merlin_tower_errors; clears them).
    DEVERR_BAD_TILE: the acting path's compact conv3 table was handed a frame that is not an observation."""
    flags = C.c_uint32()
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    with torch.cuda.device(dev):
        check(lib().merlin_tower_errors(C.byref(flags), C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)),
              "merlin_tower_errors")
    if raise_on_error and flags.value & DEVERR_BAD_TILE:
        raise MerlinNativeError("merlin_tower_codes_conv3: a frame without the agent tile at view cell (3, 6), or with "
                                "it elsewhere -- not an observation; its windows were read as other windows")
    return flags.value

def segment_sum(src, plan, out_rows: int, slot=None, sub: int = 1, name: str = "k_seg_sum", out=None,
                accumulate: bool = False, carry=None, mask=None, fill: bool = True, mark=None, mask_rows=None):
    """out f32[T, out_rows, 64]: out[t][key] = the sum, in entry order, of src[t][row(e)] over
    the plan's entries e with that key (merlin.windows.SegmentPlan); row(e) = idx[e], or
    slot[idx[e] // sub] * sub + idx[e] % sub with entries whose slot is -1 skipped.  With
    accumulate the sums are added to `out` (a list split over source blocks, in call order).
    mask (same shape as src): sum ReLU-backward rows, src where mask > 0 else 0; or the same mask as
    int64 [T, src_rows] bit words (window_conv3(bits=True)).  fill=False leaves the rows of keys
    without a live entry unwritten (merlin_segment_sum_masked).  mark (int32 [out_rows], preset to -1):
    mark[key] = key for every key that received a live entry (merlin_segment_sum_marked), the slot map of
    a following pass over these rows.  mask_rows (int32 [src_rows], with bit-word masks): row r's mask word is
    mask[t][mask_rows[r]] (merlin_segment_sum_mask_rows; conv3's patch representatives)."""
    T, src_rows = int(src.shape[0]), int(src.shape[1])
    assert src.shape[2] == 64 and src.dtype == torch.float32 and src.is_contiguous()
    mask_bits = mask is not None and mask.dtype == torch.int64
    if mask_bits:
        assert mask.shape == (T, src_rows) and mask.is_contiguous()
    elif mask is not None:
        assert mask.shape == src.shape and mask.dtype == torch.float32 and mask.is_contiguous()
    if slot is not None:
        assert slot.dtype == torch.int32
    if out is None:
        assert not accumulate
        out = torch.empty((T, out_rows, 64), dtype=torch.float32, device=src.device)
    assert out.shape == (T, out_rows, 64) and out.dtype == torch.float32 and out.is_contiguous()
    need = T * max(plan.nitems, 1) * 128
    if carry is None or carry.numel() < need:
        carry = torch.empty(need, dtype=torch.float32, device=src.device)
    # algorithmic bytes: the entry lists (+ slot lookups), src (and mask) read once, out written
    mrow = 0 if mask is None else (8 if mask_bits else 256)
    nb = plan.nnz * (8 + (4 if slot is not None else 0)) + T * (src_rows * (256 + mrow) + out_rows * 256)
    flags = (SEG_ACCUMULATE if accumulate else 0) | (0 if fill else SEG_NO_FILL) | (SEG_MASK_BITS if mask_bits else 0)
    flags |= SEG_ROLES.get(name, 0) << SEG_ROLE_SHIFT
    if mark is not None:
        assert mark.dtype == torch.int32 and mark.shape == (out_rows,) and mark.is_contiguous()
    fused = SEG_FUSED and getattr(plan, "counters", None) is not None
    if mask_rows is not None:
        assert mask_bits and mask_rows.dtype == torch.int32 and mask_rows.numel() == src_rows
        with KernelTimer.span(name, nb):
            check(lib().merlin_segment_sum_mask_rows(ptr(src), ptr(mask), src_rows, ptr(plan.idx), ptr(plan.key),
                                                     plan.nnz, ptr(slot), int(sub), plan.item_len, ptr(plan.fix),
                                                     int(plan.fix.shape[0]), T, ptr(out), int(out_rows), ptr(carry),
                                                     flags, ptr(mark), ptr(plan.head_fix) if fused else None,
                                                     ptr(plan.counters) if fused else None,
                                                     ptr(mask_rows), stream_of(src)), "merlin_segment_sum_mask_rows")
        return out
    with KernelTimer.span(name, nb):
        check(lib().merlin_segment_sum_fused(ptr(src), ptr(mask), src_rows, ptr(plan.idx), ptr(plan.key), plan.nnz,
                                             ptr(slot), int(sub), plan.item_len, ptr(plan.fix),
                                             int(plan.fix.shape[0]), T, ptr(out), int(out_rows), ptr(carry), flags,
                                             ptr(mark), ptr(plan.head_fix) if fused else None,
                                             ptr(plan.counters) if fused else None, stream_of(src)),
              "merlin_segment_sum_fused")
    return out


# -- GEMM epilogues (csrc/merlin_head.hip) -------------------------------------------------------
def bias_relu_(z, bias):
    """z f32[T, rows, cols] = relu(z + bias[t]) in place (bias f32[T, cols])."""
    T, rows, cols = (int(x) for x in z.shape)
    assert z.dtype == torch.float32 and bias.shape == (T, cols) and bias.dtype == torch.float32
    with KernelTimer.span("k_bias_relu", 2 * z.numel() * 4):
        check(lib().merlin_tower_bias_relu(ptr(z), ptr(bias), rows, cols, T, stream_of(z)), "merlin_tower_bias_relu")
    return z


def relu_bwd(y, dy, out=None, out_bias=None):
    """(dz, dbias): dz = [y > 0] * dy (out may be dy itself), dbias f32[T, cols] = column sums of dz."""
    T, rows, cols = (int(x) for x in y.shape)
    assert dy.shape == y.shape and y.dtype == dy.dtype == torch.float32
    dz = torch.empty_like(dy) if out is None else out
    db = torch.empty((T, cols), dtype=torch.float32, device=y.device) if out_bias is None else out_bias
    assert db.shape == (T, cols) and db.is_contiguous()
    with KernelTimer.span("k_relu_bwd_colsum", 3 * y.numel() * 4):
        check(lib().merlin_tower_relu_bwd(ptr(y), ptr(dy), ptr(dz), rows, cols, T, ptr(db), stream_of(y)),
              "merlin_tower_relu_bwd")
    return dz, db


def window_gemm_fwd(a2w, W3r, out=None):
    """Q = a2w W3r (merlin_window_gemm_fwd): a2w f32[T, nw, 64], W3r f32[T, 64, 576] -> f32[T, nw, 576]."""
    T, nw, ci = (int(v) for v in a2w.shape)
    assert ci == 64 and W3r.shape == (T, 64, 576) and a2w.dtype == W3r.dtype == torch.float32
    assert a2w.is_contiguous() and W3r.is_contiguous()
    Q = torch.empty((T, nw, 576), dtype=torch.float32, device=a2w.device) if out is None else out
    assert Q.shape == (T, nw, 576) and Q.is_contiguous()
    with KernelTimer.span("gemm_window_fwd", 0, flops=2 * T * nw * 64 * 576):
        check(lib().merlin_window_gemm_fwd(ptr(a2w), ptr(W3r), T, nw, ptr(Q), stream_of(a2w)),
              "merlin_window_gemm_fwd")
    return Q


_WINBWD_WORK = {}


def window_gemm_bwd(a2w, dQ, W3r, out_da2w=None, out_db2=None, out_dW3r=None, out_db3=None):
    """The window GEMM's backward (merlin_window_gemm_bwd): a2w f32[T, nw, 64], dQ f32[T, nw, 576], W3r f32[T, 64,
    576] -> (da2w = [a2w > 0] * dQ W3r^T, db2 = its column sums f32[T, 64], dW3r = a2w^T dQ f32[T, 64, 576]); with
    out_db3 f32[T, 64] also the column sums of dQ's tap-0 columns (conv3's bias gradient)."""
    T, nw, ci = (int(v) for v in a2w.shape)
    assert ci == 64 and dQ.shape == (T, nw, 576) and W3r.shape == (T, 64, 576)
    assert all(x.dtype == torch.float32 and x.is_contiguous() for x in (a2w, dQ, W3r))
    dev = a2w.device
    da2w = torch.empty_like(a2w) if out_da2w is None else out_da2w
    db2 = torch.empty((T, 64), dtype=torch.float32, device=dev) if out_db2 is None else out_db2
    dW3r = torch.empty((T, 64, 576), dtype=torch.float32, device=dev) if out_dW3r is None else out_dW3r
    assert da2w.shape == a2w.shape and db2.shape == (T, 64) and dW3r.shape == (T, 64, 576)
    assert all(x.dtype == torch.float32 and x.is_contiguous() for x in (da2w, db2, dW3r))
    need = int(lib().merlin_window_gemm_bwd_work(T, nw))
    key = (dev, T)
    work = _WINBWD_WORK.get(key)
    if work is None or work.numel() < need:  # grown once to the largest window count seen (no free inside a capture)
        work = _WINBWD_WORK[key] = torch.empty(max(need, 1 << 20), dtype=torch.float32, device=dev)
    with KernelTimer.span("k_winbwd", (2 * T * nw * (64 + 576) + T * 64 * 576) * 4):
        if out_db3 is not None:
            assert out_db3.shape == (T, 64) and out_db3.dtype == torch.float32 and out_db3.is_contiguous()
        check(lib().merlin_window_gemm_bwd(ptr(a2w), ptr(dQ), ptr(W3r), T, nw, ptr(da2w), ptr(db2), ptr(dW3r),
                                           ptr(out_db3), ptr(work), int(work.numel()), stream_of(a2w)),
              "merlin_window_gemm_bwd")
    return da2w, db2, dW3r


def colsum(x, out=None):
    """x f32[T, rows, cols] (rows may be strided, columns contiguous) -> f32[T, cols] column sums (fixed
    order)."""
    T, rows, cols = (int(v) for v in x.shape)
    assert x.dtype == torch.float32 and x.stride(2) == 1 and x.is_cuda
    if out is None:
        out = torch.empty((T, cols), dtype=torch.float32, device=x.device)
    assert out.shape == (T, cols) and out.is_contiguous()
    with KernelTimer.span("k_colsum", T * rows * cols * 4):
        check(lib().merlin_tower_colsum(C.c_void_p(x.data_ptr()), rows, cols, int(x.stride(1)), int(x.stride(0)), T,
                                        ptr(out), stream_of(x)), "merlin_tower_colsum")
    return out


def heads_fwd(h: torch.Tensor, w_actor: torch.Tensor, w_critic: torch.Tensor, b_actor=None, b_critic=None,
              name: str = "k_heads_fwd"):
    """(logits f32[n, act_dim], value f32[n]) = h[0] w_actor^T (+ b_actor), h[1] w_critic^T (+ b_critic) for h
    f32[2, n, 512] (merlin_tower_heads_fwd: both heads in one pass over h)."""
    assert h.dim() == 3 and h.shape[0] == 2 and h.shape[2] == 512 and h.dtype == torch.float32 and h.is_contiguous()
    n, A = int(h.shape[1]), int(w_actor.shape[0])
    wa, wc = w_actor.detach().contiguous(), w_critic.detach().reshape(-1).contiguous()
    assert wa.shape == (A, 512) and wc.numel() == 512
    ba = None if b_actor is None else b_actor.detach().contiguous()
    bc = None if b_critic is None else b_critic.detach().reshape(-1).contiguous()
    logits = torch.empty((n, A), dtype=torch.float32, device=h.device)
    value = torch.empty(n, dtype=torch.float32, device=h.device)
    with KernelTimer.span(name, h.numel() * 4 + n * (A + 1) * 4):
        check(lib().merlin_tower_heads_fwd(ptr(h), n, 512, ptr(wa), A, ptr(wc), ptr(ba), ptr(bc), ptr(logits),
                                           ptr(value), stream_of(h)), "merlin_tower_heads_fwd")
    return logits, value


def head_bwd(h, dlogits, dvalue, w_actor, w_critic, out_bias=None, out_w_actor=None, out_w_critic=None, amax=None,
             grad_absmax=None, dz_planes=None):
    """Heads backward through fc1's ReLU: h f32[2, n, H] = relu(fc1) of both towers, dlogits
    f32[n, A], dvalue f32[n], w_actor f32[A, H], w_critic f32[1, H] or [H] ->
    (dz f32[2, n, H], dbias f32[2, H], dw_actor f32[A, H], dw_critic f32[H]); the out_* tensors, when
    given, receive the bias / head-weight gradients (e.g. views of a flat gradient buffer).  amax int32[2], zeroed by
    the caller, receives max |dz| per tower as float bits (h3_amax's format).
    grad_absmax int32[9] (ppo_loss's, merlin_tower_head_bwd_planes): dz is written as its h3 planes instead, into
    dz_planes int16[2, n, 2H] (allocated if None; returned in dz's place), and amax[t] receives the bound on max |dz|
    the planes are scaled by."""
    _, n, H = (int(x) for x in h.shape)
    A = int(w_actor.shape[0])
    assert h.shape[0] == 2 and dlogits.shape == (n, A) and dvalue.numel() == n and w_critic.numel() == H
    db = torch.empty((2, H), dtype=torch.float32, device=h.device) if out_bias is None else out_bias
    dwa = torch.empty((A, H), dtype=torch.float32, device=h.device) if out_w_actor is None else out_w_actor
    dwc = torch.empty((H,), dtype=torch.float32, device=h.device) if out_w_critic is None else out_w_critic
    assert db.shape == (2, H) and dwa.shape == (A, H) and dwc.numel() == H
    assert db.is_contiguous() and dwa.is_contiguous() and dwc.is_contiguous()
    if grad_absmax is not None:
        assert amax is not None and amax.dtype == grad_absmax.dtype == torch.int32 and grad_absmax.numel() >= 9
        if dz_planes is None:
            dz_planes = torch.empty((2, n, 2 * H), dtype=torch.int16, device=h.device)
        assert dz_planes.shape == (2, n, 2 * H) and dz_planes.dtype == torch.int16 and dz_planes.is_contiguous()
        with KernelTimer.span("k_head_bwd", 2 * h.numel() * 4 + n * (A + 1) * 4):
            check(lib().merlin_tower_head_bwd_planes(ptr(h), ptr(dlogits), ptr(dvalue), ptr(w_actor), ptr(w_critic),
                                                     n, H, A, ptr(dz_planes), ptr(db), ptr(dwa), ptr(dwc),
                                                     ptr(grad_absmax), ptr(amax), stream_of(h)),
                  "merlin_tower_head_bwd_planes")
        return dz_planes, db, dwa, dwc
    dz = torch.empty_like(h)
    with KernelTimer.span("k_head_bwd", 2 * h.numel() * 4 + n * (A + 1) * 4):
        check(lib().merlin_tower_head_bwd(ptr(h), ptr(dlogits), ptr(dvalue), ptr(w_actor), ptr(w_critic), n, H, A,
                                          ptr(dz), ptr(db), ptr(dwa), ptr(dwc), ptr(amax), stream_of(h)),
              "merlin_tower_head_bwd")
    return dz, db, dwa, dwc


# -- PPO loss (csrc/merlin_loss.hip) -------------------------------------------------------------
def ppo_loss(logits, value, offs, order, frame_of, sample_index, actions, logp_old, adv, ret, clip_eps, vf_coef,
             ent_coef, stats=None, bias_actor=None, bias_critic=None, out_bias_actor=None, out_bias_critic=None,
             grad_absmax=None):
    """(loss f32[], dlogits f32[U, A], dvalue f32[U], dbias_actor f32[A] | None, dbias_critic f32[1] |
    None): the PPO minibatch loss of src/ppo.py:136-150 over the samples of U distinct frames (CSR
    offs int32[U+1] / order int32[n], frame_of int64[n] = the frame of sample i; sample i reads
    actions / logp_old / adv / ret at sample_index[i]) and its gradient per frame.  With the
    heads' biases given, logits / value exclude them and their gradients are returned too.
    stats f64[>=5], when given, gets (pi_loss, v_loss, entropy, approx_kl, clipfrac) added.
    grad_absmax int32[9] (zeroed by the caller): max |dlogits[:, j]| into [j], max |dvalue| into [8], float bits
    (merlin_ppo_loss_absmax; head_bwd's plane bound)."""
    U, A = (int(x) for x in logits.shape)
    n = int(order.numel())
    assert logits.dtype == value.dtype == torch.float32 and value.shape == (U,)
    assert offs.dtype == order.dtype == torch.int32 and offs.shape == (U + 1,)
    assert frame_of.dtype == torch.int64 and frame_of.numel() == n and U <= n
    assert actions.dtype == torch.int64 and logp_old.dtype == adv.dtype == ret.dtype == torch.float32
    if sample_index is not None:
        assert sample_index.dtype == torch.int64 and sample_index.numel() == n
    if stats is not None:
        assert stats.dtype == torch.float64 and stats.numel() >= 5 and stats.is_contiguous()
    dev = logits.device
    dlogits = torch.empty((U, A), dtype=torch.float32, device=dev)
    dvalue = torch.empty((U,), dtype=torch.float32, device=dev)
    loss = torch.empty((), dtype=torch.float32, device=dev)
    dba = dbc = None
    if bias_actor is not None:
        assert bias_actor.shape == (A,) and bias_actor.dtype == torch.float32
        bias_actor = bias_actor.detach().contiguous()
        dba = torch.empty((A,), dtype=torch.float32, device=dev) if out_bias_actor is None else out_bias_actor
        assert dba.shape == (A,) and dba.is_contiguous()
    if bias_critic is not None:
        assert bias_critic.numel() == 1 and bias_critic.dtype == torch.float32
        bias_critic = bias_critic.detach().contiguous()
        dbc = torch.empty((1,), dtype=torch.float32, device=dev) if out_bias_critic is None else out_bias_critic
        assert dbc.numel() == 1 and dbc.is_contiguous()
    ws = torch.empty(max(int(lib().merlin_ppo_loss_workspace(n)), 1), dtype=torch.float64, device=dev)
    with KernelTimer.span("k_ppo_loss", U * (4 * A + 4) * 2 + n * (4 + 8 + 8 + 12)):
        if grad_absmax is not None:
            assert grad_absmax.dtype == torch.int32 and grad_absmax.numel() >= 9 and grad_absmax.is_contiguous()
        check(lib().merlin_ppo_loss_absmax(ptr(logits.contiguous()), ptr(value.contiguous()), ptr(bias_actor),
                                           ptr(bias_critic), U, A, ptr(offs), ptr(order), ptr(frame_of), n,
                                           ptr(sample_index), ptr(actions.contiguous()), ptr(logp_old.contiguous()),
                                           ptr(adv.contiguous()), ptr(ret.contiguous()), float(clip_eps),
                                           float(vf_coef), float(ent_coef), ptr(dlogits), ptr(dvalue), ptr(dba),
                                           ptr(dbc), ptr(loss), ptr(stats), ptr(ws), ptr(grad_absmax),
                                           stream_of(logits)), "merlin_ppo_loss_absmax")
    return loss, dlogits, dvalue, dba, dbc


# -- acting tail (csrc/merlin_act.hip) -----------------------------------------------------------
def act_heads(z, b4, w_actor, b_actor, w_critic, b_critic, deterministic=False, seed=0, epoch=None, step=0,
              out=None, env_offset=0):
    """(action int64[n], logp f32[n], value f32[n]) from fc1's pre-activation z f32[2, n, H]:
    relu(z + b4) -> heads -> log_softmax -> argmax or a Categorical draw keyed by (seed, epoch[0],
    step, env_offset + env): the global env index, so data-parallel shards draw like one process.  out = (action, logp, value) tensors to write in place (the rollout storage).
    A draw (deterministic=False) needs the epoch counter: the key has no hidden state, so the
    caller advances it (merlin.PPO bumps it once per rollout) or every call repeats its draws.
    Non-finite logits give action -1 (the env step then raises MERLIN_DEVERR_BAD_ACTION)."""
    T, n, H = (int(x) for x in z.shape)
    A = int(w_actor.shape[0])
    assert T == 2 and z.dtype == torch.float32 and b4.shape == (2, H) and w_actor.shape == (A, H)
    assert w_critic.numel() == H and b_critic.numel() == 1 and b_actor.numel() == A
    if not deterministic and epoch is None:
        raise ValueError("act_heads: a sampled action needs an epoch counter tensor (int64[1] on the device) "
                         "that the caller advances between rollouts; without it every call repeats its draws")
    if epoch is not None:
        assert epoch.dtype == torch.int64 and epoch.is_cuda
    dev = z.device
    if out is None:
        out = (torch.empty(n, dtype=torch.int64, device=dev), torch.empty(n, dtype=torch.float32, device=dev),
               torch.empty(n, dtype=torch.float32, device=dev))
    action, logp, value = out
    assert action.dtype == torch.int64 and logp.dtype == value.dtype == torch.float32
    assert action.numel() == logp.numel() == value.numel() == n
    with KernelTimer.span("k_act_heads", z.numel() * 4 + n * 16):
        check(lib().merlin_act_heads(ptr(z), ptr(b4), n, H, ptr(w_actor), ptr(b_actor), ptr(w_critic), ptr(b_critic), A,
                                     int(bool(deterministic)), int(seed) & 0xFFFFFFFFFFFFFFFF, ptr(epoch), int(step),
                                     int(env_offset),
                                     ptr(action), ptr(logp), ptr(value), stream_of(z)), "merlin_act_heads")
    return action, logp, value


# -- fc1 on the bf16 matrix cores in exact three-plane form (csrc/merlin_gemm.hip) ------------------
# Weights as int16 planes [..., R, 3 * C] (bf16 bits; per group of 8 values three 16-B chunks,
# x = x0 + x1 + x2 exactly, include/merlin_hip.h); activations as fp32, split while staged.
# fwd / dgrad on the 32x32x16 MFMA with split hi / lo accumulators (csrc/merlin_gemm2.hip: 806 / 790 us
# against 857 / 843 for the 16x16x32 kernels at the update's shape, scripts/probe_x6_il.py); the rollout's
# 4096-row fc1 on 128 x 128 tiles of the same kernel (37.2 us against 41.3 for cfg 2, scripts/probe_rollout_fc1.py)
X6_NT_CFG = {"fwd": 20, "dgrad": 22, "rollout": 25}  # tile configurations of merlin_x6_gemm_nt (N = 512 / 576)
X6_TN_CFG = 0
X6_TN_SPLITS = 32


def x6_split(x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """fp32 [..., C] -> int16 planes [..., 3 * C]."""
    assert x.dtype == torch.float32 and x.shape[-1] % 8 == 0
    x = x.contiguous()
    if out is None:
        out = torch.empty((*x.shape[:-1], 3 * x.shape[-1]), dtype=torch.int16, device=x.device)
    with KernelTimer.span("k_x6_split", x.numel() * 10):
        check(lib().merlin_x6_split(ptr(x), x.numel(), ptr(out), stream_of(x)), "merlin_x6_split")
    return out


def x6_join(planes: torch.Tensor) -> torch.Tensor:
    """int16 planes [..., 3 * C] -> fp32 [..., C] (x0 + x1 + x2)."""
    assert planes.dtype == torch.int16 and planes.shape[-1] % 24 == 0
    out = torch.empty((*planes.shape[:-1], planes.shape[-1] // 3), dtype=torch.float32, device=planes.device)
    check(lib().merlin_x6_join(ptr(planes), out.numel(), ptr(out), stream_of(planes)), "merlin_x6_join")
    return out


def x6_gemm_nt(A: torch.Tensor, B: torch.Tensor, bias: torch.Tensor | None = None, cfg: int = 0,
               out: torch.Tensor | None = None, name: str = "x6_gemm_nt") -> torch.Tensor:
    """C f32[T, M, N] = A @ B^T per tower (+ bias[t] and ReLU when bias is given), A f32[T, M, K],
    B planes int16[T, N, 3K] (x6_split of an f32 [T, N, K])."""
    X6_SPANS.add(name)
    T, M, K = (int(v) for v in A.shape)
    if A.dtype == torch.int16:  # A as planes too (x6_split of an f32 [T, M, K]): the cfg >= 30 kernels
        assert cfg >= 30 and K % 24 == 0, "planes A needs an x6 planes-A configuration (cfg >= 30)"
        K //= 3
    else:
        assert A.dtype == torch.float32 and cfg < 30
    N = int(B.shape[1])
    assert B.dtype == torch.int16 and B.shape == (T, N, 3 * K)
    assert A.is_contiguous() and B.is_contiguous()
    if bias is not None:
        assert bias.shape == (T, N) and bias.dtype == torch.float32
        bias = bias.detach().contiguous()
    if out is None:
        out = torch.empty((T, M, N), dtype=torch.float32, device=A.device)
    assert out.shape == (T, M, N) and out.is_contiguous()
    with KernelTimer.span(name, 0, 2 * T * M * N * K):
        check(lib().merlin_x6_gemm_nt(ptr(A), ptr(B), M, N, K, T, M * K, N * K, ptr(bias), ptr(out), M * N, int(cfg),
                                      stream_of(A)), "merlin_x6_gemm_nt")
    return out


def x6_gemm_tn(A: torch.Tensor, B: torch.Tensor, splits: int | None = None, cfg: int | None = None,
               name: str = "x6_gemm_tn", out: torch.Tensor | None = None) -> torch.Tensor:
    """out f32[T, M, N] = A^T @ B per tower, A f32[T, Kd, M], B f32[T, Kd, N] (the long k range split
    into `splits` slabs summed in order)."""
    X6_SPANS.add(name)
    splits = X6_TN_SPLITS if splits is None else splits  # module settings read at call time
    cfg = X6_TN_CFG if cfg is None else cfg
    T, Kd, M = (int(v) for v in A.shape)
    N = int(B.shape[2])
    if A.dtype == torch.int16:  # both operands as planes (x6_split of f32 [T, Kd, M] / [T, Kd, N]): cfg >= 30
        assert B.dtype == torch.int16 and cfg >= 30 and M % 24 == 0 and N % 24 == 0
        M //= 3
        N //= 3
    else:
        assert A.dtype == B.dtype == torch.float32 and cfg < 30
    assert B.shape[:2] == (T, Kd)
    assert A.is_contiguous() and B.is_contiguous()
    if out is None:
        out = torch.empty((T, M, N), dtype=torch.float32, device=A.device)
    assert out.shape == (T, M, N) and out.dtype == torch.float32 and out.is_contiguous()
    slab = torch.empty(int(lib().merlin_x6_tn_slab_floats(M, N, T, int(splits))), dtype=torch.float32,
                       device=A.device)
    with KernelTimer.span(name, 0, 2 * T * M * N * Kd):
        check(lib().merlin_x6_gemm_tn(ptr(A), ptr(B), Kd, M, N, T, Kd * M, Kd * N, int(splits), ptr(slab), ptr(out),
                                      int(cfg), stream_of(A)), "merlin_x6_gemm_tn")
    return out


# -- fc1 on the f16 matrix cores in two-plane form (csrc/merlin_h3.hip) ----------------------------------------
# tile configurations of merlin_h3_gemm_nt (N = 512 / 576): the split interleaved into the MFMAs (k_h3_ntp), forward
# 128 x 256 and input gradient 128 x 192 tiles (scripts/ab_update.py, same update replayed: 204.5 vs 209.0 ms for cfg 0 / 1)
# rollout: 4,096 rows; qall: [5^9, 64] x [64, 576] (k_h3_nt, not the input gradient's k_h3_ntp instantiation, so
# profiles keep the two apart); qwin / qwin_dgrad: the update's window GEMMs (N = 576, K = 64 / N = 64, K = 576)
H3_NT_CFG = {"fwd": 13, "dgrad": 11, "rollout": 12, "qall": 1, "qwin": 11, "qwin_dgrad": 5, "dgrad_planes": 62, "fwd_planes": 60}
H3_TN_CFG = 0
H3_TN_CFG_PLANES = 20  # the weight gradient over both operands' planes: the LDS-DMA TN (merlin_h3p.hip k_h3_tq)
# the update's fc1 forward (h3, cfg "fwd" with a heads epilogue) computes the policy / value heads in its epilogue
# (merlin_h3_gemm_nt_heads + merlin_heads_combine) instead of a pass over h (merlin_heads_fwd)
H3_HEADS_EPILOGUE = True
H3_TN_CFG_WIN = 2  # the window weight gradient (M = 64)
H3_TN_SPLITS = 32


def group_act(codes, T2, b2, W3t, b3, W4p, b4, Wa, ba, Wc, bc, a3_ws=None, part=None):
    """FOMAML's acting step over G tasks with per-task weights (merlin_group_act): head partials f32[2, 8, G, 4]
    (biases added in chunk 0) for merlin_env_act_step / act_draw with zero biases.  Weights of ONE task (T2 with 2
    towers) with G > 1 frames: every task acts with them (shared_weights)."""
    G = int(codes.shape[0])
    A = int(Wa.shape[1])
    W = int(T2.shape[0]) // 2  # weight sets: G, or 1 shared by every task
    shared = W == 1 and G > 1
    assert W == G or shared
    assert codes.dtype == torch.int32 and codes.shape == (G, OBS_WORDS) and codes.is_contiguous()
    assert T2.shape == (2 * W, 2720, 64) and W3t.shape == (2 * W, 576, 64) and W4p.shape == (2 * W, 512, 576)
    assert b2.numel() == 2 * W * 64 and b3.numel() == 2 * W * 64 and b4.numel() == 2 * W * 512
    assert Wa.shape == (W, A, 512) and ba.numel() == W * A and Wc.numel() == W * 512 and bc.numel() == W
    for t in (T2, b2, W3t, b3, W4p, b4, Wa, ba, Wc, bc):
        assert t.dtype == torch.float32 and t.is_contiguous()
    if a3_ws is None:
        a3_ws = torch.empty((2 * G, 576), dtype=torch.float32, device=codes.device)
    if part is None:
        part = torch.empty((2, 8, G, 4), dtype=torch.float32, device=codes.device)
    with KernelTimer.span("k_group_act", G * 2 * (25 * 16 * 256 + 576 * 64 * 4 + 512 * 576 * 4)):
        check(lib().merlin_group_act(ptr(codes), G, ptr(T2), ptr(b2), ptr(W3t), ptr(b3), ptr(W4p), ptr(b4), ptr(Wa),
                                     ptr(ba), ptr(Wc), ptr(bc), A, ptr(a3_ws), ptr(part), int(shared),
                                     stream_of(codes)),
              "merlin_group_act")
    return part


def h3_amax(x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """int32[T] (uint32 float bits) of max |x| per tower, x f32[T, ...] contiguous (numel per tower % 4 == 0)."""
    assert x.dtype == torch.float32 and x.is_contiguous()
    T = int(x.shape[0])
    n = x.numel() // max(T, 1)
    if out is None:
        out = torch.empty(T, dtype=torch.int32, device=x.device)
    assert out.dtype == torch.int32 and out.numel() >= T and out.is_contiguous()
    with KernelTimer.span("k_h3_amax", 4 * T * n):
        check(lib().merlin_h3_amax(ptr(x), n, T, n, ptr(out), stream_of(x)), "merlin_h3_amax")
    return out


def h3_zero(amax: torch.Tensor) -> torch.Tensor:
    """amax[:T] = 0 by a kernel (merlin_h3_amax over no values): safe inside a captured graph, where a memset node
    replays with a wrong fill value on ROCm 7."""
    assert amax.dtype == torch.int32 and amax.is_contiguous()
    check(lib().merlin_h3_amax(None, 0, int(amax.numel()), 0, ptr(amax), stream_of(amax)), "merlin_h3_amax")
    return amax


def h3_split(x: torch.Tensor, amax: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """fp32 [T, ..., C] -> f16 planes as int16 [T, ..., 2C] ([..., C/8, 2, 8]: hi and lo chunk per 8 values),
    tower t scaled by the exponent of amax[t] (h3_amax)."""
    assert x.dtype == torch.float32 and x.shape[-1] % 8 == 0 and amax.dtype == torch.int32
    x = x.contiguous()
    T = int(x.shape[0])
    if out is None:
        out = torch.empty(x.shape[:-1] + (2 * x.shape[-1],), dtype=torch.int16, device=x.device)
    check(lib().merlin_h3_split(ptr(x), x.numel() // T, T, ptr(amax), ptr(out), stream_of(x)), "merlin_h3_split")
    return out


def h3_gemm_nt(A: torch.Tensor, amaxA: torch.Tensor, B: torch.Tensor, amaxB: torch.Tensor,
               bias: torch.Tensor | None = None, cfg: int = 0, out: torch.Tensor | None = None,
               name: str = "h3_gemm_nt", planes_out: torch.Tensor | None = None,
               rows: torch.Tensor | None = None) -> torch.Tensor:
    """C f32[T, M, N] = A @ B^T per tower (+ bias[t] and ReLU when bias is given), A f32[T, M, K] with its h3_amax,
    B planes int16[T, N, 2K] (h3_split of an f32 [T, N, K] with amaxB).  planes_out int16[T, M, 2K], if given,
    receives A's planes (h3_split(A, amaxA), made by the kernel while it stages A) for a later h3_gemm_tn.
    rows int32[M * K / 64] (merlin_h3_gemm_nt_gather, pipelined cfgs): A read by 64-value chunks, row m's chunk j
    from row rows[m * K / 64 + j] of A viewed as [T, M * K / 64, 64] (conv3's patch representatives)."""
    H3_SPANS.add(name)
    T, M, K = (int(v) for v in A.shape)
    N = int(B.shape[1])
    assert A.dtype == torch.float32 and B.dtype == torch.int16 and B.shape == (T, N, 2 * K)
    assert A.is_contiguous() and B.is_contiguous() and amaxA.dtype == amaxB.dtype == torch.int32
    if out is None:
        out = torch.empty((T, M, N), dtype=torch.float32, device=A.device)
    assert out.shape == (T, M, N) and out.is_contiguous()
    if bias is not None:
        assert bias.shape == (T, N) and bias.is_contiguous()
    if planes_out is not None:
        assert planes_out.dtype == torch.int16 and planes_out.shape == (T, M, 2 * K) and planes_out.is_contiguous()
    if rows is not None:
        assert planes_out is None and rows.dtype == torch.int32 and rows.is_contiguous() and K % 64 == 0
        assert rows.numel() == M * K // 64
        with KernelTimer.span(name, 0, 2 * T * M * N * K):
            check(lib().merlin_h3_gemm_nt_gather(ptr(A), ptr(amaxA), ptr(B), ptr(amaxB), M, N, K, T, M * K, N * K,
                                                 ptr(bias) if bias is not None else None, ptr(out), M * N, ptr(rows),
                                                 int(cfg), stream_of(A)), "merlin_h3_gemm_nt_gather")
        return out
    with KernelTimer.span(name, 0, 2 * T * M * N * K):
        check(lib().merlin_h3_gemm_nt(ptr(A), ptr(amaxA), ptr(B), ptr(amaxB), M, N, K, T, M * K, N * K,
                                      ptr(bias) if bias is not None else None, ptr(out), M * N,
                                      ptr(planes_out) if planes_out is not None else None, int(cfg),
                                      stream_of(A)), "merlin_h3_gemm_nt")
    return out


def h3_gemm_nt_planes(Ap: torch.Tensor, amaxA: torch.Tensor, B: torch.Tensor, amaxB: torch.Tensor,
                      bias: torch.Tensor | None = None, cfg: int = 62, out: torch.Tensor | None = None,
                      name: str = "h3_gemm_nt") -> torch.Tensor:
    """h3_gemm_nt with A already in plane form, Ap int16[T, M, 2K] scaled by amaxA's exponent (e.g. head_bwd's dz
    planes): merlin_h3_gemm_nt_planes, both operands by LDS-DMA (cfg 60 / 61 / 62, K = 512 or 576)."""
    H3_SPANS.add(name)
    T, M, K2 = (int(v) for v in Ap.shape)
    K = K2 // 2
    N = int(B.shape[1])
    assert Ap.dtype == B.dtype == torch.int16 and B.shape == (T, N, 2 * K) and Ap.is_contiguous() and B.is_contiguous()
    assert amaxA.dtype == amaxB.dtype == torch.int32
    if out is None:
        out = torch.empty((T, M, N), dtype=torch.float32, device=Ap.device)
    assert out.shape == (T, M, N) and out.is_contiguous()
    if bias is not None:
        assert bias.shape == (T, N) and bias.is_contiguous()
    with KernelTimer.span(name, 0, 2 * T * M * N * K):
        check(lib().merlin_h3_gemm_nt_planes(ptr(Ap), ptr(amaxA), ptr(B), ptr(amaxB), M, N, K, T, M * K, N * K,
                                             ptr(bias) if bias is not None else None, ptr(out), M * N, int(cfg),
                                             stream_of(Ap)), "merlin_h3_gemm_nt_planes")
    return out


def h3_gemm_nt_heads(A: torch.Tensor, amaxA: torch.Tensor, B: torch.Tensor, amaxB: torch.Tensor, bias: torch.Tensor,
                     Wa: torch.Tensor, Wc: torch.Tensor, cfg: int, rows: torch.Tensor | None = None,
                     name: str = "h3_gemm_nt", partials_only: bool = False) -> tuple:
    """(h, logits, value): h = relu(A @ B^T + bias) per tower as h3_gemm_nt (A f32[2, M, K], B planes), with the heads
    logits [M, A] = h[0] Wa^T and value [M] = h[1] wc (no biases) from partial dot products made in the GEMM's
    epilogue (merlin_h3_gemm_nt_heads) and summed in order (merlin_heads_combine, span "k_heads_fwd").
    partials_only: h is not written and the heads' partials float[2, parts, M, 4] are returned as they are (for
    act_draw)."""
    H3_SPANS.add(name)
    T, M, K = (int(v) for v in A.shape)
    ap = A.dtype == torch.int16  # A as planes (window_conv3_planes): merlin_h3_gemm_nt_heads_planes, gathered only
    if ap:
        K //= 2
        assert rows is not None and not partials_only
    N = int(B.shape[1])
    NA = int(Wa.shape[0])
    assert T == 2 and A.dtype in (torch.float32, torch.int16) and B.dtype == torch.int16 and B.shape == (T, N, 2 * K)
    assert A.is_contiguous() and B.is_contiguous() and bias.shape == (T, N) and bias.is_contiguous()
    assert Wa.shape == (NA, N) and Wa.is_contiguous() and Wc.numel() == N and Wc.is_contiguous() and 1 <= NA <= 4
    P = int(lib().merlin_h3_heads_parts(N, int(cfg)))
    assert P > 0, f"cfg {cfg}: no heads epilogue"
    if rows is not None:
        assert rows.dtype == torch.int32 and rows.is_contiguous() and rows.numel() == M * K // 64
    out = None if partials_only else torch.empty((T, M, N), dtype=torch.float32, device=A.device)
    part = torch.empty((T, P, M, 4), dtype=torch.float32, device=A.device)
    fn = lib().merlin_h3_gemm_nt_heads_planes if ap else lib().merlin_h3_gemm_nt_heads
    with KernelTimer.span(name, 0, 2 * T * M * N * K):
        check(fn(ptr(A), ptr(amaxA), ptr(B), ptr(amaxB), M, N, K, M * K, N * K, ptr(bias), ptr(out), M * N, ptr(rows),
                 ptr(Wa), NA, ptr(Wc), ptr(part), int(cfg), stream_of(A)), "merlin_h3_gemm_nt_heads")
    if partials_only:
        return part
    logits = torch.empty((M, NA), dtype=torch.float32, device=A.device)
    value = torch.empty(M, dtype=torch.float32, device=A.device)
    with KernelTimer.span("k_heads_fwd", T * P * M * 16 + M * (NA + 1) * 4):
        check(lib().merlin_heads_combine(ptr(part), P, M, NA, ptr(logits), ptr(value), stream_of(A)),
              "merlin_heads_combine")
    return out, logits, value


def act_draw(part, b_actor, b_critic, deterministic=False, seed=0, epoch=None, step=0, out=None, env_offset=0):
    """act_heads' tail (log-softmax, argmax or the counter-keyed draw; action / logp / value) from the heads' partials
    of h3_gemm_nt_heads(partials_only=True): part f32[2, P, n, 4] summed in order, the biases added here."""
    T, P, n, _ = (int(x) for x in part.shape)
    A = int(b_actor.numel())
    assert T == 2 and part.dtype == torch.float32 and part.is_contiguous() and 1 <= A <= 4 and b_critic.numel() == 1
    if not deterministic and epoch is None:
        raise ValueError("act_draw: a sampled action needs an epoch counter tensor (int64[1] on the device)")
    dev = part.device
    if out is None:
        out = (torch.empty(n, dtype=torch.int64, device=dev), torch.empty(n, dtype=torch.float32, device=dev),
               torch.empty(n, dtype=torch.float32, device=dev))
    action, logp, value = out
    assert action.dtype == torch.int64 and logp.dtype == value.dtype == torch.float32
    assert action.numel() == logp.numel() == value.numel() == n
    with KernelTimer.span("k_act_heads", part.numel() * 4 + n * 16):
        check(lib().merlin_act_draw(ptr(part), P, n, ptr(b_actor), ptr(b_critic), A, int(bool(deterministic)),
                                    int(seed) & 0xFFFFFFFFFFFFFFFF, ptr(epoch), int(step), int(env_offset), ptr(action),
                                    ptr(logp), ptr(value), stream_of(part)), "merlin_act_draw")
    return action, logp, value


def h3_gemm_tn(A: torch.Tensor, amaxA: torch.Tensor, B: torch.Tensor, amaxB: torch.Tensor,
               splits: int | None = None, cfg: int | None = None, name: str = "h3_gemm_tn",
               out: torch.Tensor | None = None, rows: torch.Tensor | None = None) -> torch.Tensor:
    """out f32[T, M, N] = A^T @ B per tower, A f32[T, Kd, M], B f32[T, Kd, N] with their h3_amax (the long k range
    split into `splits` slabs summed in order).  A and B may instead both be planes, int16[T, Kd, 2M] / [T, Kd, 2N]
    (h3_gemm_nt's planes_out of the same tensors and scales): the same product without splitting them again.
    rows int32[Kd * N / 64] (merlin_h3_gemm_tn_gather, cfgs 0-2): B read by 64-value chunks, row k's chunk j from row
    rows[k * N / 64 + j] of B viewed as [T, Kd * N / 64, 64]."""
    H3_SPANS.add(name)
    splits = H3_TN_SPLITS if splits is None else splits
    cfg = H3_TN_CFG if cfg is None else cfg
    planes = A.dtype == torch.int16
    a_planes = planes and (B.dtype == torch.float32 or rows is not None)  # A planes (head_bwd's dz), B through rows
    b_planes = a_planes and B.dtype == torch.int16  # ... B planes too (window_conv3_planes)
    if a_planes:
        planes = False
    T, Kd, M = (int(v) for v in A.shape)
    if a_planes:
        M //= 2
    N = int(B.shape[2]) // (2 if b_planes else 1)
    if a_planes:
        assert rows is not None and M % 8 == 0, "A planes: the gathered form only"
    elif planes:
        assert B.dtype == torch.int16 and M % 2 == 0 and N % 2 == 0
        M, N = M // 2, N // 2
    else:
        assert A.dtype == B.dtype == torch.float32
    assert B.shape[:2] == (T, Kd)
    assert A.is_contiguous() and B.is_contiguous() and amaxA.dtype == amaxB.dtype == torch.int32
    if out is None:
        out = torch.empty((T, M, N), dtype=torch.float32, device=A.device)
    assert out.shape == (T, M, N) and out.dtype == torch.float32 and out.is_contiguous()
    slab = torch.empty(int(lib().merlin_x6_tn_slab_floats(M, N, T, int(splits))), dtype=torch.float32,
                       device=A.device)
    if rows is not None:
        assert not planes and rows.dtype == torch.int32 and rows.is_contiguous() and N % 64 == 0
        assert rows.numel() == Kd * N // 64
        fn = (lib().merlin_h3_gemm_tn_gather_planes if b_planes else lib().merlin_h3_gemm_tn_gather_planes_a
              if a_planes else lib().merlin_h3_gemm_tn_gather)
        with KernelTimer.span(name, 0, 2 * T * M * N * Kd):
            check(fn(ptr(A), ptr(amaxA), ptr(B), ptr(amaxB), Kd, M, N, T, Kd * M, Kd * N, int(splits), ptr(slab),
                     ptr(out), ptr(rows), int(cfg), stream_of(A)), "merlin_h3_gemm_tn_gather")
        return out
    fn = lib().merlin_h3_gemm_tn_planes if planes else lib().merlin_h3_gemm_tn
    with KernelTimer.span(name, 0, 2 * T * M * N * Kd):
        check(fn(ptr(A), ptr(amaxA), ptr(B), ptr(amaxB), Kd, M, N, T, Kd * M, Kd * N, int(splits), ptr(slab),
                 ptr(out), int(cfg), stream_of(A)), "merlin_h3_gemm_tn")
    return out


# -- the conv1 / conv2 tables and their adjoint (csrc/merlin_stage.hip) -----------------------------
def stage_tables_fwd(W1, b1, W2, atlas, idx, HT=None, T2=None):
    """(HT f32[T, 680, 32], T2 f32[T, 2720, 64]) of the stacked conv weights W1 f32[T, 32, 3, 8, 8], b1 f32[T, 32],
    W2 f32[T, 64, 32, 4, 4] (atlas f32[5, 3, 8, 8] / 255, idx int16[680, 4]: CNNActorCritic.stage_consts)."""
    T = int(W1.shape[0])
    assert W1.shape == (T, 32, 3, 8, 8) and b1.shape == (T, 32) and W2.shape == (T, 64, 32, 4, 4)
    assert all(x.dtype == torch.float32 and x.is_contiguous() for x in (W1, b1, W2, atlas))
    assert idx.dtype == torch.int16 and idx.shape == (680, 4) and atlas.shape == (5, 3, 8, 8)
    HT = torch.empty((T, 680, 32), dtype=torch.float32, device=W1.device) if HT is None else HT
    T2 = torch.empty((T, LUT2_ROWS, 64), dtype=torch.float32, device=W1.device) if T2 is None else T2
    check(lib().merlin_stage_tables_fwd(ptr(W1), ptr(b1), ptr(W2), ptr(atlas), ptr(idx), T, ptr(HT), ptr(T2),
                                        stream_of(W1)), "merlin_stage_tables_fwd")
    return HT, T2


def stage_tables_bwd(W2, HT, dT2, atlas, koff, kv, dW1=None, db1=None, dW2=None, dH=None):
    """(dW1, db1, dW2) of stage_tables_fwd from dT2 f32[T, 2720, 64] (koff int16[81] / kv int16[2720]: the
    combinations of each conv1-table entry, CNNActorCritic.stage_consts)."""
    T = int(W2.shape[0])
    dev = W2.device
    assert dT2.shape == (T, LUT2_ROWS, 64) and HT.shape == (T, 680, 32) and dT2.is_contiguous()
    assert koff.dtype == kv.dtype == torch.int16 and koff.numel() == 81 and kv.numel() == 2720
    dW1 = torch.empty((T, 32, 3, 8, 8), dtype=torch.float32, device=dev) if dW1 is None else dW1
    db1 = torch.empty((T, 32), dtype=torch.float32, device=dev) if db1 is None else db1
    dW2 = torch.empty((T, 64, 32, 4, 4), dtype=torch.float32, device=dev) if dW2 is None else dW2
    dH = torch.empty((T, 680, 32), dtype=torch.float32, device=dev) if dH is None else dH
    assert all(x.is_contiguous() for x in (dW1, db1, dW2, dH))
    check(lib().merlin_stage_tables_bwd(ptr(W2), ptr(HT), ptr(dT2), ptr(atlas), ptr(koff), ptr(kv), T, ptr(dH),
                                        ptr(dW1), ptr(db1), ptr(dW2), stream_of(W2)), "merlin_stage_tables_bwd")
    return dW1, db1, dW2


def clip_adam(params, grads, exp_avgs, exp_avg_sqs, steps, lr, beta1, beta2, eps, max_norm, norm_out=None,
              workspace=None):
    """clip_grad_norm_(params, max_norm) + torch's fused Adam step (src/ppo.py:153-156) in two
    launches (merlin_clip_adam): the gradients are clipped in place, (param, exp_avg, exp_avg_sq)
    updated, each float32[1] step counter advanced.  Returns the pre-clip global norm (norm_out)."""
    n = len(params)
    if not (len(grads) == len(exp_avgs) == len(exp_avg_sqs) == len(steps) == n):
        raise ValueError("clip_adam: parameter / state lists differ in length")
    for group in (params, grads, exp_avgs, exp_avg_sqs, steps):
        for t in group:
            if t.dtype != torch.float32:
                raise MerlinNativeError("clip_adam: float32 tensors only")
    for p, g, m, v in zip(params, grads, exp_avgs, exp_avg_sqs):
        if not (p.numel() == g.numel() == m.numel() == v.numel()):
            raise ValueError("clip_adam: a parameter and its gradient / state differ in size")
    numel = (C.c_int64 * n)(*[int(p.numel()) for p in params])
    arr = lambda ts: (C.c_void_p * n)(*[ptr(t).value for t in ts])  # noqa: E731
    dev = params[0].device
    if workspace is None:
        workspace = torch.empty(int(lib().merlin_clip_adam_workspace(n, numel)), dtype=torch.float64, device=dev)
    if norm_out is None:
        norm_out = torch.empty((), dtype=torch.float32, device=dev)
    check(lib().merlin_clip_adam(n, arr(params), arr(grads), arr(exp_avgs), arr(exp_avg_sqs), arr(steps), numel,
                                 float(lr), float(beta1), float(beta2), float(eps), float(max_norm), ptr(norm_out),
                                 ptr(workspace), stream_of(params[0])), "merlin_clip_adam")
    return norm_out
