"""ctypes binding of libppox.so (the C ABI declared in include/ppox.h).

This is the ONLY way the product reaches its compute: there is no CPU or
PyTorch fallback.  If the library or a GPU is missing, `lib()` raises.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# PPOX_LIB: an A/B build of the same sources (tools/build_variant.sh) for kernel tests/timing
LIB_PATH = os.environ.get("PPOX_LIB") or os.path.join(_HERE, "libppox.so")

# The A/B switches of the product path (kernel forms, batch gates, stream placement) are constants unless
# PPOX_AB=1: only then are their PPOX_* environment variables read (tests, tools/; the library's own switches
# follow the same rule, common.h ppox::ab_env).  User-facing settings (PPOX_CONV_MATH, PPOX_NATIVE_DP,
# PPOX_ICM_NATIVE, PPOX_LIB) are read always.
AB = os.environ.get("PPOX_AB") == "1"


def ab_env(name, default):
    """os.environ.get(name, default) under PPOX_AB=1, else default"""
    return os.environ.get(name, default) if AB else default

_vp, _i64, _i32, _f64, _f32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_double, ctypes.c_float
_u64 = ctypes.c_uint64

SIMHASH_KEYS = 65536  # include/ppox.h PPOX_SIMHASH_KEYS
LOSS_PARTIALS = 64   # PPOX_LOSS_PARTIALS
NORM_PARTIALS = 256  # PPOX_NORM_PARTIALS

# name -> argtypes (restype is int unless listed in _RESTYPES)
SIGNATURES = {
    "ppox_gae": [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _f64, _f64, _vp, _vp, _vp],
    "ppox_gae_dual": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _f64, _f64, _f64,
                      _vp, _vp, _vp, _vp, _vp],
    "ppox_rms_update_u8": [_vp, _i64, _i64, _i64, _vp, _vp, _f64, _vp, _i64, _vp, _vp, _vp],
    "ppox_rms_update_f32": [_vp, _i64, _i64, _i64, _vp, _vp, _f64, _vp],
    "ppox_rms_scale_int_rewards": [_vp, _i64, _vp, _vp, _f64, _vp],
    "ppox_normalize_obs_u8": [_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp],
    "ppox_normalize_obs_f32": [_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp],
    "ppox_minibatch_adv_stats": [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _vp, _vp],
    "ppox_ppo_loss_partials": [_vp, _vp, _vp, _i64, _i32, _vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp,
                               _vp, _vp, _vp, _vp, _f32, _vp, _vp],
    "ppox_ppo_loss_backward": [_vp, _vp, _vp, _i64, _i32, _vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp,
                               _vp, _vp, _vp, _vp, _f32, _vp, _i64, _f32, _f32, _f32, _f32,
                               _vp, _vp, _vp, _vp, _vp],
    "ppox_categorical_sample": [_vp, _i64, _i32, _i64, _u64, _i64, _vp, _vp, _vp],
    "ppox_categorical_sample_dc": [_vp, _i64, _i32, _i64, _u64, _vp, _i64, _vp, _vp, _vp],
    "ppox_atari_env_step_dc": [_vp, _vp, _vp, _i64, _i64, _u64, _vp, _i64, _f32, _f32, _vp, _vp, _vp, _vp,
                               _vp, _vp, _vp],
    "ppox_counters_add": [_vp, _i32, _i64, _vp],
    "ppox_ppo_box_loss_partials": [_vp, _vp, _vp, _vp, _i64, _i32, _vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp,
                                   _vp, _vp, _vp, _vp, _f64, _vp, _vp],
    "ppox_ppo_box_loss_backward": [_vp, _vp, _vp, _vp, _i64, _i32, _vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp,
                                   _vp, _vp, _vp, _vp, _f64, _vp, _i64, _f32, _f32, _f32, _f32,
                                   _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "ppox_normal_sample": [_vp, _vp, _i64, _i32, _i64, _u64, _i64, _vp, _vp, _vp],
    "ppox_simhash_keys": [_vp, _i64, _i64, _i64, _vp, _vp, _vp],
    "ppox_simhash_apply": [_vp, _i64, _i64, _i64, _vp, _f64, _vp, _vp],
    "ppox_gather_rows": [_vp, _i64, _i64, _i64, _i64, _vp, _i64, _vp, _vp],
    "ppox_grad_sumsq": [_vp, _i64, _vp, _vp],
    "ppox_adam_step": [_vp, _vp, _vp, _vp, _i64, _vp, _f32, _f64, _f64, _f64, _f64, _i64, _vp, _vp],
    "ppox_ktime_arm": [_vp],
    "ppox_ktime_take": [],
    "ppox_adam_step_wmax": [_vp, _vp, _vp, _vp, _i64, _vp, _f32, _f64, _f64, _f64, _f64, _i64, _vp, _vp, _vp, _vp],
    "ppox_atari_env_reset": [_vp, _i64, _i64, _u64, _vp, _vp, _vp],
    "ppox_atari_env_step": [_vp, _vp, _vp, _i64, _i64, _u64, _i64, _f32, _f32, _vp, _vp, _vp, _vp,
                            _vp, _vp, _vp],
    "ppox_nature_pack_weights": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "ppox_nature_conv_dgrad": [_i32, _vp, _i64, _vp, _vp, _vp, _vp],
    "ppox_nature_conv_wgrad": [_i32, _vp, _i64, _vp, _i64, _i64, _i64, _vp, _vp, _i64, _vp],
    "ppox_nature_wgrad_reduce": [_i32, _i64, _vp, _vp, _vp, _vp],
    "ppox_nchw_to_nhwc_relu_grad": [_vp, _vp, _i64, _vp, _vp],
    "ppox_nature_conv_fwd": [_i32, _vp, _i64, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp],
    "ppox_nature_pack_split": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "ppox_nature_conv_fwd_split": [_i32, _vp, _i64, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                   _vp, _vp],
    "ppox_nature_conv_dgrad_split": [_i32, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "ppox_relu_backward_": [_vp, _vp, _i64, _vp],
    "ppox_relu_backward_amax_": [_vp, _vp, _i64, _vp, _vp],
    "ppox_amax": [_vp, _i64, _vp, _vp],
    "ppox_u8_to_f32": [_vp, _i64, _vp, _vp],
    "ppox_skinny_linear": [_vp, _vp, _vp, _i64, _i64, _i64, _vp, _vp],
    "ppox_skinny_dgrad": [_vp, _vp, _i64, _i64, _i64, _vp, _vp],
    "ppox_head_grads": [_vp] * 9 + [_i64, _i64, _i64] + [_vp] * 10 + [_i32, _vp, _vp, _vp, _vp, _vp],
    "ppox_head_dgrad_outer": [_vp] * 5 + [_i64, _i64, _i64] + [_vp] * 4,
    "ppox_nature_fc_pack": [_vp, _vp, _vp, _vp],
    "ppox_nature_pack_all": [_vp] * 19 + [_i64, _vp],
    "ppox_nature_pack_all_wmax": [_vp] * 21 + [_i64, _vp],
    "ppox_nature_conv1_fwd_planes": [_vp, _i64, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp],
    "ppox_nature_conv2_fwd_planes": [_vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "ppox_nature_conv2_wgrad_planes": [_vp, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp],
    "ppox_nature_fc_fwd": [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "ppox_head_hidden_fwd": [_vp, _i64, _vp, _vp, _vp, _vp, _vp],
    "ppox_head_hidden_fwd_splitk": [_vp, _i64, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp],
    "ppox_head_hidden_dgrad": [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp],
    "ppox_head_backward": [_vp] * 7 + [_i64, _i64, _i64] + [_vp] * 5,
    "ppox_head_hidden_wgrad": [_vp, _i64, _vp, _vp, _i64, _vp, _vp, _vp, _vp],
    "ppox_nature_fc_dgrad": [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "ppox_nature_fc_wgrad": [_vp, _i64, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp],
    "ppox_px_split": [_vp, _i64, _vp, _vp, _vp, _vp],
    "ppox_es_noise": [_i64, _i64, _i64, _i64, _u64, _vp, _vp],
    "ppox_es_env_noise": [_i32, _i32, _u64, _vp, _vp],
    "ppox_es_evaluate": [_vp, _vp, _f64, _i64, _i32, _i32, _i32, _i32, _i32, _u64, _vp, _vp, _vp, _vp],
    "ppox_es_update": [_vp, _vp, _i64, _i64, _vp, _i64, _vp, _vp],
    "ppox_normalize_obs_f32_ex": [_vp, _i64, _i64, _i64, _vp, _vp, _f64, _f64, _vp, _vp],
    "ppox_vecnorm_reward": [_vp, _vp, _vp, _i64, _f64, _vp, _vp, _f64, _f64, _f64, _i32, _vp],
    "ppox_outer_relu_backward": [_vp, _vp, _vp, _i64, _i64, _vp, _vp, _vp],
    "ppox_nature_conv_wgrad_split": [_i32, _vp, _i64, _i64, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "ppox_nature_conv_wgrad_split_idx": [_i32, _vp, _i64, _vp, _i64, _i64, _vp, _vp, _i64, _vp, _vp, _vp, _vp],
    "ppox_vec_env_reset": [_vp, _i64, _i32, _i64, _u64, _vp, _vp, _vp],
    "ppox_vec_env_step": [_vp, _vp, _i64, _i32, _i64, _u64, _i64, _f32, _i32, _vp, _vp, _vp, _vp,
                          _vp, _vp, _vp],
    "ppox_nature_fc_fwd_splitk": [_vp, _i64, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp],
    "ppox_icm_pack_w1": [_vp, _i64, _vp, _vp],
    "ppox_icm_encode": [_vp, _i64, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "ppox_icm_pair_backward": [_vp, _i64, _vp, _vp, _vp, _i64, _i64, _i32, _f32, _vp, _vp, _vp, _vp, _vp],
    "ppox_icm_row_backward": [_vp, _vp, _vp, _i64, _vp, _vp, _i32, _vp, _vp, _vp],
    "ppox_icm_scatter_positions": [_vp, _vp, _vp, _vp, _i64, _i64, _vp, _vp],
    "ppox_icm_grad_reduce": [_vp, _i64, _i64, _i32, _f32, _i64, _vp, _vp, _vp],
    "ppox_icm_enc_wgrad": [_vp, _vp, _i64, _i64, _vp, _vp, _vp],
    "ppox_icm_int_reward": [_vp, _vp, _vp, _i64, _i32, _vp, _f32, _vp, _vp, _vp],
    "ppox_dp_load": [ctypes.c_char_p],
    "ppox_event_create": [ctypes.c_uint32, ctypes.POINTER(_vp)],
    "ppox_event_destroy": [_vp],
    "ppox_stream_order": [_vp, _vp, _vp],
    "ppox_dp_unique_id_bytes": [],
    "ppox_dp_unique_id": [_vp],
    "ppox_dp_comm_init": [_vp, _i32, _i32, _i32, ctypes.POINTER(_vp)],
    "ppox_dp_comm_destroy": [_vp],
    "ppox_dp_all_reduce": [_vp, _vp, _i64, _i32, _i32, _vp],
    "ppox_dp_wait": [_vp, _vp],
}
_RESTYPES = {"ppox_version": ctypes.c_char_p, "ppox_last_error": ctypes.c_char_p,
             "ppox_rms_u8_workspace_bytes": ctypes.c_int64, "ppox_nature_wgrad_splits": ctypes.c_int64,
             "ppox_nature_wgrad_workspace_bytes": ctypes.c_int64, "ppox_nature_split_pack_elems": ctypes.c_int64,
             "ppox_nature_wgrad_split_workspace_bytes": ctypes.c_int64,
             "ppox_es_update_workspace_bytes": ctypes.c_int64,
             "ppox_nature_fc_pack_elems": ctypes.c_int64, "ppox_head_grads_workspace_bytes": ctypes.c_int64,
             "ppox_nature_fc_wgrad_workspace_bytes": ctypes.c_int64, "ppox_icm_param_elems": ctypes.c_int64,
             "ppox_icm_w1_pack_elems": ctypes.c_int64, "ppox_icm_encode_workspace_bytes": ctypes.c_int64,
             "ppox_icm_partials_bytes": ctypes.c_int64, "ppox_icm_g1_pack_elems": ctypes.c_int64,
             "ppox_nature_fc_fwd_splitk_workspace_bytes": ctypes.c_int64, "ppox_amax_slots": ctypes.c_int32,
             "ppox_head_hidden_pack_elems": ctypes.c_int64, "ppox_head_hidden_wgrad_workspace_bytes": ctypes.c_int64,
             "ppox_head_hidden_fwd_splitk_workspace_bytes": ctypes.c_int64,
             "ppox_nature_conv2_wgrad_planes_workspace_bytes": ctypes.c_int64}
_RESTYPE_ARGS = {"ppox_rms_u8_workspace_bytes": [_i64, _i64], "ppox_nature_wgrad_splits": [_i32, _i64],
                 "ppox_nature_wgrad_workspace_bytes": [_i32, _i64], "ppox_nature_split_pack_elems": [_i32],
                 "ppox_nature_wgrad_split_workspace_bytes": [_i32, _i64],
                 "ppox_es_update_workspace_bytes": [_i64, _i64],
                 "ppox_nature_fc_pack_elems": [], "ppox_head_grads_workspace_bytes": [_i64, _i64, _i64, _i32],
                 "ppox_nature_fc_wgrad_workspace_bytes": [_i64], "ppox_icm_param_elems": [_i32],
                 "ppox_icm_w1_pack_elems": [_i64], "ppox_icm_encode_workspace_bytes": [_i64, _i64],
                 "ppox_icm_partials_bytes": [_i64, _i32], "ppox_icm_g1_pack_elems": [_i64],
                 "ppox_nature_fc_fwd_splitk_workspace_bytes": [_i64], "ppox_head_hidden_wgrad_workspace_bytes": [_i64],
                 "ppox_head_hidden_fwd_splitk_workspace_bytes": [_i64],
                 "ppox_nature_conv2_wgrad_planes_workspace_bytes": [_i64]}

_lib = None


class NativeError(RuntimeError):
    pass


def load(path=LIB_PATH):
    """Load and bind the library (no GPU needed: used by the CPU ABI tests)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(f"libppox.so not built at {path}: run `make -C ppo-exploration_amd` "
                          "(or __graft_entry__.build()); there is no fallback path")
    lib = ctypes.CDLL(path)
    for name, argtypes in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = ctypes.c_int
    for name, rt in _RESTYPES.items():
        fn = getattr(lib, name)
        fn.argtypes = _RESTYPE_ARGS.get(name, [])
        fn.restype = rt
    _lib = lib
    return lib


_gpu_ok = False


def lib():
    """The library, for compute calls: also requires a visible GPU (checked once: the
    per-launch host cost matters where the minibatch / collect loops are launch-bound)."""
    global _gpu_ok
    l = load()
    if not _gpu_ok:
        if not torch.cuda.is_available():
            raise RuntimeError("ppo-exploration_amd needs an MI355X (HIP device); none is visible")
        _gpu_ok = True
    return l


def version():
    return load().ppox_version().decode()


_timed = set()
_events = {}


def enable_event_timing(names):
    """Bracket every launch of the named entry points with HIP events recorded on
    the stream the kernel is launched on (bench.py roofline measurement)."""
    _timed.clear()
    _timed.update(names)
    for n in names:
        _events[n] = []


def event_times_ms(name):
    """[(ms, args)] for every timed launch of `name` (or 'name:layer' for the conv entry points)."""
    torch.cuda.synchronize()
    return [(a.elapsed_time(b), args) for a, b, args in _events.get(name, [])]


_LAYERED = ("ppox_nature_conv_fwd", "ppox_nature_conv_dgrad", "ppox_nature_conv_wgrad",
            "ppox_nature_conv_fwd_split", "ppox_nature_conv_dgrad_split", "ppox_nature_conv_wgrad_split",
            "ppox_nature_conv_wgrad_split_idx")


_fns = {}


def call(name, *args):
    fn = _fns.get(name)
    if fn is None:  # bound once per entry point (the per-launch host cost matters on the hot loops)
        fn = _fns[name] = getattr(lib(), name)
    if _timed:
        key = f"{name}:{args[0]}" if name in _LAYERED else name
        if key in _timed and not torch.cuda.is_current_stream_capturing():  # (captured launches replay untimed)
            # events on the stream the kernel is launched on (every entry point's last argument)
            sp = args[-1].value if isinstance(args[-1], _vp) else None
            s = torch.cuda.ExternalStream(sp) if sp else torch.cuda.current_stream()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            k = torch.cuda.Event(enable_timing=True)  # the main kernel's end, where the entry has a trailing reduce
            a.record(s)
            k.record(s)  # (creates the event; re-recorded by the entry point)
            lib().ppox_ktime_arm(ctypes.c_void_p(k.cuda_event))
            rc = fn(*args)
            used = lib().ppox_ktime_take()
            b.record(s)
            _events[key].append((a, k if used else b, args))
            if rc != 0:
                raise NativeError(f"{name} failed ({rc}): {load().ppox_last_error().decode()}")
            return
    rc = fn(*args)
    if rc != 0:
        raise NativeError(f"{name} failed ({rc}): {load().ppox_last_error().decode()}")


def stream_ptr(stream=None):
    """Raw HIP stream of `stream`, default torch's current stream on the current device
    (read through the raw-stream accessor: torch.cuda.current_stream() costs several us of
    host time per launch)."""
    if stream is not None:
        return _vp(stream.cuda_stream)
    return _vp(torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice()))


def ptr(t, dtype=None, numel=None, name="tensor"):
    """Device pointer of a contiguous tensor (validated)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if numel is not None and t.numel() != numel:
        raise ValueError(f"{name} has {t.numel()} elements, expected {numel}")
    return _vp(t.data_ptr())


# ---------------------------------------------------------------------------
# K1 GAE
# ---------------------------------------------------------------------------
def gae(rewards, values, dones, last_value, last_done, gamma, lam, advantages, returns, stream=None):
    T, N = rewards.shape
    f32, u8 = torch.float32, torch.uint8
    call("ppox_gae", ptr(rewards, f32, T * N, "rewards"), ptr(values, f32, T * N, "values"),
         ptr(dones, u8, T * N, "dones"), ptr(last_value, f32, N, "last_value"),
         ptr(last_done, u8, N, "last_done"), T, N, float(gamma), float(lam),
         ptr(advantages, f32, T * N, "advantages"), ptr(returns, f32, T * N, "returns"), stream_ptr(stream))


def gae_dual(rewards, values, dones, last_value, last_done, int_rewards, int_values, last_int_value,
             gamma, int_gamma, lam, advantages, returns, int_advantages, int_returns, stream=None):
    T, N = rewards.shape
    f32, u8 = torch.float32, torch.uint8
    call("ppox_gae_dual", ptr(rewards, f32, T * N, "rewards"), ptr(values, f32, T * N, "values"),
         ptr(dones, u8, T * N, "dones"), ptr(last_value, f32, N, "last_value"),
         ptr(last_done, u8, N, "last_done"), ptr(int_rewards, f32, T * N, "int_rewards"),
         ptr(int_values, f32, T * N, "int_values"), ptr(last_int_value, f32, N, "last_int_value"),
         T, N, float(gamma), float(int_gamma), float(lam),
         ptr(advantages, f32, T * N, "advantages"), ptr(returns, f32, T * N, "returns"),
         ptr(int_advantages, f32, T * N, "int_advantages"), ptr(int_returns, f32, T * N, "int_returns"),
         stream_ptr(stream))


def _p(t):
    """Unchecked device pointer (hot loops; shapes were validated at setup)."""
    return None if t is None else _vp(t.data_ptr())


# ---------------------------------------------------------------------------
# K2/K3 running moments + normalisation
# ---------------------------------------------------------------------------
def rms_u8_workspace_bytes(rows, cols):
    return int(load().ppox_rms_u8_workspace_bytes(rows, cols))


def rms_update_u8(x, rows, cols, row_stride, mean, var, count, workspace, batch_mean=None, batch_var=None,
                  stream=None):
    call("ppox_rms_update_u8", _p(x), rows, cols, row_stride, _p(mean), _p(var), float(count), _p(workspace),
         workspace.numel() * workspace.element_size(), _p(batch_mean), _p(batch_var), stream_ptr(stream))


def rms_update_f32(x, rows, cols, row_stride, mean, var, count, stream=None):
    call("ppox_rms_update_f32", _p(x), rows, cols, row_stride, _p(mean), _p(var), float(count), stream_ptr(stream))


def rms_scale_int_rewards(int_rewards, mean, var, count, stream=None):
    call("ppox_rms_scale_int_rewards", ptr(int_rewards, torch.float32, name="int_rewards"), int_rewards.numel(),
         _p(mean), _p(var), float(count), stream_ptr(stream))


def _check_moments(name, cols, mean, var):
    if mean.numel() != cols or var.numel() != cols or mean.dtype != torch.float64 or var.dtype != torch.float64:
        raise ValueError(f"{name}: mean/var must be {cols} float64 values (got {mean.numel()}, {var.numel()})")


def normalize_obs(x, rows, cols, row_stride, mean, var, out, stream=None):
    name = "ppox_normalize_obs_u8" if x.dtype == torch.uint8 else "ppox_normalize_obs_f32"
    _check_moments(name, cols, mean, var)
    call(name, _p(x), rows, cols, row_stride, _p(mean), _p(var), ptr(out, torch.float32, rows * cols, "out"),
         stream_ptr(stream))


# ---------------------------------------------------------------------------
# K4 loss + categorical head
# ---------------------------------------------------------------------------
def minibatch_adv_stats(adv, int_adv, perm, total, batch_size, T, N, out, stream=None):
    call("ppox_minibatch_adv_stats", _p(adv), _p(int_adv), _p(perm), total, batch_size, T, N, _p(out),
         stream_ptr(stream))


def ppo_loss_partials(logits, values, int_values, B, A, idx, T, N, roll, adv_stats, clip, partials, stream=None):
    """roll: dict of step-major rollout tensors (actions i32, log_probs, values, advantages, returns,
    int_values, int_advantages, int_returns)."""
    g = roll.get
    call("ppox_ppo_loss_partials", _p(logits), _p(values), _p(int_values), B, A, _p(idx), T, N,
         _p(g("actions")), _p(g("log_probs")), _p(g("values")), _p(g("advantages")), _p(g("returns")),
         _p(g("int_values") if int_values is not None else None),
         _p(g("int_advantages") if int_values is not None else None),
         _p(g("int_returns") if int_values is not None else None), _p(adv_stats), float(clip), _p(partials),
         stream_ptr(stream))


def ppo_loss_backward(logits, values, int_values, B, A, idx, T, N, roll, adv_stats, clip, partials, B_global,
                      ent_coef, vf_coef, int_vf_coef, scale, dlogits, dvalues, dint_values, loss_accum,
                      stream=None):
    g = roll.get
    call("ppox_ppo_loss_backward", _p(logits), _p(values), _p(int_values), B, A, _p(idx), T, N,
         _p(g("actions")), _p(g("log_probs")), _p(g("values")), _p(g("advantages")), _p(g("returns")),
         _p(g("int_values") if int_values is not None else None),
         _p(g("int_advantages") if int_values is not None else None),
         _p(g("int_returns") if int_values is not None else None), _p(adv_stats), float(clip), _p(partials),
         int(B_global), float(ent_coef), float(vf_coef), float(int_vf_coef), float(scale), _p(dlogits),
         _p(dvalues), _p(dint_values), _p(loss_accum), stream_ptr(stream))


def _box_roll_args(int_values, roll):
    g = roll.get
    dual = int_values is not None
    return (_p(g("actions")), _p(g("log_probs")), _p(g("values")), _p(g("advantages")), _p(g("returns")),
            _p(g("int_values") if dual else None), _p(g("int_advantages") if dual else None),
            _p(g("int_returns") if dual else None))


def ppo_box_loss_partials(mu, log_std, values, int_values, B, D, idx, T, N, roll, adv_stats, clip, partials,
                          stream=None):
    """Box head: roll["actions"] / roll["log_probs"] are (T, N, D) f32."""
    call("ppox_ppo_box_loss_partials", _p(mu), _p(log_std), _p(values), _p(int_values), B, D, _p(idx), T, N,
         *_box_roll_args(int_values, roll), _p(adv_stats), float(clip), _p(partials), stream_ptr(stream))


def ppo_box_loss_backward(mu, log_std, values, int_values, B, D, idx, T, N, roll, adv_stats, clip, partials,
                          B_global, ent_coef, vf_coef, int_vf_coef, scale, dmu, dls_partials, dlog_std, dvalues,
                          dint_values, loss_accum, stream=None):
    call("ppox_ppo_box_loss_backward", _p(mu), _p(log_std), _p(values), _p(int_values), B, D, _p(idx), T, N,
         *_box_roll_args(int_values, roll), _p(adv_stats), float(clip), _p(partials), int(B_global),
         float(ent_coef), float(vf_coef), float(int_vf_coef), float(scale), _p(dmu), _p(dls_partials),
         _p(dlog_std), _p(dvalues), _p(dint_values), _p(loss_accum), stream_ptr(stream))


def normal_sample(mu, log_std, N, D, env_offset, seed, counter, actions, log_probs, stream=None):
    call("ppox_normal_sample", _p(mu), _p(log_std), N, D, env_offset, seed & 0xFFFFFFFFFFFFFFFF, counter,
         _p(actions), _p(log_probs), stream_ptr(stream))


def simhash_keys(obs, N, D, stride, A, keys, stream=None):
    call("ppox_simhash_keys", _p(obs), N, D, stride, _p(A), _p(keys), stream_ptr(stream))


def simhash_apply(keys_all, n_total, offset, n_local, counts, beta, rewards, stream=None):
    call("ppox_simhash_apply", _p(keys_all), n_total, offset, n_local, _p(counts), float(beta), _p(rewards),
         stream_ptr(stream))


def categorical_sample(logits, N, A, env_offset, seed, counter, actions, log_probs, stream=None):
    call("ppox_categorical_sample", _p(logits), N, A, env_offset, seed & 0xFFFFFFFFFFFFFFFF, counter,
         _p(actions), _p(log_probs), stream_ptr(stream))


def categorical_sample_dc(logits, N, A, env_offset, seed, counter_base, counter_off, actions, log_probs,
                          stream=None):
    """counter = *counter_base + counter_off, read on the device (counter_base: int64 device tensor)."""
    call("ppox_categorical_sample_dc", _p(logits), N, A, env_offset, seed & 0xFFFFFFFFFFFFFFFF, _p(counter_base),
         counter_off, _p(actions), _p(log_probs), stream_ptr(stream))


def counters_add(counters, delta, stream=None):
    call("ppox_counters_add", _p(counters), counters.numel(), int(delta), stream_ptr(stream))


# ---------------------------------------------------------------------------
# K5 gather, optimiser, envs
# ---------------------------------------------------------------------------
def gather_rows(src, T, N, row_bytes, src_row_stride, idx, nrows, dst, stream=None):
    call("ppox_gather_rows", _p(src), T, N, row_bytes, src_row_stride, _p(idx), nrows, _p(dst), stream_ptr(stream))


def grad_sumsq(grads, partials, stream=None):
    call("ppox_grad_sumsq", _p(grads), grads.numel(), _p(partials), stream_ptr(stream))


def adam_step(params, grads, m, v, norm_partials, max_norm, lr, beta1, beta2, eps, step, norm_out=None,
              stream=None):
    call("ppox_adam_step", _p(params), _p(grads), _p(m), _p(v), params.numel(), _p(norm_partials),
         float(max_norm), float(lr), float(beta1), float(beta2), float(eps), int(step), _p(norm_out),
         stream_ptr(stream))


WMAX_TENSORS, WMAX_SLOTS = 5, 256  # include/ppox.h PPOX_WMAX_*


def adam_step_wmax(params, grads, m, v, norm_partials, max_norm, lr, beta1, beta2, eps, step, ranges, amax_out,
                   norm_out=None, stream=None):
    """adam_step that also records the new weights' amax partials (ranges: a CPU int64 tensor of
    WMAX_TENSORS offsets then counts into params; amax_out: int32 [WMAX_TENSORS * WMAX_SLOTS], zeroed)"""
    assert ranges.device.type == "cpu" and ranges.dtype == torch.int64 and ranges.numel() == 2 * WMAX_TENSORS
    assert amax_out.numel() == WMAX_TENSORS * WMAX_SLOTS
    call("ppox_adam_step_wmax", _p(params), _p(grads), _p(m), _p(v), params.numel(), _p(norm_partials),
         float(max_norm), float(lr), float(beta1), float(beta2), float(eps), int(step), _p(norm_out),
         ctypes.c_void_p(ranges.data_ptr()), _p(amax_out), stream_ptr(stream))


def atari_env_reset(obs, N, env_offset, seed, ep_ret=None, ep_len=None, stream=None):
    call("ppox_atari_env_reset", _p(obs), N, env_offset, seed, _p(ep_ret), _p(ep_len), stream_ptr(stream))


def atari_env_step(obs_in, obs_out, actions, N, env_offset, seed, step, p_reward, p_done, rewards, dones,
                   ep_ret=None, ep_len=None, done_ret=None, done_len=None, stream=None):
    call("ppox_atari_env_step", _p(obs_in), _p(obs_out), _p(actions), N, env_offset, seed, step, float(p_reward),
         float(p_done), _p(rewards), _p(dones), _p(ep_ret), _p(ep_len), _p(done_ret), _p(done_len),
         stream_ptr(stream))


def atari_env_step_dc(obs_in, obs_out, actions, N, env_offset, seed, step_base, step_off, p_reward, p_done, rewards,
                      dones, ep_ret=None, ep_len=None, done_ret=None, done_len=None, stream=None):
    """step = *step_base + step_off, read on the device (step_base: int64 device tensor)."""
    call("ppox_atari_env_step_dc", _p(obs_in), _p(obs_out), _p(actions), N, env_offset, seed, _p(step_base),
         int(step_off), float(p_reward), float(p_done), _p(rewards), _p(dones), _p(ep_ret), _p(ep_len),
         _p(done_ret), _p(done_len), stream_ptr(stream))


def vec_env_reset(obs, N, D, env_offset, seed, ep_ret=None, ep_len=None, stream=None):
    call("ppox_vec_env_reset", _p(obs), N, D, env_offset, seed, _p(ep_ret), _p(ep_len), stream_ptr(stream))


def vec_env_step(obs, actions, N, D, env_offset, seed, step, p_done, max_len, rewards, dones, ep_ret=None,
                 ep_len=None, done_ret=None, done_len=None, stream=None):
    call("ppox_vec_env_step", _p(obs), _p(actions), N, D, env_offset, seed, step, float(p_done), int(max_len),
         _p(rewards), _p(dones), _p(ep_ret), _p(ep_len), _p(done_ret), _p(done_len), stream_ptr(stream))


# ---------------------------------------------------------------------------
# K6 NatureCNN convolutions
# ---------------------------------------------------------------------------
def nature_pack_weights(w1, w2, w3, wp1, wp2, wp3, wpd2=None, wpd3=None, stream=None):
    call("ppox_nature_pack_weights", _p(w1), _p(w2), _p(w3), _p(wp1), _p(wp2), _p(wp3), _p(wpd2), _p(wpd3),
         stream_ptr(stream))


def nature_conv_dgrad(layer, grad_out, batch, wpd, prev_act, grad_in, stream=None):
    call("ppox_nature_conv_dgrad", int(layer), _p(grad_out), int(batch), _p(wpd), _p(prev_act), _p(grad_in),
         stream_ptr(stream))


def nature_wgrad_workspace_bytes(layer, batch):
    return int(load().ppox_nature_wgrad_workspace_bytes(int(layer), int(batch)))


def nature_conv_wgrad(layer, x, batch, idx, T, N_env, x_sample_stride, grad_out, workspace, dw, db, stream=None):
    call("ppox_nature_conv_wgrad", int(layer), _p(x), int(batch), _p(idx), int(T), int(N_env), int(x_sample_stride),
         _p(grad_out), _p(workspace), workspace.numel() * workspace.element_size(), stream_ptr(stream))
    call("ppox_nature_wgrad_reduce", int(layer), int(batch), _p(workspace), _p(dw), _p(db), stream_ptr(stream))


def nchw_to_nhwc_relu_grad(grad, act, batch, out, stream=None):
    call("ppox_nchw_to_nhwc_relu_grad", _p(grad), _p(act), int(batch), _p(out), stream_ptr(stream))


def nature_conv_fwd(layer, x, batch, idx, T, N_env, x_sample_stride, wp, bias, y, stream=None):
    call("ppox_nature_conv_fwd", int(layer), _p(x), int(batch), _p(idx), int(T), int(N_env), int(x_sample_stride),
         _p(wp), _p(bias), _p(y), stream_ptr(stream))


# split-f16 forms (csrc/conv_split.hip, csrc/conv.hip): weights packed as two fp16 planes
# (int16 tensors) times a power-of-two scale; f32 operands carry "amax slots" (include/ppox.h)
AMAX_SLOTS = 256  # include/ppox.h ppox_amax_slots()
PACK_TAIL32 = 2 * AMAX_SLOTS + 8  # uint32 tail of a split-packed buffer (amax partials, exponents, PX bounds)


def amax_table(n, device):
    """n zeroed amax-slot rows (int32 storage of the uint32 slots), one per tensor."""
    return torch.zeros((n, AMAX_SLOTS), dtype=torch.int32, device=device)


def amax(x, slots, stream=None):
    """Record max |x| into `slots` (an amax_table row)."""
    call("ppox_amax", _p(x), x.numel(), _p(slots), stream_ptr(stream))


def _amax_of(x, slots, stream=None):
    """`slots` if given, else a fresh row holding max |x| (callers that did not record the operand)."""
    if slots is not None:
        return slots
    slots = amax_table(1, x.device)[0]
    amax(x.contiguous(), slots, stream)
    return slots


def nature_split_pack_elems(which):
    """uint16 elements of a split-packed buffer (planes + scale tail): which = 1, 2, 3 (forward)
    or 12, 13 (dgrad of conv2/3)."""
    return int(load().ppox_nature_split_pack_elems(int(which)))


def nature_pack_split(w1, w2, w3, q1, q2, q3, qd2=None, qd3=None, stream=None):
    call("ppox_nature_pack_split", _p(w1), _p(w2), _p(w3), _p(q1), _p(q2), _p(q3), _p(qd2), _p(qd3),
         stream_ptr(stream))


def _need_amax(x, slots, x_exp, stream, what):
    """the amax slots of an operand: given, computed (f32 x), or an error (a PX x has no f32 to scan)"""
    if slots is not None or x_exp is None:
        return _amax_of(x, slots, stream)
    raise ValueError(f"{what}: the amax slots of a PX (planes) operand must be passed (its producer records them)")


def nature_conv_fwd_split(layer, x, batch, idx, T, N_env, x_sample_stride, wq, bias, y, amax_x=None, amax_y=None,
                          relu_bits=None, x_exp=None, y_exp=None, stream=None):
    """amax_x: x's slots (layers 2, 3; computed here when None); amax_y: y's slots to record (or None);
    relu_bits: int32 ReLU bitmask of y to write (batch * P * C / 32 words; or None).  PX (layer 3):
    x_exp — x is h2 as planes, its exponent in this int32 element; y_exp — write y as planes, storing
    the exponent there (include/ppox.h)."""
    if layer != 1 and batch and (x_exp is None or y_exp is not None):
        amax_x = _need_amax(x, amax_x, x_exp, stream, "nature_conv_fwd_split")
    call("ppox_nature_conv_fwd_split", int(layer), _p(x), int(batch), _p(idx), int(T), int(N_env),
         int(x_sample_stride), _p(wq), _p(bias), _p(y), _p(amax_x) if layer != 1 else None, _p(amax_y),
         _p(relu_bits), _p(x_exp), _p(y_exp), stream_ptr(stream))


def normalize_obs_f32_ex(x, rows, cols, row_stride, mean, var, eps, clip, out, stream=None):
    _check_moments("ppox_normalize_obs_f32_ex", cols, mean, var)
    call("ppox_normalize_obs_f32_ex", _p(x), int(rows), int(cols), int(row_stride), _p(mean), _p(var), float(eps),
         float(clip), _p(out), stream_ptr(stream))


def vecnorm_reward(rewards, dones, ret, gamma, mean, var, count, eps, clip, update=True, stream=None):
    call("ppox_vecnorm_reward", _p(rewards), _p(dones), _p(ret), rewards.numel(), float(gamma), _p(mean), _p(var),
         float(count), float(eps), float(clip), int(bool(update)), stream_ptr(stream))


# NatureCNN fc layer 3136 -> 512 (split-f16 GEMM, csrc/conv.hip)
def nature_fc_pack_elems():
    return int(load().ppox_nature_fc_pack_elems())


def nature_fc_pack(w, q_fwd, q_dgrad, stream=None):
    call("ppox_nature_fc_pack", _p(w), _p(q_fwd), _p(q_dgrad), stream_ptr(stream))


def nature_pack_all(w1, w2, w3, wfc, wpd2, q1, q2, q3, qd2, qd3, qfc_fwd, qfc_dgrad, wh=None, qh_fwd=None,
                    qh_dgrad=None, b1=None, zero=None, b2=None, b3=None, stream=None):
    """Every weight packing of a training step in two launches (None = skip); q1 needs the conv1
    bias b1 (the H1P exponent of conv1's output is derived from W1 and b1); b2 / b3 give the PX
    output bounds of conv2 / conv3 their bias term; `zero` (an int32 tensor, e.g. the next pass's
    amax table) is zeroed on the way."""
    call("ppox_nature_pack_all", _p(w1), _p(b1), _p(w2), _p(b2), _p(w3), _p(b3), _p(wfc), _p(wpd2), _p(q1), _p(q2),
         _p(q3), _p(qd2), _p(qd3), _p(qfc_fwd), _p(qfc_dgrad), _p(wh), _p(qh_fwd), _p(qh_dgrad), _p(zero),
         0 if zero is None else zero.numel(), stream_ptr(stream))


def nature_pack_all_wmax(w1, w2, w3, wfc, wpd2, q1, q2, q3, qd2, qd3, qfc_fwd, qfc_dgrad, wh=None, qh_fwd=None,
                         qh_dgrad=None, b1=None, zero=None, b2=None, b3=None, amax_in=None, amax_next=None,
                         stream=None):
    """nature_pack_all with the weights' amax partials from adam_step_wmax (amax_in: one launch, no amax
    pass; None: the amax pass) and amax_next (the partials buffer the next adam_step_wmax records into)
    zeroed on the way"""
    for t in (amax_in, amax_next):
        assert t is None or t.numel() == WMAX_TENSORS * WMAX_SLOTS
    call("ppox_nature_pack_all_wmax", _p(w1), _p(b1), _p(w2), _p(b2), _p(w3), _p(b3), _p(wfc), _p(wpd2), _p(q1),
         _p(q2), _p(q3), _p(qd2), _p(qd3), _p(qfc_fwd), _p(qfc_dgrad), _p(wh), _p(qh_fwd), _p(qh_dgrad), _p(amax_in),
         _p(amax_next), _p(zero), 0 if zero is None else zero.numel(), stream_ptr(stream))


# conv1 -> conv2 on H1P (conv1's output as two f16 planes; include/ppox.h)
def nature_conv1_fwd_planes(x, batch, idx, T, N_env, x_sample_stride, wq1, bias, h1p, relu_bits=None, amax_y=None,
                            stream=None):
    call("ppox_nature_conv1_fwd_planes", _p(x), int(batch), _p(idx), int(T), int(N_env), int(x_sample_stride),
         _p(wq1), _p(bias), _p(h1p), _p(amax_y), _p(relu_bits), stream_ptr(stream))


def nature_conv2_fwd_planes(h1p, q1, batch, wq2, bias, y, amax_y=None, relu_bits=None, amax_x=None, y_exp=None,
                            stream=None):
    """conv2 forward on H1P; y_exp (PX output): y written as planes, its exponent stored there (the
    bound needs h1's amax slots amax_x, recorded by nature_conv1_fwd_planes)."""
    if y_exp is not None and amax_x is None:
        raise ValueError("nature_conv2_fwd_planes: a PX output needs h1's amax slots (amax_x)")
    call("ppox_nature_conv2_fwd_planes", _p(h1p), _p(q1), int(batch), _p(wq2), _p(bias), _p(y), _p(amax_x),
         _p(amax_y), _p(relu_bits), _p(y_exp), stream_ptr(stream))


def nature_conv2_wgrad_planes_workspace_bytes(batch):
    return int(load().ppox_nature_conv2_wgrad_planes_workspace_bytes(int(batch)))


def nature_conv2_wgrad_planes(h1p, q1, batch, grad_out, workspace, dw, db, amax_g=None, g_exp=None, stream=None):
    """dW2, db2 from H1P and the NHWC output grad (slabs + fixed-order reduce in one call): f32 g2 (its amax
    slots amax_g, computed here when None) or, g_exp given, g2 as PX planes with that exponent."""
    if g_exp is None:
        amax_g = _amax_of(grad_out, amax_g, stream)
    call("ppox_nature_conv2_wgrad_planes", _p(h1p), _p(q1), int(batch), _p(grad_out), _p(workspace),
         workspace.numel() * workspace.element_size(), _p(dw), _p(db), _p(amax_g), _p(g_exp), stream_ptr(stream))


def nature_fc_fwd(h3, batch, q_fwd, bias, f, amax_h3=None, amax_f=None, h3_exp=None, stream=None):
    """f = relu(h3 @ W^T + b), h3 (batch, 7, 7, 64) NHWC (h3_exp: as PX planes); amax_f: f's slots to
    record (or None)."""
    if batch and h3_exp is None:
        amax_h3 = _amax_of(h3, amax_h3, stream)
    call("ppox_nature_fc_fwd", _p(h3), int(batch), _p(q_fwd), _p(bias), _p(f), _p(amax_h3), _p(amax_f),
         _p(h3_exp), stream_ptr(stream))


# the heads' hidden layer Linear(512, 512) (split-f16 GEMM, csrc/conv.hip; include/ppox.h)
def head_hidden_pack_elems():
    return int(load().ppox_head_hidden_pack_elems())


def head_hidden_fwd(f, q_fwd, bias, e, amax_f=None, stream=None):
    """e = relu(f W^T + b) (rows x 512)."""
    rows = f.shape[0]
    if rows:
        amax_f = _amax_of(f, amax_f, stream)
    call("ppox_head_hidden_fwd", _p(f), rows, _p(q_fwd), _p(bias), _p(e), _p(amax_f), stream_ptr(stream))


def head_hidden_fwd_splitk_workspace_bytes(rows):
    return int(load().ppox_head_hidden_fwd_splitk_workspace_bytes(int(rows)))


def head_hidden_fwd_splitk(f, q_fwd, bias, workspace, e, amax_f=None, critic=None, value=None, stream=None):
    """e = relu(f W^T + b) split over K (small batches); with critic = (w (1 x 512), b) the reduce
    also writes value (rows,) = e w^T + b (bitwise as the skinny kernel)."""
    rows = f.shape[0]
    if rows:
        amax_f = _amax_of(f, amax_f, stream)
    wc, bc = critic if critic is not None else (None, None)
    call("ppox_head_hidden_fwd_splitk", _p(f), rows, _p(q_fwd), _p(bias), _p(workspace),
         workspace.numel() * workspace.element_size(), _p(e), _p(amax_f), _p(wc), _p(bc), _p(value),
         stream_ptr(stream))


def head_hidden_dgrad(de, q_dgrad, f, df, amax_de=None, amax_df=None, stream=None):
    """df = (f > 0) ? df + de W : 0, in place; amax_df: df's slots to record (or None)."""
    rows = de.shape[0]
    if rows:
        amax_de = _amax_of(de, amax_de, stream)
    call("ppox_head_hidden_dgrad", _p(de), rows, _p(q_dgrad), _p(f), _p(df), _p(amax_de), _p(amax_df),
         stream_ptr(stream))


def head_backward(dout, w_actor, dv, w_critic, e, f, q_dgrad, df, de, amax_de, amax_df, stream=None):
    """de = (e > 0) dv w_critic, df = (f > 0) (dout w_actor + de W) in one launch (ppox_head_backward)."""
    rows = e.shape[0]
    call("ppox_head_backward", _p(dout), _p(w_actor), _p(dv), _p(w_critic), _p(e), _p(f), _p(q_dgrad), rows,
         e.shape[1], dout.shape[1], _p(df), _p(de), _p(amax_de), _p(amax_df), stream_ptr(stream))


def head_hidden_wgrad_workspace_bytes(rows):
    return int(load().ppox_head_hidden_wgrad_workspace_bytes(int(rows)))


def head_hidden_wgrad(de, f, workspace, dw, amax_de=None, amax_f=None, stream=None):
    """dw (512 x 512) = de^T f, deterministic."""
    rows = de.shape[0]
    if rows:
        amax_de, amax_f = _amax_of(de, amax_de, stream), _amax_of(f, amax_f, stream)
    call("ppox_head_hidden_wgrad", _p(de), rows, _p(f), _p(workspace), workspace.numel() * workspace.element_size(),
         _p(dw), _p(amax_de), _p(amax_f), stream_ptr(stream))


def nature_fc_fwd_splitk_workspace_bytes(batch):
    return int(load().ppox_nature_fc_fwd_splitk_workspace_bytes(int(batch)))


def nature_fc_fwd_splitk(h3, batch, q_fwd, bias, workspace, f, amax_h3=None, amax_f=None, actor=None, logits=None,
                         h3_exp=None, stream=None):
    """fc forward split over K (small batches), bias + ReLU in the fixed-order reduce; with
    actor = (w, b) (<= 8 actions) the reduce also writes the actor head's logits = f w^T + b.
    h3_exp: h3 is PX planes."""
    if batch and h3_exp is None:
        amax_h3 = _amax_of(h3, amax_h3, stream)
    wa, ba = actor if actor is not None else (None, None)
    call("ppox_nature_fc_fwd_splitk", _p(h3), int(batch), _p(q_fwd), _p(bias), _p(workspace),
         workspace.numel() * workspace.element_size(), _p(f), _p(amax_h3), _p(amax_f), _p(wa), _p(ba),
         0 if wa is None else wa.shape[0], _p(logits), _p(h3_exp), stream_ptr(stream))


def nature_fc_dgrad(df, batch, q_dgrad, h3, g3, amax_df=None, amax_g3=None, relu_bits=None, g3_exp=None,
                    df_exp=None, stream=None):
    """g3 (batch, 7, 7, 64) NHWC = ((df @ W) in Flatten order) * (h3 > 0); amax_g3: g3's slots to record;
    relu_bits: h3's ReLU bitmask from the conv3 split forward (used instead of h3); g3_exp: write g3
    as PX planes, storing the exponent there (relu_bits required); df_exp: df is PX planes (px_split)
    with that exponent (amax_df still required)."""
    if batch and df_exp is None:
        amax_df = _amax_of(df, amax_df, stream)
    call("ppox_nature_fc_dgrad", _p(df), int(batch), _p(q_dgrad), _p(h3), _p(g3), _p(amax_df), _p(amax_g3),
         _p(relu_bits), _p(g3_exp), _p(df_exp), stream_ptr(stream))


def nature_fc_wgrad_workspace_bytes(batch):
    return int(lib().ppox_nature_fc_wgrad_workspace_bytes(int(batch)))


def nature_fc_wgrad(df, batch, h3, workspace, dw, amax_df=None, amax_h3=None, h3_exp=None, df_exp=None,
                    stream=None):
    """dw (512, 3136) in the fc weight's Flatten order = df^T @ h3 (h3 NHWC (batch, 7, 7, 64); h3_exp /
    df_exp: that operand as PX planes)."""
    if batch:
        if df_exp is None:
            amax_df = _amax_of(df, amax_df, stream)
        if h3_exp is None:
            amax_h3 = _amax_of(h3, amax_h3, stream)
    call("ppox_nature_fc_wgrad", _p(df), int(batch), _p(h3), _p(workspace), workspace.numel() * workspace.element_size(),
         _p(dw), _p(amax_df), _p(amax_h3), _p(h3_exp), _p(df_exp), stream_ptr(stream))


def px_split(x, amax, y, exp_out, stream=None):
    """y (int16, x's bytes) = the PX planes of f32 x at the split scale of its amax slots; the
    exponent into exp_out (one int32)."""
    assert x.is_contiguous() and x.dtype == torch.float32 and x.numel() % 32 == 0
    assert y.dtype == torch.int16 and y.numel() == 2 * x.numel()
    call("ppox_px_split", _p(x), x.numel(), _p(amax), _p(y), _p(exp_out), stream_ptr(stream))


# ES-NSRA (csrc/es.hip)
def es_noise(P, n_params, member0, generation, seed, eps, stream=None):
    call("ppox_es_noise", int(P), int(n_params), int(member0), int(generation), int(seed) & 0xFFFFFFFFFFFFFFFF,
         _p(eps), stream_ptr(stream))


def es_env_noise(T, D, env_seed, xi, stream=None):
    call("ppox_es_env_noise", int(T), int(D), int(env_seed) & 0xFFFFFFFFFFFFFFFF, _p(xi), stream_ptr(stream))


def es_evaluate(w, eps, sigma, P, D, H1, H2, A, T, env_seed, xi, fitness, bc=None, stream=None):
    call("ppox_es_evaluate", _p(w), _p(eps), float(sigma), int(P), int(D), int(H1), int(H2), int(A), int(T),
         int(env_seed) & 0xFFFFFFFFFFFFFFFF, _p(xi), _p(fitness), _p(bc), stream_ptr(stream))


def es_update_workspace_bytes(P, n_params):
    return int(load().ppox_es_update_workspace_bytes(int(P), int(n_params)))


def es_update(eps, coef, P, n_params, workspace, out, stream=None):
    call("ppox_es_update", _p(eps), _p(coef), int(P), int(n_params), _p(workspace),
         workspace.numel() * workspace.element_size(), _p(out), stream_ptr(stream))


def relu_backward_(grad, act, amax=None, stream=None):
    """grad = act > 0 ? grad : 0, in place (same-shape contiguous f32); amax: slots recording max |grad|."""
    if amax is None:
        call("ppox_relu_backward_", _p(grad), _p(act), grad.numel(), stream_ptr(stream))
    else:
        call("ppox_relu_backward_amax_", _p(grad), _p(act), grad.numel(), _p(amax), stream_ptr(stream))


def _aligned(t):
    return t.data_ptr() % 16 == 0


def head_linear(x, w, b):
    """x w^T + b for the actor / critic heads: the skinny-row kernel for <= 8 outputs on
    16-byte-aligned operands, the library GEMM otherwise (e.g. 18 Montezuma actions)."""
    rows, h = x.shape
    n = w.shape[0]
    if n <= 8 and h % 4 == 0 and x.is_contiguous() and _aligned(x) and _aligned(w) and w.is_contiguous():
        y = torch.empty(rows, n, device=x.device)
        call("ppox_skinny_linear", _p(x), _p(w), _p(b), rows, h, n, _p(y), stream_ptr(None))
        return y
    return torch.addmm(b, x, w.t())


def head_dgrad(g, w):
    """g (rows x n) @ w (n x h) for the actor head's input grad (same dispatch as head_linear)."""
    rows, n = g.shape
    h = w.shape[1]
    if n <= 8 and h % 4 == 0 and g.is_contiguous() and _aligned(w) and w.is_contiguous():
        d = torch.empty(rows, h, device=g.device)
        call("ppox_skinny_dgrad", _p(g), _p(w), rows, h, n, _p(d), stream_ptr(None))
        return d
    return torch.mm(g, w)


def u8_to_f32(x, out=None, stream=None):
    """float copy of a contiguous uint8 tensor (same shape)."""
    out = torch.empty(x.shape, dtype=torch.float32, device=x.device) if out is None else out
    call("ppox_u8_to_f32", _p(x), x.numel(), _p(out), stream_ptr(stream))
    return out


def head_grads_workspace_bytes(rows, h, n_actions, intrinsic):
    n = int(lib().ppox_head_grads_workspace_bytes(int(rows), int(h), int(n_actions), int(bool(intrinsic))))
    if n < 0:
        raise RuntimeError("ppox_head_grads_workspace_bytes: unsupported head shape")
    return n


def head_grads(f, e, dout, dv, de, df, ws, w_actor, b_actor, w_critic, b_critic, b_extra, b_fc,
               ie=None, div=None, die=None, w_critic_int=None, b_critic_int=None, b_int_extra=None, relu_df=False,
               amax_df=None, df_planes=None, df_planes_amax=None, df_planes_exp=None, stream=None):
    """Column-reduction head gradients (see include/ppox.h ppox_head_grads); outputs overwritten.
    relu_df: df is first masked by f's ReLU in place (amax_df: its slots to record).  df_planes: df's PX planes
    (int16, rows x 2h) written in the same pass at the exponent of df_planes_amax, stored to df_planes_exp."""
    call("ppox_head_grads", _p(f), _p(e), _p(dout), _p(dv), _p(de), _p(df), _p(ie), _p(div), _p(die),
         f.shape[0], f.shape[1], dout.shape[1], _p(ws), _p(w_actor), _p(b_actor), _p(w_critic), _p(b_critic),
         _p(b_extra), _p(b_fc), _p(w_critic_int), _p(b_critic_int), _p(b_int_extra), int(bool(relu_df)),
         _p(amax_df), _p(df_planes), _p(df_planes_amax), ptr(df_planes_exp, torch.int32, name="df_planes_exp"),
         stream_ptr(stream))


def head_dgrad_outer(dout, w_actor, dv, w_critic, e, amax_de=None):
    """(df, de): the actor head's input grad dout w_actor and the critic's ReLU-layer grad
    dv w_critic (e > 0) in one launch (ppox_head_dgrad_outer; <= 8 actions, aligned operands),
    else the two separate kernels."""
    rows, n = dout.shape
    h = w_actor.shape[1]
    df = torch.empty(rows, h, device=dout.device)
    de = torch.empty_like(e)
    if n <= 8 and h % 4 == 0 and dout.is_contiguous() and _aligned(w_actor) and w_actor.is_contiguous():
        call("ppox_head_dgrad_outer", _p(dout), _p(w_actor), _p(dv), _p(w_critic), _p(e), rows, h, n, _p(df), _p(de),
             _p(amax_de), stream_ptr(None))
        return df, de
    df = torch.mm(dout, w_actor)
    outer_relu_backward(dv, w_critic, e, de, amax=amax_de)
    return df, de


def outer_relu_backward(dv, w, act, out, amax=None, stream=None):
    """out[b][j] = dv[b] * w[j] * (act[b][j] > 0); amax: out's slots to record (or None)."""
    call("ppox_outer_relu_backward", _p(dv), _p(w), _p(act), act.shape[0], act.shape[1], _p(out), _p(amax),
         stream_ptr(stream))


def nature_wgrad_split_workspace_bytes(layer, batch):
    return int(load().ppox_nature_wgrad_split_workspace_bytes(int(layer), int(batch)))


def nature_conv_wgrad_split(layer, x, batch, x_sample_stride, grad_out, workspace, dw, db, amax_x=None, amax_g=None,
                            x_exp=None, g_exp=None, stream=None):
    """dW, db of one conv layer (slabs + fixed-order reduce in one call), split-f16 MFMA; x_exp / g_exp
    (layer 3): x / grad_out are PX planes."""
    if g_exp is None:
        amax_g = _amax_of(grad_out, amax_g, stream)
    if layer != 1 and x_exp is None:
        amax_x = _amax_of(x, amax_x, stream)
    call("ppox_nature_conv_wgrad_split", int(layer), _p(x), int(batch), int(x_sample_stride), _p(grad_out),
         _p(workspace), workspace.numel() * workspace.element_size(), _p(dw), _p(db),
         _p(amax_x) if layer != 1 else None, _p(amax_g), _p(x_exp), _p(g_exp), stream_ptr(stream))


def nature_conv_wgrad_split_idx(layer, x, batch, idx, T, N_env, grad_out, workspace, dw, db, amax_g=None,
                                stream=None):
    """conv1 dW, db from the step-major (T, N_env, 4, 84, 84) rollout frames through env-major
    rows idx (the minibatch gather fused), split-f16 MFMA."""
    amax_g = _amax_of(grad_out, amax_g, stream)
    call("ppox_nature_conv_wgrad_split_idx", int(layer), _p(x), int(batch), _p(idx), int(T), int(N_env),
         _p(grad_out), _p(workspace), workspace.numel() * workspace.element_size(), _p(dw), _p(db), _p(amax_g),
         stream_ptr(stream))


def nature_conv_dgrad_split(layer, grad_out, batch, wqd, prev_act, grad_in, amax_g=None, amax_out=None,
                            relu_bits=None, g_exp=None, y_exp=None, stream=None):
    """amax_g: grad_out's slots (computed here when None); amax_out: grad_in's slots to record (or None);
    relu_bits: the ReLU bitmask of the layer below from its split forward, used instead of prev_act;
    g_exp: grad_out is PX planes with that exponent (layer 3: g3; layer 2: g2 — the direct form);
    y_exp (layer 3): write g2 as PX planes, storing the exponent there (relu_bits and amax_g required)."""
    if batch and g_exp is None:
        amax_g = _amax_of(grad_out, amax_g, stream)
    call("ppox_nature_conv_dgrad_split", int(layer), _p(grad_out), int(batch), _p(wqd), _p(prev_act), _p(grad_in),
         _p(amax_g), _p(amax_out), _p(relu_bits), _p(g_exp), _p(y_exp), stream_ptr(stream))


# ---------------------------------------------------------------------------
# K11 ICM on image observations (csrc/icm.hip; see include/ppox.h)
# ---------------------------------------------------------------------------
def icm_param_elems(n_actions):
    return int(load().ppox_icm_param_elems(int(n_actions)))


def icm_w1_pack_elems(K):
    return int(load().ppox_icm_w1_pack_elems(int(K)))


def icm_encode_workspace_bytes(rows, K):
    return int(load().ppox_icm_encode_workspace_bytes(int(rows), int(K)))


def icm_partials_bytes(rows, n_actions):
    return int(load().ppox_icm_partials_bytes(int(rows), int(n_actions)))


def icm_g1_pack_elems(rows):
    return int(load().ppox_icm_g1_pack_elems(int(rows)))


def icm_pack_w1(w1, q, stream=None):
    call("ppox_icm_pack_w1", ptr(w1, torch.float32, name="w1"), int(w1.shape[1]), ptr(q, torch.int16, name="q"),
         stream_ptr(stream))


def icm_encode(x, rows, idx, T, N_env, K, q, seg, workspace, pre1, phi, rowno=None, stream=None):
    """pre1 / phi (rows x 32) of `rows` uint8 frame rows of K bytes (x contiguous rows, or the
    step-major rollout frames read through env-major rows idx)."""
    call("ppox_icm_encode", _p(x), int(rows), _p(idx), int(T), int(N_env), int(K), _p(q), _p(seg), _p(workspace),
         _p(pre1), _p(phi), _p(rowno), stream_ptr(stream))


def icm_pair_backward(phi, B, actions, rowno, pairs, n_pairs, n_pairs_global, n_actions, beta, seg, dS, dN,
                      partials, stream=None):
    call("ppox_icm_pair_backward", _p(phi), int(B), ptr(actions, torch.int32, name="actions"), _p(rowno), _p(pairs),
         int(n_pairs), int(n_pairs_global), int(n_actions), float(beta), _p(seg), _p(dS), _p(dN), _p(partials),
         stream_ptr(stream))


def icm_scatter_positions(phi, actions, rowno, pos, rows, B, fa, stream=None):
    """fa = [B x 32 | B actions as f32]: this rank's rows at their minibatch positions, zero elsewhere."""
    call("ppox_icm_scatter_positions", _p(phi), _p(actions), _p(rowno), _p(pos), int(rows), int(B), _p(fa),
         stream_ptr(stream))


def icm_row_backward(dS, dN, pos, rows, pre1, seg, n_actions, g1q, partials, stream=None):
    call("ppox_icm_row_backward", _p(dS), _p(dN), _p(pos), int(rows), _p(pre1), _p(seg), int(n_actions), _p(g1q),
         _p(partials), stream_ptr(stream))


def icm_grad_reduce(partials, rows, n_pairs, n_actions, beta, n_pairs_global, grad_seg, loss_accum=None,
                    stream=None):
    call("ppox_icm_grad_reduce", _p(partials), int(rows), int(n_pairs), int(n_actions), float(beta),
         int(n_pairs_global), _p(grad_seg), ptr(loss_accum, torch.float64, name="loss_accum"), stream_ptr(stream))


def icm_enc_wgrad(x, rowno, rows, K, g1q, dw1, stream=None):
    call("ppox_icm_enc_wgrad", _p(x), ptr(rowno, torch.int32, name="rowno"), int(rows), int(K), _p(g1q),
         ptr(dw1, torch.float32, name="dw1"), stream_ptr(stream))


def icm_int_reward(phi_s, phi_n, actions, N, n_actions, seg, eta, rewards, int_rewards, stream=None):
    call("ppox_icm_int_reward", _p(phi_s), _p(phi_n), ptr(actions, torch.int32, name="actions"), int(N),
         int(n_actions), _p(seg), float(eta), ptr(rewards, torch.float32, name="rewards"),
         ptr(int_rewards, torch.float32, name="int_rewards"), stream_ptr(stream))


# ---------------------------------------------------------------------------
# Data-parallel exchange (RCCL from native code; dist.DistContext drives it)
# ---------------------------------------------------------------------------
def rccl_path():
    """The RCCL library torch loaded (torch/lib/librccl.so on ROCm builds)."""
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    if not os.path.exists(p):
        raise ImportError(f"no RCCL at {p}")
    return p


class DpComm:
    """One RCCL communicator over the job's ranks with its own stream (csrc/dp.cpp).  Construct on every
    rank in the same order: `broadcast_id(buf)` must hand rank 0's id bytes to every rank (a collective
    over the process group that already exists)."""

    def __init__(self, world, rank, device, broadcast_id, rccl=None):
        l = lib()
        call("ppox_dp_load", (rccl or rccl_path()).encode())
        n = l.ppox_dp_unique_id_bytes()
        buf = (ctypes.c_uint8 * n)()
        if rank == 0:
            call("ppox_dp_unique_id", buf)
        buf = (ctypes.c_uint8 * n).from_buffer_copy(broadcast_id(bytes(buf)))
        h = _vp()
        call("ppox_dp_comm_init", buf, world, rank, device, ctypes.byref(h))
        self.handle, self.world, self.rank, self.inflight = h, world, rank, False

    def all_reduce_(self, t, wait=True, stream=None):
        """In-place SUM over ranks of a contiguous float32 / float64 device tensor, ordered after the work on
        `stream` (default: the current stream) and after the communicator's previous reduction; wait: that
        stream waits for it (else join with wait() — one asynchronous reduction at a time: a second one
        before the join raises)."""
        if not self.handle:
            raise NativeError("DpComm.all_reduce_: the communicator is closed")
        if not wait and self.inflight:
            raise NativeError("DpComm.all_reduce_: an asynchronous reduction is in flight (wait() first)")
        dt = 0 if t.dtype == torch.float32 else 1 if t.dtype == torch.float64 else None
        if dt is None or not t.is_cuda or not t.is_contiguous():
            raise TypeError(f"DpComm.all_reduce_: contiguous float32/float64 device tensor, got {t.dtype} "
                            f"on {t.device}")
        call("ppox_dp_all_reduce", self.handle, _p(t), t.numel(), dt, 1 if wait else 0, stream_ptr(stream))
        self.inflight = not wait and t.numel() > 0
        return t

    def wait(self, stream=None):
        call("ppox_dp_wait", self.handle, stream_ptr(stream))
        self.inflight = False

    def close(self):
        """Sync and destroy (ppox_dp_comm_destroy); returns its status, 0.  Idempotent."""
        if not self.handle:
            return 0
        h, self.handle = self.handle, None
        call("ppox_dp_comm_destroy", h)
        return 0


# ---------------------------------------------------------------------------
# Stream ordering with device-scope events (convs.fork / join)
# ---------------------------------------------------------------------------
EVENT_RELEASE_TO_DEVICE, EVENT_DISABLE_SYSTEM_FENCE = 0x40000000, 0x20000000  # hipEventCreateWithFlags


def event_create(flags):
    h = _vp()
    call("ppox_event_create", int(flags), ctypes.byref(h))
    return h


def stream_order(event, record_stream, wait_stream):
    """wait_stream waits for everything enqueued so far on record_stream (torch streams)."""
    call("ppox_stream_order", event, _vp(record_stream.cuda_stream), _vp(wait_stream.cuda_stream))
