"""ctypes mirror of include/heligym_amd.h and the loader of the native library.

The library `libheligym_amd.so` (HIP kernels for gfx950 + the C-ABI + host trim) is built
in-tree by `__graft_entry__.build()`.  There is no fallback: if it is missing or its HIP runtime
cannot run, every device call raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HELIGYM_AMD_LIB") or os.path.join(_HERE, "libheligym_amd.so")

HG_N_OBS = 17
HG_N_ACT = 4
HG_N_HELI = 18
HG_N_WIND = 5
HG_N_CARRY = 4
HG_STATE_COLS = HG_N_HELI + HG_N_WIND + HG_N_CARRY
HG_COUNTER_COLS = 3

HG_OK = 0
HG_TASK_HELI, HG_TASK_HOVER, HG_TASK_FORWARD_FLIGHT = 0, 1, 2
HG_INFO_FAILED, HG_INFO_SUCCESSED, HG_INFO_TIME_UP, HG_INFO_SUCCESS_STEP, HG_INFO_RESET = 1, 2, 4, 8, 16
HG_RESET_TEMPLATE, HG_RESET_RETRIM = 0, 1
RESET_MODES = {"template": HG_RESET_TEMPLATE, "retrim": HG_RESET_RETRIM}
HG_AUTORESET_SAME_STEP, HG_AUTORESET_NEXT_STEP = 0, 1
AUTORESET_MODES = {"same_step": HG_AUTORESET_SAME_STEP, "next_step": HG_AUTORESET_NEXT_STEP}
HG_ABI_VERSION = 3

AIRFRAME_FIELDS = (
    ["env_R", "env_T0", "env_LAPSE", "env_RO_SEA", "env_GRAV", "env_MAX_GR_ALT", "env_NS_MAX",
     "env_EW_MAX", "env_WIND_DIR_deg", "env_WIND_SPD"],
    ["HP_LOSS", "VTRANS", "FS_CG", "WL_CG", "WT", "IX", "IY", "IZ", "IXZ", "COL_OS", "COL_L", "COL_H",
     "LON_L", "LON_H", "LAT_L", "LAT_H", "PED_OS", "PED_L", "PED_H",
     "mr_FS", "mr_WL", "mr_IS", "mr_E", "mr_IB", "mr_R", "mr_A", "mr_RPM", "mr_CD0", "mr_B", "mr_C",
     "mr_TWST", "mr_K1",
     "tr_FS", "tr_WL", "tr_R", "tr_A", "tr_C", "tr_RPM", "tr_CD0", "tr_TWST", "tr_B",
     "fus_FS", "fus_WL", "fus_XUU", "fus_YVV", "fus_ZWW", "fus_COR",
     "ht_FS", "ht_WL", "ht_ZUU", "ht_ZUW", "ht_ZMAX",
     "vt_FS", "vt_WL", "vt_YUU", "vt_YUV", "vt_YMAX",
     "wn_FS", "wn_WL", "wn_ZUU", "wn_ZUW", "wn_ZMAX", "wn_B",
     "lg_K", "lg_C", "lg_BL_MN", "lg_FS_MN", "lg_FS_N", "lg_WL"],
)


class hg_airframe(ctypes.Structure):
    _fields_ = ([(n, ctypes.c_double) for n in AIRFRAME_FIELDS[0]]
                + [("env_TURB_LVL", ctypes.c_int32), ("_pad0", ctypes.c_int32)]
                + [(n, ctypes.c_double) for n in AIRFRAME_FIELDS[1]])


class hg_trim_cond(ctypes.Structure):
    _fields_ = [("yaw", ctypes.c_double), ("yaw_rate", ctypes.c_double),
                ("ned_vel", ctypes.c_double * 3), ("gr_alt", ctypes.c_double),
                ("xy", ctypes.c_double * 2), ("psi_mr", ctypes.c_double), ("psi_tr", ctypes.c_double)]


class hg_target(ctypes.Structure):
    _fields_ = [("north_loc", ctypes.c_double), ("east_loc", ctypes.c_double),
                ("sea_alt", ctypes.c_double), ("heading", ctypes.c_double), ("vel", ctypes.c_double)]


class hg_config(ctypes.Structure):
    _fields_ = [("af", hg_airframe), ("trim", hg_trim_cond), ("target", hg_target),
                ("dt", ctypes.c_double), ("max_time", ctypes.c_double),
                ("task", ctypes.c_int32), ("autoreset", ctypes.c_int32),
                ("seed", ctypes.c_uint64), ("env_offset", ctypes.c_int64),
                ("reset_mode", ctypes.c_int32), ("autoreset_mode", ctypes.c_int32),
                ("max_episode_steps", ctypes.c_int64)]


class hg_trim_result(ctypes.Structure):
    _fields_ = [("state", ctypes.c_double * HG_N_HELI), ("action", ctypes.c_double * HG_N_ACT),
                ("obs", ctypes.c_double * HG_N_OBS), ("state_dots", ctypes.c_double * HG_N_HELI),
                ("residual", ctypes.c_double), ("iterations", ctypes.c_int32),
                ("failed", ctypes.c_int32)]


# Every symbol include/heligym_amd.h declares, with its ctypes signature.
_P = ctypes.c_void_p
_SIGS = {
    "hg_abi_version": (ctypes.c_int32, []),
    "hg_last_error": (ctypes.c_char_p, []),
    "hg_default_config": (None, [ctypes.POINTER(hg_config)]),
    "hg_trim": (ctypes.c_int32, [ctypes.POINTER(hg_config), _P, ctypes.c_int32, ctypes.c_int32,
                                 ctypes.POINTER(ctypes.c_double), ctypes.POINTER(hg_trim_result)]),
    "hg_create": (ctypes.c_int32, [ctypes.POINTER(hg_config), _P, ctypes.c_int32, ctypes.c_int32,
                                   ctypes.c_int64, ctypes.POINTER(_P)]),
    "hg_destroy": (None, [_P]),
    "hg_num_envs": (ctypes.c_int64, [_P]),
    "hg_set_max_time": (ctypes.c_int32, [_P, ctypes.c_double]),
    "hg_set_target": (ctypes.c_int32, [_P, ctypes.POINTER(hg_target)]),
    "hg_set_specialized": (ctypes.c_int32, [_P, ctypes.c_int32]),
    "hg_load_specialized": (ctypes.c_int32, [_P, ctypes.c_char_p, ctypes.c_int32, _P, ctypes.c_int64]),
    "hg_set_trim_cond": (ctypes.c_int32, [_P, ctypes.POINTER(hg_trim_cond)]),
    "hg_get_template": (ctypes.c_int32, [_P, ctypes.POINTER(hg_trim_result)]),
    "hg_reset": (ctypes.c_int32, [_P, _P, _P, _P]),
    "hg_step": (ctypes.c_int32, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "hg_step_chained": (ctypes.c_int32, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "hg_step_rows": (ctypes.c_int32, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "hg_get_state": (ctypes.c_int32, [_P, _P, _P, _P]),
    "hg_set_state": (ctypes.c_int32, [_P, _P, _P, _P]),
    "hg_random_actions": (ctypes.c_int32, [_P, _P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_float,
                                           ctypes.c_float, _P]),
    "hg_rollout": (ctypes.c_int32, [_P, _P, ctypes.c_int32, _P, _P, _P, _P, _P, _P, _P]),
    "hg_trim_batch": (ctypes.c_int32, [_P, _P, ctypes.c_int64, _P, _P, _P, _P, _P]),
    "hg_retrim_failures": (ctypes.c_int32, [_P, ctypes.POINTER(ctypes.c_int64)]),
    "hg_set_retrim_overlap": (ctypes.c_int32, [_P, ctypes.c_int32]),
    "hg_debug_retrim_invalid": (ctypes.c_int32, [_P, ctypes.POINTER(ctypes.c_int64)]),
    "hg_debug_retrim_solves": (ctypes.c_int32, [_P, ctypes.POINTER(ctypes.c_int64)]),
    "hg_debug_queues": (ctypes.c_int32, [_P, ctypes.POINTER(ctypes.c_int32)]),
    "hg_debug_launches": (ctypes.c_int32, [_P, ctypes.POINTER(ctypes.c_int64)]),
    "hg_clock_stamp": (ctypes.c_int32, [_P, _P]),
    "hg_debug_eta": (ctypes.c_int32, [_P, _P, _P]),
    "hg_debug_philox": (ctypes.c_int32, [_P, _P, ctypes.c_int64, _P]),
    "hg_trim_conds_batch": (ctypes.c_int32, [_P, ctypes.POINTER(hg_trim_cond), ctypes.c_int64, _P, _P, _P, _P,
                                             _P, _P]),
    "hg_set_reset_templates": (ctypes.c_int32, [_P, _P, _P]),
    "hg_debug_params": (ctypes.c_int32, [ctypes.POINTER(hg_config), ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                         _P, ctypes.c_int64]),
    "hg_config_is_baked": (ctypes.c_int32, [ctypes.POINTER(hg_config), ctypes.c_int32, ctypes.c_int32]),
    "hg_host_alloc": (ctypes.c_int32, [ctypes.c_int64, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p)]),
    "hg_host_free": (None, [_P]),
}
EXPORTED_SYMBOLS = tuple(_SIGS)

_lib = None


class HeliGymError(RuntimeError):
    pass


def load_library(path=None):
    """Load libheligym_amd.so (once).  Import torch first so the library binds to the HIP runtime
    torch already loaded (both carry the SONAME libamdhip64.so.7)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise HeliGymError(
            f"native library {p} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            " (no CPU fallback exists)")
    try:
        import torch  # noqa: F401  (shared HIP runtime)
    except ImportError:
        pass
    lib = ctypes.CDLL(p)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.hg_abi_version() != HG_ABI_VERSION:
        raise HeliGymError("ABI version mismatch")
    if path is None:
        _lib = lib
    return lib


def check(rc, lib=None):
    if rc != HG_OK:
        lib = lib or load_library()
        msg = lib.hg_last_error()
        raise HeliGymError(f"heligym_amd error {rc}: {msg.decode() if msg else ''}")
    return rc
