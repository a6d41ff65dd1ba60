"""Airframe / task configuration: our parameter file -> `hg_config` (include/heligym_amd.h).

Mirrors what the reference does in Heli.__init__ (heligym/envs/helicopter.py:47-62: yaml load,
DT, default max time / target / trim condition) and the task constructors
(heligym/envs/helicopter_with_tasks.py:6-25, 56-76).
"""
import copy
import os

import numpy as np
import yaml

from . import _abi

_HERE = os.path.dirname(os.path.abspath(__file__))

FPS = 50.0
DT = 1.0 / FPS                       # helicopter.py:18-19
DEFAULT_MAX_TIME = 40.0              # helicopter.py:33-34
DEFAULT_TRIM_COND = {                # helicopter.py:36-44
    "yaw": 0.0, "yaw_rate": 0.0, "ned_vel": [0.0, 0.0, 0.0], "gr_alt": 100.0,
    "xy": [0.0, 0.0], "psi_mr": 0.0, "psi_tr": 0.0,
}
TASKS = {"heli": _abi.HG_TASK_HELI, "hover": _abi.HG_TASK_HOVER,
         "forward_flight": _abi.HG_TASK_FORWARD_FLIGHT}
# Task targets: helicopter_with_tasks.py:9-13 (hover) and :59-63 (forward flight).
DEFAULT_TARGETS = {
    "heli": {},
    "hover": {"sea_alt": 4000.0, "north_loc": 0.0, "east_loc": 0.0},
    "forward_flight": {"sea_alt": 4000.0, "heading": 0.0, "vel": 100.0},
}
TARGET_KEYS = ("north_loc", "east_loc", "sea_alt", "heading", "vel")


# The reference's airframe schema (heligym/envs/helis/aw109.yaml): ENV / HELI sections, rotor and
# surface sub-sections under HELI.  Keys map onto the flat hg_airframe names used here.
_REF_ENV_KEYS = {"R": "env_R", "T0": "env_T0", "LAPSE": "env_LAPSE", "RO_SEA": "env_RO_SEA",
                 "GRAV": "env_GRAV", "MAX_GR_ALT": "env_MAX_GR_ALT", "NS_MAX": "env_NS_MAX",
                 "EW_MAX": "env_EW_MAX", "WIND_DIR": "env_WIND_DIR_deg", "WIND_SPD": "env_WIND_SPD",
                 "TURB_LVL": "env_TURB_LVL"}
_REF_SECTIONS = {"MR": "mr_", "TR": "tr_", "FUS": "fus_", "HT": "ht_", "VT": "vt_", "WN": "wn_", "LG": "lg_"}
BUNDLED_TERRAIN = "assets/terrain_hmap_u16.npz"


def airframe_from_reference_schema(ref, resource_dir=None):
    """Convert a parameter document in the reference's schema (helicopter.py:49-54 loads it;
    ENV, HELI and HELI.{MR,TR,FUS,HT,VT,WN,LG}) into this package's {"airframe", "terrain"} doc.
    The terrain is ENV.HMAP_PATH under `resource_dir` (the reference's HELIGYM_RESOURCE_DIR,
    helicopter_dynamics.py:39); the reference's own map resolves to the bundled derived copy."""
    env, heli = ref["ENV"], ref["HELI"]
    af = {dst: env[src] for src, dst in _REF_ENV_KEYS.items()}
    for k, v in heli.items():
        if k in _REF_SECTIONS:
            af.update({_REF_SECTIONS[k] + kk: vv for kk, vv in v.items()})
        else:
            af[k] = v
    missing = [n for n in _abi.AIRFRAME_FIELDS[0] + _abi.AIRFRAME_FIELDS[1] + ["env_TURB_LVL"] if n not in af]
    if missing:
        raise ValueError(f"airframe document lacks {missing}")
    terrain = {"file": BUNDLED_TERRAIN}
    hmap = env.get("HMAP_PATH")
    if hmap:
        root = resource_dir if resource_dir is not None else os.environ.get("HELIGYM_RESOURCE_DIR", "")
        path = root + hmap
        if os.path.exists(path):
            terrain = {"file": path}
        elif os.path.basename(hmap) != "terrain_hmap.png":
            raise FileNotFoundError(f"terrain {path} not found (set HELIGYM_RESOURCE_DIR)")
    return {"airframe": af, "terrain": terrain}


def load_airframe(heli_name="aw109", resource_dir=None):
    """Parameter document for `heli_name`: a bundled airframe ("aw109", helis/<name>.yaml), or a
    path to a YAML file in either this package's schema or the reference's (helis/aw109.yaml)."""
    if isinstance(heli_name, dict):
        doc = heli_name
    else:
        path = heli_name if heli_name.endswith((".yaml", ".yml")) else os.path.join(_HERE, "helis", heli_name + ".yaml")
        with open(path) as f:
            doc = yaml.safe_load(f)
    if "ENV" in doc and "HELI" in doc:
        doc = airframe_from_reference_schema(doc, resource_dir)
    return doc


def read_terrain(path):
    """uint16 [rows, cols] height samples from a .npz (key "hmap") or a 16-bit grayscale PNG."""
    if path.endswith(".npz"):
        with np.load(path, allow_pickle=False) as z:
            return np.ascontiguousarray(z["hmap"], dtype=np.uint16)
    from PIL import Image
    with Image.open(path) as im:
        a = np.asarray(im)
    if a.ndim == 3:
        a = a[..., 0]
    return np.ascontiguousarray(a, dtype=np.uint16)


def load_terrain(doc):
    """uint16 [rows, cols] samples of the document's terrain (helicopter_dynamics.py:39-43)."""
    f = doc["terrain"]["file"]
    return read_terrain(f if os.path.isabs(f) else os.path.join(_HERE, f))


def terrain_ft(u16, max_gr_alt):
    """Heights in ft, fp64 exactly as the reference computes them: png / 65535 * MAX_GR_ALT."""
    return np.ascontiguousarray((u16.astype(np.float64) / 65535.0) * max_gr_alt)


def fill_trim(tc, trim_cond):
    d = copy.deepcopy(DEFAULT_TRIM_COND)
    d.update(trim_cond or {})
    tc.yaw, tc.yaw_rate = float(d["yaw"]), float(d["yaw_rate"])
    for i in range(3):
        tc.ned_vel[i] = float(d["ned_vel"][i])
    tc.gr_alt = float(d["gr_alt"])
    tc.xy[0], tc.xy[1] = float(d["xy"][0]), float(d["xy"][1])
    tc.psi_mr, tc.psi_tr = float(d["psi_mr"]), float(d["psi_tr"])
    return d


def fill_target(tg, target):
    t = dict.fromkeys(TARGET_KEYS, 0.0)
    t.update(target or {})
    for k in TARGET_KEYS:
        setattr(tg, k, float(t[k]))
    return t


def make_config(task="hover", dt=DT, heli_name="aw109", max_time=None, target=None,
                trim_cond=None, autoreset=True, seed=0, env_offset=0, turbulence_level=None,
                reset_mode="template", autoreset_mode="same_step", max_episode_steps=None):
    doc = load_airframe(heli_name)
    cfg = _abi.hg_config()
    af = doc["airframe"]
    for name, _ in _abi.hg_airframe._fields_:
        if name == "_pad0":
            continue
        if name == "env_TURB_LVL":
            cfg.af.env_TURB_LVL = int(af[name] if turbulence_level is None else turbulence_level)
        else:
            setattr(cfg.af, name, float(af[name]))
    if task not in TASKS:
        raise ValueError(f"unknown task {task!r}; one of {sorted(TASKS)}")
    fill_trim(cfg.trim, trim_cond)
    tgt = dict(DEFAULT_TARGETS[task])
    tgt.update(target or {})
    fill_target(cfg.target, tgt)
    cfg.dt = float(dt)
    cfg.max_time = float(DEFAULT_MAX_TIME if max_time is None else max_time)
    cfg.task = TASKS[task]
    cfg.autoreset = 1 if autoreset else 0
    cfg.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    cfg.env_offset = int(env_offset)
    if reset_mode not in _abi.RESET_MODES:
        raise ValueError(f"unknown reset_mode {reset_mode!r}; one of {sorted(_abi.RESET_MODES)}")
    cfg.reset_mode = _abi.RESET_MODES[reset_mode]
    if autoreset_mode not in _abi.AUTORESET_MODES:
        raise ValueError(f"unknown autoreset_mode {autoreset_mode!r}; one of {sorted(_abi.AUTORESET_MODES)}")
    cfg.autoreset_mode = _abi.AUTORESET_MODES[autoreset_mode]
    cfg.max_episode_steps = int(max_episode_steps or 0)
    return cfg, doc
