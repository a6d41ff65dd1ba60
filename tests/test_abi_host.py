"""CPU-side checks of the product library: it loads, exports every symbol include/heligym_amd.h
declares, its host trim (the reset template) matches the reference's trim, and argument errors
are reported through error codes.  No device calls."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT, load_golden, trim_dict
import golden_cases

from heligym_amd import _abi, config

HEADER = os.path.join(ROOT, "include", "heligym_amd.h")


@pytest.fixture(scope="module")
def lib():
    return _abi.load_library()


def header_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(hg_[a-z_0-9]+)\s*\(", txt)))


def test_exports_every_declared_symbol(lib):
    syms = header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), s
    assert sorted(_abi.EXPORTED_SYMBOLS) == syms


def test_struct_layout_matches_header(lib):
    # hg_default_config writes the AW109 defaults through the C struct: compare with our yaml
    c = _abi.hg_config()
    lib.hg_default_config(ctypes.byref(c))
    y, _ = config.make_config()
    for name, _ in _abi.hg_airframe._fields_:
        assert getattr(c.af, name) == getattr(y.af, name), name
    assert c.dt == y.dt and c.max_time == y.max_time and c.task == y.task
    assert c.trim.gr_alt == 100.0 and c.target.sea_alt == 4000.0
    assert ctypes.sizeof(_abi.hg_trim_result) == 8 * (18 + 4 + 17 + 18 + 1) + 8


@pytest.mark.parametrize("i", range(16))
def test_host_trim_matches_reference(lib, terrain_u16, i):
    t = load_golden("trim.npz")
    cfg, _ = config.make_config(dt=float(t["dt"][i]), trim_cond=trim_dict(t["cond"][i]))
    hm = config.terrain_ft(terrain_u16, cfg.af.env_MAX_GR_ALT)
    w = (ctypes.c_double * 3)(*t["wind_ned"][i])
    r = _abi.hg_trim_result()
    _abi.check(lib.hg_trim(ctypes.byref(cfg), hm.ctypes.data, 1024, 1024, w, ctypes.byref(r)), lib)
    for name in ("state", "action", "obs"):
        got, ref = np.array(getattr(r, name)), t[name][i]
        assert np.all(np.abs(got - ref) <= 1e-4 * (np.abs(ref) + 1)), (name, got - ref)
    assert r.residual <= 1e-4 and not r.failed


def test_host_trim_second_episode_wind(lib, terrain_u16):
    t = load_golden("trim.npz")
    cfg, _ = config.make_config(dt=0.02)
    hm = config.terrain_ft(terrain_u16, cfg.af.env_MAX_GR_ALT)
    w = (ctypes.c_double * 3)(*t["reset2_wind_ned"])
    r = _abi.hg_trim_result()
    _abi.check(lib.hg_trim(ctypes.byref(cfg), hm.ctypes.data, 1024, 1024, w, ctypes.byref(r)), lib)
    assert np.all(np.abs(np.array(r.state) - t["reset2_state"]) <= 1e-4 * (np.abs(t["reset2_state"]) + 1))


def test_errors_are_codes_not_crashes(lib, terrain_u16):
    cfg, _ = config.make_config()
    hm = config.terrain_ft(terrain_u16, cfg.af.env_MAX_GR_ALT)
    h = ctypes.c_void_p()
    bad = _abi.hg_config.from_buffer_copy(cfg)
    bad.dt = -1.0
    assert lib.hg_create(ctypes.byref(bad), hm.ctypes.data, 1024, 1024, 16, ctypes.byref(h)) == -1
    assert b"dt" in lib.hg_last_error()
    assert lib.hg_create(ctypes.byref(cfg), hm.ctypes.data, 1024, 1024, 0, ctypes.byref(h)) == -1
    assert lib.hg_create(ctypes.byref(cfg), hm.ctypes.data, 1024, 512, 16, ctypes.byref(h)) == -1
    bad = _abi.hg_config.from_buffer_copy(cfg)
    bad.task = 9
    assert lib.hg_create(ctypes.byref(bad), hm.ctypes.data, 1024, 1024, 16, ctypes.byref(h)) == -1
    assert lib.hg_step(None, None, None, None, None, None, None, None, None, None, None, None) == -1
    assert lib.hg_reset(None, None, None, None) == -1
    assert lib.hg_num_envs(None) == -1
    # impossible trim condition: the reference asserts after 5 s (helicopter_dynamics.py:543-544)
    wild = _abi.hg_config.from_buffer_copy(cfg)
    wild.trim.ned_vel[0] = 5000.0
    r = _abi.hg_trim_result()
    rc = lib.hg_trim(ctypes.byref(wild), hm.ctypes.data, 1024, 1024, None, ctypes.byref(r))
    assert rc in (0, -3)


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(_abi.HeliGymError):
        _abi.load_library(str(tmp_path / "nope.so"))


def test_vector_env_refuses_without_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("device present")
    from heligym_amd import HeliVecEnv
    with pytest.raises(_abi.HeliGymError):
        HeliVecEnv(8)


@pytest.mark.parametrize("i", range(11))
def test_host_trim_f8_resets(lib, terrain_u16, i):
    """Second-episode resets (F8): the reference trims against the last step's wind; the host trim
    given that wind reproduces its reset state, action and observation."""
    dt, cond, wind, state, action, obs = golden_cases.f8_resets()[i]
    cfg, _ = config.make_config(dt=dt, trim_cond=trim_dict(cond) if cond is not None else None)
    hm = config.terrain_ft(terrain_u16, cfg.af.env_MAX_GR_ALT)
    r = _abi.hg_trim_result()
    _abi.check(lib.hg_trim(ctypes.byref(cfg), hm.ctypes.data, 1024, 1024, (ctypes.c_double * 3)(*wind),
                           ctypes.byref(r)), lib)
    for name, ref in (("state", state), ("action", action), ("obs", obs)):
        got = np.array(getattr(r, name))
        assert np.all(np.abs(got - ref) <= 1e-4 * (np.abs(ref) + 1)), (name, got - ref)


def test_reset_mode_is_validated(lib, terrain_u16):
    cfg, _ = config.make_config(reset_mode="retrim")
    assert cfg.reset_mode == _abi.HG_RESET_RETRIM
    with pytest.raises(ValueError):
        config.make_config(reset_mode="sometimes")
    bad = _abi.hg_config.from_buffer_copy(cfg)
    bad.reset_mode = 7
    hm = config.terrain_ft(terrain_u16, cfg.af.env_MAX_GR_ALT)
    h = ctypes.c_void_p()
    assert lib.hg_create(ctypes.byref(bad), hm.ctypes.data, 1024, 1024, 16, ctypes.byref(h)) == -1
    assert b"reset_mode" in lib.hg_last_error()


def _build_c_example(tmp_path):
    exe = tmp_path / "c_abi_step"
    cmd = ["gcc", "-O2", "-std=c11", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), "-I",
           "/opt/rocm/include", "-D__HIP_PLATFORM_AMD__", os.path.join(ROOT, "examples", "c_abi_step.c"),
           "-L", os.path.dirname(_abi.LIB_PATH), "-lheligym_amd", "-L", "/opt/rocm/lib", "-lamdhip64",
           "-o", str(exe)]
    import subprocess
    subprocess.check_call(cmd)
    return exe


@pytest.mark.skipif(not os.path.exists("/opt/rocm/include/hip/hip_runtime_api.h"), reason="no ROCm headers")
def test_plain_c_host_compiles_against_header(tmp_path):
    """The C-ABI is usable from plain C (gcc, no torch): examples/c_abi_step.c builds and links."""
    assert _build_c_example(tmp_path).exists()


@pytest.mark.gpu
def test_plain_c_host_runs(tmp_path):
    import subprocess
    exe = _build_c_example(tmp_path)
    env = dict(os.environ, LD_LIBRARY_PATH=os.path.dirname(_abi.LIB_PATH) + ":/opt/rocm/lib")
    out = subprocess.run([str(exe), "4096", "200"], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    f = dict(zip(out.stdout.split()[0::2], out.stdout.split()[1::2]))
    assert int(f["envs"]) == 4096 and int(f["resets"]) == 0
    assert abs(float(f["mean_ground_alt_ft"]) - (100 + 38.5 / 12)) < 5.0    # trimmed hover holds altitude
    assert 400 < float(f["mean_power_hp"]) < 800


def test_baked_constants_current(lib):
    """csrc/baked_aw109.inc (the default airframe's constants compiled into the specialised step
    kernel) is what derive<float>() gives today: regenerate with scripts/gen_baked_constants.py."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen_baked", os.path.join(ROOT, "scripts", "gen_baked_constants.py"))
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    assert open(gen.OUT).read() == gen.current_text()


@pytest.mark.parametrize("kw,baked", [(dict(), True), (dict(dt=0.02), True), (dict(task="forward_flight"), True),
                                      (dict(max_time=20.0, target={"sea_alt": 3000.0}), True),
                                      (dict(turbulence_level=5), False), (dict(variant="heavy"), False),
                                      (dict(variant="turb7_wind"), False)])
def test_specialised_kernel_selection(lib, kw, baked):
    """The specialised kernel is selected for the default airframe whatever the dt, task, target or
    time limit (those stay runtime values), and for nothing else."""
    if "variant" in kw:
        cfg, _ = config.make_config(heli_name=golden_cases.load_variant(kw["variant"])[1])
    else:
        cfg, _ = config.make_config(**kw)
    assert lib.hg_config_is_baked(ctypes.byref(cfg), 1024, 1024) == (1 if baked else 0)
    assert lib.hg_config_is_baked(ctypes.byref(cfg), 512, 512) == 0   # other terrain size


def test_rtc_flags_match_library_build():
    """heligym_amd._rtc compiles the step code with the flags the library's step translation unit
    gets (__graft_entry__.HIP_FLAGS and heligym_amd.hip's own), so its kernels round alike."""
    import __graft_entry__ as ge
    from heligym_amd import _rtc
    step_flags = dict(ge.SOURCES)[ge.SRC]
    assert _rtc.FLAGS == ge.HIP_FLAGS + step_flags


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="no hipcc")
def test_rtc_code_object_builds(lib, tmp_path, monkeypatch):
    """The run-time specialisation pipeline on the CPU side: another airframe's constant image,
    compiled into a gfx950 code object holding the six per-step kernels, cached by key."""
    from heligym_amd import _rtc
    monkeypatch.setenv("HELIGYM_AMD_CACHE", str(tmp_path))
    cfg, _ = config.make_config(heli_name=golden_cases.load_variant("heavy")[1])
    assert lib.hg_config_is_baked(ctypes.byref(cfg), 1024, 1024) == 0
    path, img = _rtc.build(lib, cfg, 1024, 1024, cfg.task)
    assert os.path.getsize(path) > 10000 and len(img) % 4 == 0
    blob = open(path, "rb").read()
    for name in ("hg_rtc_step_nt", "hg_rtc_step_nt_feat", "hg_rtc_step_nts", "hg_rtc_step_nts_feat",
                 "hg_rtc_step_bulk", "hg_rtc_step_bulk_feat", "hg_rtc_image", "hg_rtc_task"):
        assert name.encode() in blob
    # the build's constant file is process-private and removed afterwards
    assert not [f for f in os.listdir(tmp_path) if f.endswith((".inc", ".tmp"))]
    t = os.path.getmtime(path)
    assert _rtc.build(lib, cfg, 1024, 1024, cfg.task)[0] == path and os.path.getmtime(path) == t   # cached
    # the image is the baked fields of this airframe, not the default one's
    cfg0, _ = config.make_config()
    assert _rtc.image(lib, cfg0, 1024, 1024) != img
