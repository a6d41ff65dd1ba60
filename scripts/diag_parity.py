"""Diagnostics: per-scenario, per-column max error of the HIP step vs the reference goldens and
vs the oracle (single steps from the reference's own pre-step states)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "heli-gym_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np, torch
import golden_cases as gc
from heligym_amd import HeliVecEnv, config
from oracle.oracle import Oracle
np.set_printoptions(precision=2, linewidth=250)
for tag in ["0.02", "0.01"]:
    b = gc.single_step_batch(gc.load(tag), "hover")
    env = HeliVecEnv(len(b["state"]), task="hover", dt=b["dt"], autoreset=False)
    env.set_state(b["state"].astype(np.float32), b["counters"].astype(np.int32))
    obs, rew, term, trunc, info = env.step(torch.as_tensor(b["actions"].astype(np.float32), device=env.device),
                                           eta=torch.as_tensor(b["eta"].astype(np.float32), device=env.device))
    st, _ = env.get_state()
    obs = obs.cpu().numpy().astype(np.float64); st = st.cpu().numpy().astype(np.float64)
    cfg, doc = config.make_config(task="hover", dt=b["dt"])
    orc = Oracle(cfg, config.load_terrain(doc))
    oo = np.zeros_like(obs); os_ = np.zeros((len(obs), 18))
    for i in range(len(obs)):
        s = b["state"][i].astype(np.float32).astype(np.float64)
        prev = np.zeros(17); prev[4:7], prev[16] = s[23:26], s[26]
        e = orc.env_from(s[:18], s[18:23], prev, np.zeros(18))
        o = orc.step(e, b["actions"][i].astype(np.float32), b["eta"][i].astype(np.float32))
        oo[i] = o.obs; os_[i] = e.heli
    for sc in np.unique(b["scenario"]):
        m = b["scenario"] == sc
        eg = gc.step_errors(obs[m], b["obs"][m], gc.OBS_ANGLE_COLS) / (2e-4 + 2e-5 * np.abs(b["obs"][m]))
        eo = gc.step_errors(obs[m], oo[m], gc.OBS_ANGLE_COLS) / (2e-4 + 2e-5 * np.abs(oo[m]))
        og = gc.step_errors(oo[m], b["obs"][m], gc.OBS_ANGLE_COLS) / (2e-4 + 2e-5 * np.abs(b["obs"][m]))
        sg = gc.step_errors(st[m, :18], b["heli"][m], gc.HELI_ANGLE_COLS) / (2e-4 + 2e-5 * np.abs(b["heli"][m]))
        print(tag, sc, "kern/gold obs", eg.max(0), "\n   kern/orc obs", eo.max(0), "\n   orc/gold obs", og.max(0), "\n   kern/gold state", sg.max(0))
        worst = np.argmax(eg.max(1)); idx = np.nonzero(m)[0][worst]
        print("   worst t", b["t"][idx], "kern", obs[idx], "\n   gold", b["obs"][idx], "\n   orc ", oo[idx])
