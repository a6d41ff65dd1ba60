"""One line per bench JSON file: the headline and every secondary's ms/step and resets in window."""
import json
import sys

for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    t = d.get("timing", {})
    out = [f"{f}: K={d['steps']} head {d['ms_per_step'] * 1e3:.3f} us (resets/window {t.get('resets_in_window')}, "
           f"aged {t.get('aged_steps')}) frac {d['roofline']['frac']:.3f}"]
    for k in ("step_with_reset_info", "step_api_eager", "generic_kernel", "rollout", "retrim", "retrim_next_step", "out_of_cache"):
        v = d.get(k)
        if v:
            ms = v.get("ms_per_step") if v.get("ms_per_step") is not None else v.get("window_ms_per_step")
            out.append(f"  {k}: {ms * 1e3 if ms else float('nan'):.2f} us resets {v.get('resets_in_window')}")
    af = d.get("airframes")
    if af and "error" not in af:
        for k, v in af.items():
            if isinstance(v, dict):
                out.append(f"  airframe {k}: generic {v['generic_ms_per_step']*1e3:.2f} us, specialised "
                           f"{v['specialised_ms_per_step']*1e3:.2f} us ({v['specialised_over_default_airframe']:.3f} x default), "
                           f"build {v['specialise_s']:.1f} s")
    elif af:
        out.append(f"  airframes: {af}")
    print("\n".join(out))
