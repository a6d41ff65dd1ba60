"""Static instruction mix of the step kernels in a gfx950 assembly listing (hipcc -S --cuda-device-only).

usage: python scripts/isa_stats.py file.s [name-filter]
Prints, per kernel: instruction count by class, SGPR spill traffic (v_writelane / v_readlane),
packed-fp32 ops, transcendental ops, and the register counts from the metadata.
"""
import collections
import re
import sys

TRANS = ("v_exp_f32", "v_log_f32", "v_rcp_f32", "v_sqrt_f32", "v_rsq_f32", "v_sin_f32", "v_cos_f32")


def kernels(text):
    for m in re.finditer(r"^(_Z\S*step_kernel\S*):\s*;.*$", text, re.M):
        name = m.group(1)
        end = text.index(".Lfunc_end", m.end())
        yield name, text[m.end():end]


def meta(text, name):
    i = text.find(".name:           " + name)
    blk = text[max(0, i - 2500):i]
    out = {}
    for key in ("sgpr_count", "sgpr_spill_count", "vgpr_count", "vgpr_spill_count"):
        ms = re.findall(r"\." + key + r":\s+(\d+)", blk)
        out[key] = int(ms[-1]) if ms else None
    return out


def main():
    text = open(sys.argv[1]).read()
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    for name, body in kernels(text):
        if filt not in name:
            continue
        ins = []
        for line in body.split("\n"):
            t = line.strip()
            if not t or t.startswith((".", ";")) or t.endswith(":"):
                continue
            ins.append(t.split()[0])
        c = collections.Counter(ins)
        cls = collections.Counter()
        for k, n in c.items():
            if k.startswith(("global_", "buffer_", "flat_")):
                cls["vmem"] += n
            elif k.startswith("ds_"):
                cls["lds"] += n
            elif k.startswith("s_load") or k.startswith("s_buffer_load"):
                cls["smem"] += n
            elif k.startswith("s_"):
                cls["salu"] += n
            elif k.startswith("v_"):
                cls["valu"] += n
        print(name)
        print("  ", dict(cls), "total", len(ins), meta(text, name))
        print("   writelane", c["v_writelane_b32"], "readlane", c["v_readlane_b32"],
              "pk", sum(n for k, n in c.items() if k.startswith("v_pk_")),
              "trans", sum(c[t] for t in TRANS), "cndmask", c["v_cndmask_b32"], "mov", c["v_mov_b32"],
              "waitcnt", c["s_waitcnt"])
        if "-v" in sys.argv:
            for k, n in c.most_common(40):
                print("     ", k, n)


if __name__ == "__main__":
    main()
