"""Static instruction counts between the PROBE markers of scripts/isa/stage_probe.hip's kernels
(analysis only).  usage: python scripts/isa/probe_count.py file.s [-v]"""
import collections
import re
import sys

text = open(sys.argv[1]).read()
for name in ("probe_new", "probe_old"):
    m = re.search(r"^(_Z\d+" + name + r"\S*):", text, re.M)
    body = text[m.end():text.index(".Lfunc_end", m.end())]
    seg = body[body.index("PROBE begin"):body.index("PROBE end")]
    ins = [l.strip().split()[0] for l in seg.split("\n")
           if l.strip() and not l.strip().startswith((";", ".")) and not l.strip().endswith(":")]
    c = collections.Counter(ins)
    v = sum(n for k, n in c.items() if k.startswith("v_"))
    s = sum(n for k, n in c.items() if k.startswith("s_"))
    tr = sum(c[k] for k in c if k.split("_e32")[0] in ("v_rcp_f32", "v_sqrt_f32", "v_exp_f32", "v_log_f32"))
    print(f"{name}: valu {v} salu {s} trans {tr} mov {c['v_mov_b32_e32'] + c['v_pk_mov_b32']} xor {c['v_xor_b32_e32']} "
          f"pk {sum(n for k, n in c.items() if k.startswith('v_pk'))} cndmask {c['v_cndmask_b32_e32'] + c['v_cndmask_b32_e64']}")
    if "-v" in sys.argv:
        for k, n in c.most_common(30):
            print("    ", k, n)
