"""Run-time specialisation of the step kernel for airframes other than the compiled-in default.

The library's step kernel has the default AW109 airframe's model constants compiled in as
instruction literals (csrc/baked.h); any other airframe (a YAML document in the reference's schema,
another mean wind or turbulence level, another terrain size) runs the generic kernel, which loads
~120 constants per RK stage.  `build()` compiles csrc/step_rtc.hip -- the same step code, nothing
else of the library -- with this env's constant image into a gfx950 code object (hipcc --genco,
about 4 s), cached under $HELIGYM_AMD_CACHE or ~/.cache/heligym_amd by a hash of the image, the task,
the flags and the sources; `hg_load_specialized` then steps the env with it.  The specialised
kernels' results are bitwise those of the generic kernel (tests/test_gpu_variants.py).
"""
import ctypes
import hashlib
import os
import subprocess
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(_HERE), "csrc")
INCLUDE = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# the step translation unit's flags: __graft_entry__.HIP_FLAGS plus heligym_amd.hip's own
# (tests/test_abi_host.py keeps the two lists equal)
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
         "-fno-hip-fp32-correctly-rounded-divide-sqrt", "-fgpu-flush-denormals-to-zero", "-fno-slp-vectorize",
         "-ffp-contract=on", "-Wno-unused-result",
         "-mllvm", "-amdgpu-kernarg-preload-count=6", "-mllvm", "-disable-vector-combine",
         "-mllvm", "-amdgpu-atomic-optimizer-strategy=None", "-mllvm", "-amdgpu-mfma-vgpr-form"]
PARAMS_BYTES_MAX = 4096


def cache_dir():
    d = os.environ.get("HELIGYM_AMD_CACHE") or os.path.join(os.path.expanduser("~"), ".cache", "heligym_amd")
    os.makedirs(d, exist_ok=True)
    return d


def image(lib, cfg, rows, cols):
    """The baked fields of derive<float>(cfg) as the bytes of Params<float> (hg_debug_params)."""
    for nbytes in range(4, PARAMS_BYTES_MAX, 4):
        buf = (ctypes.c_uint32 * (nbytes // 4))()
        if lib.hg_debug_params(ctypes.byref(cfg), rows, cols, 1, buf, nbytes) == 0:
            return bytes(buf)
    raise RuntimeError("hg_debug_params rejected every size")


def render(img):
    words = [int.from_bytes(img[k:k + 4], "little") for k in range(0, len(img), 4)]
    lines = ["// written by heligym_amd._rtc: an airframe's baked constants (csrc/baked.h), Params<float> dwords"]
    for k in range(0, len(words), 8):
        lines.append(" ".join(f"0x{w:08x}u," for w in words[k:k + 8]))
    return "\n".join(lines) + "\n"


def _sources_digest():
    h = hashlib.sha256()
    for d in (CSRC, INCLUDE):
        for f in sorted(os.listdir(d)):
            if f.endswith((".h", ".hip", ".inc")):
                h.update(f.encode())
                with open(os.path.join(d, f), "rb") as fh:
                    h.update(fh.read())
    return h.hexdigest()


def build(lib, cfg, rows, cols, task):
    """(code object path, constant image) for `cfg` and `task`, compiled on the first request."""
    img = image(lib, cfg, rows, cols)
    key = hashlib.sha256(img + f"|{task}|{' '.join(FLAGS)}|{_sources_digest()}".encode()).hexdigest()[:24]
    d = cache_dir()
    path = os.path.join(d, f"step_{key}.hsaco")
    if not os.path.exists(path):
        # every file of a build is this process's own (pid-unique names): concurrent builders of the
        # same key (the ranks of a sharded env) never read a constant file another one is writing
        tag = f"{os.getpid()}.{threading.get_ident()}"
        inc = os.path.join(d, f"step_{key}.{tag}.inc")
        with open(inc, "w") as f:
            f.write(render(img))
        tmp = f"{path}.{tag}.tmp"
        cmd = [HIPCC, *FLAGS, "--genco", f'-DHG_BAKED_INC="{inc}"', f"-DHG_RTC_TASK={int(task)}", "-o", tmp,
               os.path.join(CSRC, "step_rtc.hip")]
        try:
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"step specialisation failed ({' '.join(cmd)}):\n{r.stderr[-2000:]}")
            os.replace(tmp, path)   # atomic: concurrent builders of the same key agree
        finally:
            os.unlink(inc)
            if os.path.exists(tmp):   # a failed or interrupted build leaves no stray code object
                os.unlink(tmp)
    # (hg_load_specialized also checks the image the code object was built with against img)
    return path, img
