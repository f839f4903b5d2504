"""Build libsddm_hip.so in-tree with hipcc for gfx950 (no JIT cache, no torch extension).

    python -m sddm_hip.build            # from speech-denoising-diffusion-model-2_amd/
    python speech-denoising-diffusion-model-2_amd/sddm_hip/build.py

Objects are rebuilt when a source or header is newer; the .so lands next to this file so it
travels to the GPU box with the repository snapshot.
"""
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(os.path.dirname(PKG), "include")
# SDDM_BUILD_VARIANT=stamps builds a phase-timestamp profiling variant into tools/_stamps/
VARIANT = os.environ.get("SDDM_BUILD_VARIANT", "")
if VARIANT:
    _OUT = os.path.join(os.path.dirname(PKG), "tools", "_" + VARIANT)
    BUILD = os.path.join(_OUT, "_build")
    LIB = os.path.join(_OUT, "libsddm_hip.so")
else:
    BUILD = os.path.join(HERE, "_build")
    LIB = os.path.join(HERE, "libsddm_hip.so")
SOURCES = ["kernels.hip", "conv_strip.hip", "conv_strip_bf16.hip", "conv_strip_f16.hip", "conv_strip_f32.hip", "conv_deep.hip", "conv_tile.hip", "conv_chain.hip", "diffwave.hip", "wavegrad.hip", "q_sample.hip", "stft.hip", "sddm_runtime.cpp",
           "schedule.cpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("SDDM_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", CSRC, "-I", INCLUDE,
         "-Wno-unused-result"] + (["-DSDDM_STAMPS"] if VARIANT.startswith("stamps") else [])
# experiment variants: extra -D flags for a variant build (e.g. SDDM_EXTRA_DEFS="-DFOO -DBAR")
if VARIANT:
    FLAGS += os.environ.get("SDDM_EXTRA_DEFS", "").split()


def _deps(path, seen=None):
    """Headers a source includes (transitively), found in csrc/ or include/."""
    import re
    seen = set() if seen is None else seen
    with open(path) as f:
        for name in re.findall(r'^\s*#\s*include\s+"([^"]+)"', f.read(), re.M):
            for d in (CSRC, INCLUDE):
                h = os.path.join(d, name)
                if os.path.exists(h) and h not in seen:
                    seen.add(h)
                    _deps(h, seen)
    return sorted(seen)


def _stale(target, inputs):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(i) > t for i in inputs)


def _compile(src):
    obj = os.path.join(BUILD, os.path.basename(src) + ".o")
    if _stale(obj, [os.path.join(CSRC, src)] + _deps(os.path.join(CSRC, src))):
        cmd = [HIPCC] + FLAGS + ["-c", os.path.join(CSRC, src), "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(verbose=False):
    os.makedirs(BUILD, exist_ok=True)
    with cf.ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        objs = list(ex.map(_compile, SOURCES))
    if _stale(LIB, objs):
        cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-Wl,--no-undefined", "-o", LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    if verbose:
        print("built", LIB)
    return LIB


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
