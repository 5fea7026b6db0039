"""Build the gfx950 C-ABI library `libasrx.so` in-tree with hipcc (no torch extension machinery).

    python -m asrx._build            (from asr-transformer_amd/)
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
REPO = os.path.dirname(ROOT)
CSRC = os.path.join(ROOT, "csrc")
OUTDIR = os.path.join(PKG, "lib")
LIB = os.path.join(OUTDIR, "libasrx.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("ASRX_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=fast",
         "-I" + os.path.join(REPO, "include"), "-Wno-unused-result"] + os.environ.get("ASRX_CFLAGS", "").split()
# (ASRX_CFLAGS: diagnostic builds only, e.g. -DASRX_ATTN_STAMPS for tools/attn_bench.py --dbg; the objects are not
#  tracked by flags, so build with force=True when switching)


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def _newer(target, deps):
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(d) <= t for d in deps)


def build(force=False, verbose=False, jobs=8):
    os.makedirs(OUTDIR, exist_ok=True)
    srcs = sources()
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    headers.append(os.path.join(REPO, "include", "asrx.h"))
    objs = []

    def compile_one(src):
        obj = os.path.join(OUTDIR, os.path.basename(src).replace(".hip", ".o"))
        if force or not _newer(obj, [src] + headers):
            cmd = [HIPCC] + FLAGS + ["-c", src, "-o", obj]
            if verbose:
                print(" ".join(cmd), flush=True)
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
        return obj

    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(compile_one, srcs))
    if force or not _newer(LIB, objs):
        cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", LIB] + objs
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
