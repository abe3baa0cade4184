"""Build the in-tree native library ``libdrynx_native.so`` for gfx950.

Each ``csrc/kernels/*.hip`` translation unit is compiled by ``hipcc
--offload-arch=gfx950`` in parallel (one process per TU, bounded by a
timeout) and linked into one shared object that lives next to this file, so
it travels with the repo snapshot to the GPU box.  The library contains both
the gfx950 device code and the host (CPU) path of every batched op.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
CSRC = os.path.join(ROOT, "csrc")
LIB = os.path.join(HERE, "libdrynx_native.so")
OBJDIR = os.path.join(ROOT, "build", "native")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0] or "gfx950"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result"]


def _sources():
    kdir = os.path.join(CSRC, "kernels")
    return sorted(os.path.join(kdir, f) for f in os.listdir(kdir) if f.endswith(".hip"))


def _headers():
    out = []
    for d in ("bn254", "kernels"):
        p = os.path.join(CSRC, d)
        out += sorted(os.path.join(p, f) for f in os.listdir(p) if f.endswith(".h"))
    return out


def _digest(paths):
    """Content digest of sources/headers, keyed by repo-relative paths (the
    tree is copied to other locations, e.g. a GPU box, and must not rebuild)."""
    h = hashlib.sha256()
    for p in paths:
        with open(p, "rb") as f:
            h.update(os.path.relpath(p, ROOT).encode() + f.read())
    h.update(" ".join(FLAGS).encode())
    return h.hexdigest()


# host-side sanitizers for the CPU path of every op: -fsanitize
# goes to the host compilation only (-Xarch_host), never into gfx950 code
SAN_FLAGS = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
             "-Xarch_host", "-fno-omit-frame-pointer", "-Xarch_host", "-fno-sanitize-recover=undefined"]
SAN_LIB = os.path.join(ROOT, "build", "libdrynx_native_asan.so")


def _closure(src: str) -> list:
    """The source and every header it reaches through quoted #includes
    (resolved next to the including file, then under csrc/)."""
    seen, todo = [], [os.path.abspath(src)]
    while todo:
        f = todo.pop()
        if f in seen or not os.path.exists(f):
            continue
        seen.append(f)
        with open(f) as fh:
            for line in fh:
                t = line.strip()
                if t.startswith("#include") and '"' in t:
                    inc = t.split('"')[1]
                    for d in (os.path.dirname(f), CSRC):
                        cand = os.path.abspath(os.path.join(d, inc))
                        if os.path.exists(cand):
                            todo.append(cand)
                            break
    return sorted(seen)


def _compile(src, hdr_digest, sanitize=False):
    """``hdr_digest`` is unused for the object key: an object depends on its
    own include closure only, so a header edit recompiles the translation
    units that include it (the library stamp still covers every file)."""
    objdir = OBJDIR + ("_asan" if sanitize else "")
    os.makedirs(objdir, exist_ok=True)
    key = _digest(_closure(src)) + ("san" if sanitize else "")
    obj = os.path.join(objdir, os.path.basename(src) + ".o")
    stamp = obj + ".stamp"
    if os.path.exists(obj) and os.path.exists(stamp) and open(stamp).read() == key:
        return obj
    cmd = [HIPCC, *FLAGS, *(SAN_FLAGS if sanitize else []), "-I", CSRC, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=1800)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-4000:]}")
    with open(stamp, "w") as f:
        f.write(key)
    return obj


def build(force: bool = False, verbose: bool = True) -> str:
    gen = os.path.join(ROOT, "tools", "gen_constants.py")
    subprocess.run([sys.executable, gen], check=True)
    srcs = _sources()
    hdr_digest = _digest(_headers())
    lib_stamp = LIB + ".stamp"
    all_key = _digest(srcs) + hdr_digest
    if not force and os.path.exists(LIB) and os.path.exists(lib_stamp) and open(lib_stamp).read() == all_key:
        return LIB
    workers = min(len(srcs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16)
    with cf.ThreadPoolExecutor(max_workers=workers) as ex:
        objs = list(ex.map(lambda s: _compile(s, hdr_digest), srcs))
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs, "-lpthread"]
    subprocess.run(cmd, check=True, timeout=600)
    with open(lib_stamp, "w") as f:
        f.write(all_key)
    if verbose:
        print(f"[drynx_amd] built {LIB}")
    return LIB


def build_sanitized(verbose: bool = True) -> str:
    """build/libdrynx_native_asan.so: the same library with ASan + UBSan on the
    host path.  Run the CPU suite against it with
      LD_PRELOAD=$(hipcc -print-file-name=libclang_rt.asan-x86_64.so) \
      ASAN_OPTIONS=detect_leaks=0 DRYNX_NATIVE_LIB=build/libdrynx_native_asan.so pytest -m "not gpu"
    (``make sanitize``)."""
    gen = os.path.join(ROOT, "tools", "gen_constants.py")
    subprocess.run([sys.executable, gen], check=True)
    srcs = _sources()
    hdr_digest = _digest(_headers())
    workers = min(len(srcs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16)
    with cf.ThreadPoolExecutor(max_workers=workers) as ex:
        objs = list(ex.map(lambda s: _compile(s, hdr_digest, True), srcs))
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-shared-libasan", "-fsanitize=address,undefined",
           "-o", SAN_LIB, *objs, "-lpthread"]
    subprocess.run(cmd, check=True, timeout=600)
    if verbose:
        print(f"[drynx_amd] built {SAN_LIB}")
    return SAN_LIB


if __name__ == "__main__":
    if "--sanitize" in sys.argv:
        build_sanitized()
    else:
        build(force="--force" in sys.argv)
