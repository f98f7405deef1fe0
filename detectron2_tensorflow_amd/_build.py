"""In-tree build of libd2mi_hip.so (gfx950) with plain hipcc.

Every csrc/*.hip becomes one object (compiled in parallel, skipped when
up to date); the objects link into detectron2_tensorflow_amd/lib/libd2mi_hip.so,
which the ctypes loader in _C.py opens.  -ffp-contract=off keeps the float
expressions that restate the TF 1.x CPU kernels un-fused (bit-exact NMS
decisions, ROIAlign sample positions).
"""
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
OBJDIR = os.path.join(LIBDIR, "obj")
LIB = os.path.join(LIBDIR, "libd2mi_hip.so")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")

ARCH = os.environ.get("D2MI_OFFLOAD_ARCH", "gfx950")
CFLAGS = [
    "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", f"--offload-arch={ARCH}",
    "-Wall", "-Wno-unused-function", "-Wno-unused-variable", f"-I{INCLUDE}",
]


def _sources():
    names = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".h")))
    return [os.path.join(CSRC, f) for f in names] + [os.path.join(INCLUDE, "d2mi.h")]


def source_hash():
    """sha256 (first 16 hex digits) over the names and contents of every
    source the library is built from; compiled into d2mi_source_hash() and
    checked by _C.load (a prebuilt library from other sources is refused)."""
    h = hashlib.sha256()
    for p in _sources():
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def _hipcc():
    h = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(h):
        raise RuntimeError("hipcc not found: the HIP toolchain is required to build libd2mi_hip.so")
    return h


def _deps(src):
    heads = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    heads.append(os.path.join(INCLUDE, "d2mi.h"))
    return [src] + heads


def _stale(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src, obj, verbose, extra=()):
    cmd = [_hipcc(), *CFLAGS, *extra, "-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {os.path.basename(src)}:\n{r.stderr}")
    return obj


def build(verbose=False, jobs=None):
    os.makedirs(OBJDIR, exist_ok=True)
    srcs = sorted(f for f in os.listdir(CSRC) if f.endswith(".hip"))
    objs, todo = [], []
    hsh = source_hash()
    stamp = os.path.join(OBJDIR, "source_hash.txt")
    old = open(stamp).read().strip() if os.path.exists(stamp) else None
    for f in srcs:
        src = os.path.join(CSRC, f)
        obj = os.path.join(OBJDIR, f[:-4] + ".o")
        objs.append(obj)
        # errors.hip carries the hash of ALL sources: rebuilt whenever it changes
        extra = (f'-DD2MI_SOURCE_HASH="{hsh}"',) if f == "errors.hip" else ()
        if _stale(obj, _deps(src)) or (extra and old != hsh):
            todo.append((src, obj, extra))
    jobs = jobs or min(8, max(1, len(todo)))
    if todo:
        with cf.ThreadPoolExecutor(jobs) as ex:
            list(ex.map(lambda a: _compile(a[0], a[1], verbose, a[2]), todo))
    with open(stamp, "w") as f:
        f.write(hsh + "\n")
    if todo or _stale(LIB, objs):
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", LIB]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link of libd2mi_hip.so failed:\n{r.stderr}")
    return LIB


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
