"""In-tree build of libd2mi_hip.so (gfx950) with plain hipcc.

Every csrc/*.hip becomes one object (compiled in parallel, skipped when
up to date); the objects link into detectron2_tensorflow_amd/lib/libd2mi_hip.so,
which the ctypes loader in _C.py opens.  -ffp-contract=off keeps the float
expressions that restate the TF 1.x CPU kernels un-fused (bit-exact NMS
decisions, ROIAlign sample positions).
"""
import concurrent.futures as cf
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


def _compile(src, obj, verbose):
    cmd = [_hipcc(), *CFLAGS, "-c", src, "-o", obj]
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
    for f in srcs:
        src = os.path.join(CSRC, f)
        obj = os.path.join(OBJDIR, f[:-4] + ".o")
        objs.append(obj)
        if _stale(obj, _deps(src)):
            todo.append((src, obj))
    jobs = jobs or min(8, max(1, len(todo)))
    if todo:
        with cf.ThreadPoolExecutor(jobs) as ex:
            list(ex.map(lambda a: _compile(a[0], a[1], verbose), todo))
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
