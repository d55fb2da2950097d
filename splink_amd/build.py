"""Build libsplink_hip.so in-tree for gfx950 (hipcc, no CMake).

Each translation unit compiles to its own object in parallel (build/), then one link.

    python -m splink_amd.build [--force]
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
SOURCES = ["spk_ctx.hip", "spk_block.hip", "spk_gamma.hip", "spk_filter.hip", "spk_em.hip", "spk_tf.hip", "spk_ingest.hip"]
HEADERS = ["spk_internal.h", "spk_strsim.h", "spk_gamma.h"]
OUT = os.path.join(HERE, "libsplink_hip.so")
OBJ = os.path.join(HERE, "build")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
         # the Jaro-Winkler / E-step arithmetic must round exactly like the JVM: no FMA contraction
         "-ffp-contract=off", "-fno-fast-math"]


def _hipcc():
    return os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _headers():
    return [os.path.join(HERE, "csrc", h) for h in HEADERS] + [os.path.join(HERE, "..", "include", "splink_hip.h")]


def _obj(src):
    return os.path.join(OBJ, os.path.splitext(src)[0] + ".o")


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src, force):
    obj = _obj(src)
    path = os.path.join(HERE, "csrc", src)
    if force or _stale(obj, [path] + _headers()):
        subprocess.run([_hipcc(), *FLAGS, "-c", "-o", obj + ".tmp", path], check=True)
        os.replace(obj + ".tmp", obj)
    return obj


def build(force: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    srcs = [s for s in SOURCES if os.path.exists(os.path.join(HERE, "csrc", s))]
    with ThreadPoolExecutor(max_workers=min(len(srcs), int(os.environ.get("MAX_JOBS", "8")))) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), srcs))
    if force or _stale(OUT, objs):
        subprocess.run([_hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", OUT + ".tmp", *objs], check=True)
        os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
