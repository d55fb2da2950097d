"""Build libsplink_hip.so in-tree for gfx950 (hipcc, no CMake).

    python -m splink_amd.build
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SOURCES = ["spk_ctx.hip", "spk_block.hip", "spk_gamma.hip", "spk_em.hip"]
HEADERS = ["spk_internal.h", "spk_strsim.h"]
OUT = os.path.join(HERE, "libsplink_hip.so")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
         # the Jaro-Winkler / E-step arithmetic must round exactly like the JVM: no FMA contraction
         "-ffp-contract=off", "-fno-fast-math"]


def _stale():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    srcs = [os.path.join(HERE, "csrc", s) for s in SOURCES + HEADERS]
    srcs.append(os.path.join(HERE, "..", "include", "splink_hip.h"))
    return any(os.path.getmtime(s) > t for s in srcs)


def build(force: bool = False) -> str:
    if not force and not _stale():
        return OUT
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, *FLAGS, "-o", OUT + ".tmp", *[os.path.join(HERE, "csrc", s) for s in SOURCES]]
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
