"""Build an A/B variant of libsplink_hip.so: one translation unit recompiled with extra defines, linked
with the in-tree objects of the others (python -m splink_amd.build first).

    python tools/build_ab.py OUT.so SOURCE.hip[,SOURCE2.hip...] -DNAME=VALUE ...

(the defines apply to every listed source)
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from splink_amd import build as B  # noqa: E402

out, srcs, defs = sys.argv[1], sys.argv[2].split(","), sys.argv[3:]
B.build()
ab = {}
for src in srcs:
    obj = os.path.join(B.OBJ, "ab_" + os.path.splitext(src)[0] + ".o")
    subprocess.run([B._hipcc(), *B.FLAGS, *defs, "-c", "-o", obj, os.path.join(B.HERE, "csrc", src)], check=True)
    ab[src] = obj
objs = [ab.get(s, B._obj(s)) for s in B.SOURCES]
subprocess.run([B._hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out, *objs], check=True)
print(out)
