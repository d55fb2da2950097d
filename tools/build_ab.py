"""Build an A/B variant of libsplink_hip.so: one translation unit recompiled with extra defines, linked
with the in-tree objects of the others (python -m splink_amd.build first).

    python tools/build_ab.py OUT.so SOURCE.hip -DNAME=VALUE ...
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from splink_amd import build as B  # noqa: E402

out, src, defs = sys.argv[1], sys.argv[2], sys.argv[3:]
B.build()
obj = os.path.join(B.OBJ, "ab_" + os.path.splitext(src)[0] + ".o")
subprocess.run([B._hipcc(), *B.FLAGS, *defs, "-c", "-o", obj, os.path.join(B.HERE, "csrc", src)], check=True)
objs = [obj if os.path.basename(B._obj(s)) == os.path.splitext(src)[0] + ".o" else B._obj(s) for s in B.SOURCES]
subprocess.run([B._hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out, *objs], check=True)
print(out)
