"""Build libsplink_hip.so from a copy of the working tree's C++/HIP sources with literal text edits
applied (A/B of a change that is not behind a build option).

    python tools/build_ab_tree.py OUT.so FILE 'OLD' 'NEW' [FILE 'OLD' 'NEW' ...]
"""
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from splink_amd import build as B  # noqa: E402

out, edits = sys.argv[1], sys.argv[2:]
tmp = "/tmp/ab_tree_" + os.path.basename(out)
shutil.rmtree(tmp, ignore_errors=True)
shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
shutil.copytree(os.path.join(ROOT, "splink_amd", "csrc"), os.path.join(tmp, "splink_amd", "csrc"))
csrc = os.path.join(tmp, "splink_amd", "csrc")
for i in range(0, len(edits), 3):
    f, old, new = edits[i:i + 3]
    path = os.path.join(csrc, f)
    s = open(path).read()
    assert old in s, (f, old)
    open(path, "w").write(s.replace(old, new))


def comp(src):
    o = os.path.join(tmp, os.path.splitext(src)[0] + ".o")
    subprocess.run([B._hipcc(), *B.FLAGS, "-c", "-o", o, os.path.join(csrc, src)], check=True)
    return o


with cf.ThreadPoolExecutor(8) as ex:
    objs = list(ex.map(comp, B.SOURCES))
subprocess.run([B._hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out, *objs], check=True)
print(out)
