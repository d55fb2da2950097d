"""Build libsplink_hip.so from the C++/HIP sources of a git revision, for A/B runs against the working
tree (the Python side stays the working tree's, so the revision must export the same entry points).

    python tools/build_ab_rev.py REV OUT.so [-DNAME=VALUE ...]   (defines apply to every source)
"""
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from splink_amd import build as B  # noqa: E402

rev, out, defs = sys.argv[1], sys.argv[2], sys.argv[3:]
tmp = "/tmp/ab_rev_" + rev.replace("/", "_")
shutil.rmtree(tmp, ignore_errors=True)
os.makedirs(tmp)
arch = subprocess.run(["git", "-C", ROOT, "archive", rev, "splink_amd/csrc", "include"], check=True,
                      capture_output=True).stdout
subprocess.run(["tar", "-x", "-C", tmp], input=arch, check=True)
csrc = os.path.join(tmp, "splink_amd", "csrc")


def comp(src):
    o = os.path.join(tmp, os.path.splitext(src)[0] + ".o")
    subprocess.run([B._hipcc(), *B.FLAGS, *defs, "-c", "-o", o, os.path.join(csrc, src)], check=True)
    return o


with cf.ThreadPoolExecutor(8) as ex:
    objs = list(ex.map(comp, B.SOURCES))
subprocess.run([B._hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out, *objs], check=True)
print(out)
