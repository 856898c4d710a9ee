"""Experiment library from a patched copy of retina_amd/csrc (diagnostics, not product code):

    python exp/variant.py exp/lib_NAME.so exp/patch_A.py [exp/patch_B.py ...]

Each patch script is run as `python patch.py SRC_DIR` and edits the copied sources in place,
so an experiment never changes the product sources (nor their build id)."""

import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from retina_amd import build as B  # noqa: E402

out, patches = sys.argv[1], sys.argv[2:]
# same depth as retina_amd/csrc so the sources' "../../include" resolves
top = "/tmp/gpuagg_src_" + os.path.basename(out).replace(".so", "")
src = top + "/pkg/csrc"
shutil.rmtree(top, ignore_errors=True)
os.makedirs(top)
os.symlink(os.path.join(ROOT, "include"), top + "/include")
shutil.copytree(B.CSRC, src, ignore=shutil.ignore_patterns("*.o", "*.so"))
for p in patches:
    subprocess.run([sys.executable, p, src], check=True)
print(B.build_variant([], out, src_dir=src))
