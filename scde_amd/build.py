"""Build ``libscde_hip.so`` in-tree for gfx950 (hipcc via make)."""
from __future__ import annotations

import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")


def build(jobs: int = 4, force: bool = False) -> str:
    if shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"):
        raise RuntimeError("hipcc not found: cannot build the gfx950 library")
    if force:
        subprocess.check_call(["make", "-s", "-C", CSRC, "clean"])
    subprocess.check_call(["make", "-s", "-j", str(jobs), "-C", CSRC])
    return os.path.join(HERE, "libscde_hip.so")


if __name__ == "__main__":
    print(build())
