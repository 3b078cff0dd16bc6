"""Build libpnol_amd.so (hipcc, --offload-arch=gfx950) through csrc/Makefile."""
from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")


def build(jobs: int = 8, verbose: bool = False) -> str:
    cmd = ["make", "-C", CSRC, f"-j{jobs}"]
    if not verbose:
        cmd.insert(1, "-s")
    subprocess.run(cmd, check=True)
    return os.path.join(HERE, "libpnol_amd.so")


if __name__ == "__main__":
    print(build(verbose=True))
